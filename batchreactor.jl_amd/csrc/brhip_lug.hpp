// brhip_lug.hpp -- the integrator's LU of A = I - gamma*J on a 4 x 16 lane grid (CPL = 1, NMAX 32 / 56 /
// 64). Included by brhip.hip after brhip_device.hpp; selected by BR_LU_GRID (brhip.hip).
//
// Same factorization as lu_factor (SUNDIALS denseGETRF: partial pivoting on the max |a_ik|, exact
// ties to the lowest ORIGINAL row; multipliers l = a_ik * (1 / a_kk); a_ij = fma(-a_kj, l, a_ij) in
// step order) and the same stored form (column-major factor matrix M with NMAX rows per column in
// pivot-step order: L below the diagonal, U' = D^-1 U above it, 0 on it and in rows >= n; D^-1 in step
// order after it), so lu_solve is unchanged and the results are bit-identical to lu_factor's.
//
// Why a grid. In lu_factor a lane holds one ROW; every pivot-row element has to reach all 64 lanes,
// and a v_readlane pair per element (+ the FMA) is 40 % of the GRI integrator's VALU instructions
// (profiles/r04_pmc_phase_valu_gri.json). Here lane (r, c) = 16 r + c holds the entries of the rows
// at positions s = c + 16 t (t = 0..3, "slots") in the columns j = 4 q + r (q = 0..7 per panel):
// * the pivot-row values a_kj a lane needs are in its own 16-lane DPP row (position k sits at lane
//   c = k % 16 of every row), so they are broadcast by the FMA itself (v_fmac_f64_dpp row_newbcast:
//   one VALU op per update, no readlane);
// * the multipliers of column k live in one DPP row (r = k % 4); its 16 lanes write their 4 values
//   to LDS once and every lane reads the 4 it needs (2 + 2 b128 LDS ops per step, no VALU);
// * the pivot search is a max over 4 slots and a 16-lane DPP row max.
// Position = pivot step (denseGETRF's physical row order). The rows are loaded in the previous
// factorization's pivot order (perm_io), so a step's pivot is almost always on its position already
// (1.2 % of GRI steps are not, 2.9 % for the surface case; scripts/lu_order_stats.py). Each step
// checks that with two ballots (the largest high word of |a_sk| is held by position k alone: then it
// is the pivot under any tie rule). When it is not, one shared handler per block finds the exact
// pivot (max |a|, ties to the lowest original row) and, if that is another position p, interchanges
// rows k and p in place: their register rows (staged through LDS: the DPP row of each column holds
// both), their stored multipliers of columns 0..k-1 and their entries in the load order; the step
// then resumes with its check skipped. (BR_LUG_RESTART=1: the A/B variant that instead restarts the
// panel with the two rows interchanged in the load order.)
//
// Steps run in blocks of 16 (the pivot positions of a block are slot 0 of a shifting frame: after a
// block, slot t <- t + 1 and register q <- q + 4), so one unrolled block body serves every block.
// Panel 1 = columns 0..31 (registers a[t][0..7]); for NMAX > 32 panel 2 = columns 32..NMAX-1 is loaded
// when block 2 starts, receives the updates of steps 0..31 left-looking (multipliers re-read from M,
// pivot-row values by the same DPP broadcast), and is then factored by blocks 2 and 3.
#pragma once

// 1: a pivot off its position restarts the panel with the two rows interchanged in the load order
// (A/B variant); 0 (default): the two rows are interchanged in place (staged through LDS) and the
// step resumes
#ifndef BR_LUG_RESTART
#define BR_LUG_RESTART 0
#endif

namespace brhip {

// diagnostic build (-DBR_LUG_STATS=1): device-wide event counts of the grid LU, read and reset by
// br_debug_lug_stats (brhip.hip): factorizations, steps run, pivot handler calls, ties, interchanges
#if BR_LUG_STATS
__device__ unsigned long long g_lug_stats[8];
__device__ unsigned long long g_lug_dump[256][8];   // first fast-check failures: I, k, b0, b1, rm, |a| bits...
#define BR_LUG_COUNT(i, v) do { if (__builtin_amdgcn_mbcnt_lo(~0u, 0) == 0 && (threadIdx.x & 63) == 0) atomicAdd(&g_lug_stats[i], (unsigned long long)(v)); } while (0)
#else
#define BR_LUG_COUNT(i, v) do { } while (0)
#endif

// r += -f * x[lane K of this lane's 16-lane row]  (DPP broadcast inside the FMA)
template <int K>
__device__ __forceinline__ void g_fnma(double& r, double x, double f) {
    asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(x), "v"(f), "i"(K));
}
// r += -f * r[lane K of this row]. No s_nop: in the update sequences below the instruction before
// it writes another register (slot t > 0 of the same column), and each step's sequence starts
// after an explicit s_nop 1 (VALU write -> DPP read hazard)
template <int K>
__device__ __forceinline__ void g_fnma_self(double& r, double f) {
    asm volatile("v_fmac_f64_dpp %0, %0, -%1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(f), "i"(K));
}
// max over this lane's 16-lane DPP row (every lane gets it)
__device__ __forceinline__ unsigned g_row_umax(unsigned x) {
    unsigned r;
    asm volatile(
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1"
        : "=&v"(r)
        : "v"(x));
    return r;
}
template <int B, int E, class F>
__device__ __forceinline__ void g_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        g_for<B + 1, E>(f);
    }
}
// opaque copies of register-array elements before a data-dependent select among them: without it
// InstCombine turns select(load a[i], load a[j]) into a load through a selected pointer, and SROA
// then cannot keep the array in registers (it is demoted to scratch memory)
__device__ __forceinline__ double g_opq(double v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ int g_opq(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// opaque uniform int: readfirstlane first, so a value the compiler later moves to a VGPR (loop phis
// mixing in per-lane values after inlining) reaches the SGPR constraint legally
__device__ __forceinline__ int g_uni(int v) {
    v = __builtin_amdgcn_readfirstlane(v);
    asm volatile("" : "+s"(v));
    return v;
}
// opaque uniform global pointer (as launder, through readfirstlane)
template <class T>
__device__ __forceinline__ BR_GLOBAL T* g_ptr(T* p) {
    unsigned long long u = (unsigned long long)p;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
    u = ((unsigned long long)hi << 32) | lo;
    asm volatile("" : "+s"(u));
    return (BR_GLOBAL T*)u;
}
// 32-bit lane pull (ds_bpermute: the LDS crossbar, no memory)
__device__ __forceinline__ int g_pull(int v, int src) { return __builtin_amdgcn_ds_bpermute(src * 4, v); }

template <int NMAX>
struct LugState {
    static constexpr int TS = NMAX > 32 ? 4 : 2;   // 16-position slots
    static constexpr int FR = NMAX;                 // factor column stride (rows)
    double a[TS][8];             // frame: slot t = positions kb + c + 16 t, register q = column kb + 4 q + r
    unsigned so8[TS];            // store offsets of the frame slots' positions (out of range: >= n)
    double dinv0;                // 1 / pivot of the frame slot-0 position (once pivoted)
    int pr[TS];                  // original row at ABSOLUTE position c + 16 t (the load order)
};

// fast pivot check of local step I (position k = kb + I = frame slot 0, lane I of each row; column k
// = register I / 4 of DPP row I % 4): the largest high word of |a_sk| over the candidates s >= k is
// held by position k alone
template <int NMAX, int I>
__device__ __forceinline__ bool lug_check(const LugState<NMAX>& S, int c) {
    constexpr int TS = LugState<NMAX>::TS;
    constexpr int rk = I & 3, qk = I >> 2;
    unsigned h[TS];
#pragma unroll
    for (int t = 0; t < TS; ++t) {
        const unsigned hv = (unsigned)(__double_as_longlong(S.a[t][qk]) >> 32) & 0x7fffffffu;
        h[t] = (t > 0 || c >= I) ? hv : 0u;   // slot 0: positions < k are pivoted
    }
    unsigned m = h[0];
#pragma unroll
    for (int t = 1; t < TS; ++t) m = max(m, h[t]);
    const unsigned rm = g_row_umax(m);
    const unsigned long long b0 = __ballot(h[0] == rm);
    bool e1 = false;
#pragma unroll
    for (int t = 1; t < TS; ++t) e1 = e1 || (h[t] == rm);
    const unsigned long long b1 = __ballot(e1);
    const bool ok = (((unsigned)(b0 >> (16 * rk)) & 0xffffu) == (1u << I)) && (((unsigned)(b1 >> (16 * rk)) & 0xffffu) == 0u);
#if BR_LUG_STATS
    if (!ok) {
        const unsigned h0p = __builtin_amdgcn_readlane(h[0], 16 * rk + I), mp = __builtin_amdgcn_readlane(m, 16 * rk + I);
        const unsigned rmp = __builtin_amdgcn_readlane(rm, 16 * rk + I);
        const double a0p = bcast(S.a[0][qk], 16 * rk + I), a1p = bcast(S.a[1][qk], 16 * rk + I);
        if ((threadIdx.x & 63) == 0) {
            const unsigned long long slot = atomicAdd(&g_lug_stats[6], 1ull);
            if (slot < 256) {
                g_lug_dump[slot][0] = I;
                g_lug_dump[slot][1] = b0;
                g_lug_dump[slot][2] = b1;
                g_lug_dump[slot][3] = rmp;
                g_lug_dump[slot][4] = (unsigned long long)__double_as_longlong(a0p);
                g_lug_dump[slot][5] = (unsigned long long)__double_as_longlong(a1p);
                g_lug_dump[slot][6] = h0p;
                g_lug_dump[slot][7] = mp;
            }
        }
    }
#endif
    return ok;
}

// exact pivot of local step dev (any column register qk < 4 of the frame): max |a| over the candidate
// positions, exact ties to the lowest original row. Returns the pivot's lane in DPP row rk (-1: none)
// and its frame slot; |pivot| bits in pb.
template <int NMAX>
__device__ __forceinline__ int lug_exact_pivot(const LugState<NMAX>& S, int blk, int dev, int qk, int rk, int c, int n,
                                               int& tp, unsigned long long& pb) {
    constexpr int TS = LugState<NMAX>::TS;
    unsigned long long kbest = 0;
    unsigned kr = 0;   // ~original row of the lane's best candidate (0: none)
    int kt = 0;
#pragma unroll
    for (int t = 0; t < TS; ++t) {
        double v = g_opq(S.a[t][0]);
#pragma unroll
        for (int q = 1; q < 4; ++q) v = (qk == q) ? g_opq(S.a[t][q]) : v;
        int row = g_opq(S.pr[0]);
#pragma unroll
        for (int s2 = 1; s2 < TS; ++s2) row = (blk + t == s2) ? g_opq(S.pr[s2]) : row;
        const int pos = c + 16 * (blk + t);
        const bool cand = (blk + t < TS) && pos < n && (t > 0 || c >= dev);
        const unsigned long long bits = (unsigned long long)__double_as_longlong(v) & 0x7fffffffffffffffull;
        const unsigned key = ~(unsigned)row;
        const bool better = cand && (kr == 0 || bits > kbest || (bits == kbest && key > kr));
        kbest = better ? bits : kbest;
        kr = better ? key : kr;
        kt = better ? t : kt;
    }
    const unsigned hi = (unsigned)(kbest >> 32), lo = (unsigned)kbest;
    const unsigned long long rmask = 0xffffull << (16 * rk);
    const unsigned mh = g_row_umax(kr ? hi : 0u);
    bool top = kr != 0 && hi == mh;
    unsigned long long m = __ballot(top) & rmask;
    if (__builtin_popcountll(m) > 1) {
        const unsigned ml = g_row_umax(top ? lo : 0u);
        top = top && lo == ml;
        m = __ballot(top) & rmask;
        if (__builtin_popcountll(m) > 1) {
            const unsigned mk = g_row_umax(top ? kr : 0u);
            top = top && kr == mk;
            m = __ballot(top) & rmask;
        }
    }
    if (m == 0) return -1;
    // (uniform by construction; readfirstlane says so to the compiler: with several inlined copies it
    // otherwise keeps the lane index in a VGPR and cannot select readlane)
    const int p = __builtin_amdgcn_readfirstlane((int)__builtin_ctzll(m));
    tp = __builtin_amdgcn_readlane(kt, p);
    pb = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)hi, p) << 32) | (unsigned)__builtin_amdgcn_readlane((int)lo, p);
    return p;
}

// the load order: positions (blk, lane dev) and (blk + tp, lane cp) exchange their original rows
template <int NMAX>
__device__ __forceinline__ void lug_swap_order(LugState<NMAX>& S, int blk, int dev, int tp, int cp, int c) {
    constexpr int TS = LugState<NMAX>::TS;
    int vk = g_opq(S.pr[0]), vp = vk;
#pragma unroll
    for (int s2 = 1; s2 < TS; ++s2) {
        const int x = g_opq(S.pr[s2]);
        vk = (blk == s2) ? x : vk;
        vp = (blk + tp == s2) ? x : vp;
    }
    const int rowk = g_pull(vk, dev), rowp = g_pull(vp, cp);   // (rows are the same in every DPP row)
#pragma unroll
    for (int s2 = 0; s2 < TS; ++s2) {
        S.pr[s2] = (s2 == blk && c == dev) ? rowp : S.pr[s2];
        S.pr[s2] = (s2 == blk + tp && c == cp) ? rowk : S.pr[s2];
    }
}

// elimination step I once its pivot is on position k: multipliers, column k of the factors, the
// multipliers through LDS to every DPP row, rank-1 update of the live registers
template <int NMAX, int I>
__device__ __forceinline__ void lug_elim(LugState<NMAX>& S, int k, int c, int r, int nq, int ns,
                                         __amdgpu_buffer_rsrc_t rs, LDSd* xch) {
    constexpr int TS = LugState<NMAX>::TS, FR = LugState<NMAX>::FR;
    constexpr int rk = I & 3, qk = I >> 2;
    auto& a = S.a;
    const double piv = bcast(a[0][qk], 16 * rk + I);
    const double rinv = 1.0 / piv;
    double l[TS];
    l[0] = (c > I) ? a[0][qk] * rinv : 0.0;
#pragma unroll
    for (int t = 1; t < TS; ++t) l[t] = a[t][qk] * rinv;   // (padding rows: 0; never stored)
    const double f0 = (c < I) ? a[0][qk] * S.dinv0 : l[0];  // U' above the diagonal, 0 on it
    S.dinv0 = (c == I) ? rinv : S.dinv0;
    if (r == rk) {
        // column k of the factors (this DPP row holds it) and its multipliers to LDS
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f0), rs, S.so8[0], k * (FR * 8), 0);
#pragma unroll
        for (int t = 1; t < TS; ++t)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, l[t]), rs, S.so8[t], k * (FR * 8), 0);
#pragma unroll
        for (int t = 0; t < TS; ++t) xch[TS * c + t] = l[t];
    }
    wave_sync();
    double lb[TS];
#pragma unroll
    for (int t = 0; t < TS; ++t) lb[t] = xch[TS * c + t];
    wave_sync();
    asm volatile("s_nop 1");
    // rank-1 update of the live registers: slots TS-1..1 first (they read the pivot-row values of
    // slot 0 by DPP), slot 0 last; columns beyond the panel's live ones: q >= 4 only when nq > 4
    g_for<1, TS>([&](auto T) {
        constexpr int t = TS - decltype(T)::value;
        if (t < ns) {
            g_for<qk, 4>([&](auto Q) { g_fnma<I>(a[t][decltype(Q)::value], a[0][decltype(Q)::value], lb[t]); });
            if (nq > 4) g_for<(qk > 4 ? qk : 4), 8>([&](auto Q) { g_fnma<I>(a[t][decltype(Q)::value], a[0][decltype(Q)::value], lb[t]); });
        }
    });
    g_for<qk, 4>([&](auto Q) { g_fnma_self<I>(a[0][decltype(Q)::value], lb[0]); });
    if (nq > 4) g_for<(qk > 4 ? qk : 4), 8>([&](auto Q) { g_fnma_self<I>(a[0][decltype(Q)::value], lb[0]); });
}

// one step, in-place interchange variant: on a failed fast check the exact pivot is found and, when it
// is another position p, rows k and p are exchanged in place (registers staged through LDS, their
// stored multipliers of columns 0..k-1, the load order). false: singular (fail = k + 1)
template <int NMAX, int I>
__device__ __forceinline__ bool lug_step_ip(LugState<NMAX>& S, int kb, int blk, int c, int r, int lane, int n, int nq, int ns,
                                            __amdgpu_buffer_rsrc_t rs, LDSd* xch, BR_GLOBAL double* wsg, int& fail) {
    constexpr int TS = LugState<NMAX>::TS, FR = LugState<NMAX>::FR;
    constexpr int rk = I & 3, qk = I >> 2;
    auto& a = S.a;
    // opaque per step: the lane tests against this step's constants are made here (hoisted out of
    // the panel loop they become ~60 live lane masks, and the SGPRs spill)
    c = launder_v(c);
    r = launder_v(r);
    nq = g_uni(nq);
    ns = g_uni(ns);
    const int k = g_uni(kb) + I;
    if (__builtin_expect(!lug_check<NMAX, I>(S, c), 0)) {
        BR_LUG_COUNT(2, 1);
        int tp = 0;
        unsigned long long pb = 0;
        const int p = lug_exact_pivot<NMAX>(S, g_uni(blk), I, qk, rk, c, n, tp, pb);
        if (p < 0 || pb == 0ull) {   // no candidate / every candidate 0: singular
            fail = k + 1;
            return false;
        }
        const int cp = p & 15;
        if (tp != 0 || cp != I) {
            BR_LUG_COUNT(4, 1);
            BR_LUG_COUNT(5, k);
            const int pos_p = cp + 16 * (blk + tp);
            __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's factor stores are done
            if (lane < k) {
                BR_GLOBAL double* col = wsg + (size_t)lane * FR;
                const double vk = col[k], vpp = col[pos_p];
                col[k] = vpp;
                col[pos_p] = vk;
            }
            LDSd* stk = xch + 64;
            LDSd* stp = xch + 96;
            if (c == I) {
#pragma unroll
                for (int q = 0; q < 8; ++q) stk[8 * r + q] = a[0][q];
            }
            if (c == cp) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    double x = g_opq(a[0][q]);
#pragma unroll
                    for (int t = 1; t < TS; ++t) x = (tp == t) ? g_opq(a[t][q]) : x;
                    stp[8 * r + q] = x;
                }
            }
            wave_sync();
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const double x = stp[8 * r + q];
                a[0][q] = (c == I) ? x : a[0][q];
            }
            // (selects, not branches on tp: stores to a[tp][q] under a branch become stores through a
            // selected pointer, and the register array is demoted to scratch memory)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const double y = stk[8 * r + q];
#pragma unroll
                for (int t = 0; t < TS; ++t) a[t][q] = (tp == t && c == cp) ? y : a[t][q];
            }
            wave_sync();
            lug_swap_order<NMAX>(S, blk, I, tp, cp, c);
        } else {
            BR_LUG_COUNT(3, 1);
        }
    }
    lug_elim<NMAX, I>(S, k, c, r, nq, ns, rs, xch);
    return true;
}

// one step, restart variant: false = the fast check failed (the caller's handler restarts the panel)
template <int NMAX, int I>
__device__ __forceinline__ bool lug_step_rs(LugState<NMAX>& S, int kb, int c, int r, int nq, int ns,
                                            unsigned long long forced, __amdgpu_buffer_rsrc_t rs, LDSd* xch) {
    c = launder_v(c);
    r = launder_v(r);
    nq = g_uni(nq);
    ns = g_uni(ns);
    const int k = g_uni(kb) + I;
    if (!((forced >> k) & 1ull) && !lug_check<NMAX, I>(S, c)) return false;
    lug_elim<NMAX, I>(S, k, c, r, nq, ns, rs, xch);
    return true;
}

template <int NMAX>
__device__ __forceinline__ int lu_factor_g(const double* __restrict__ J_, double* __restrict__ ws, LDSd* xch,
                                           double gamma, int n, int lane, int& perm_io) {
    static_assert(NMAX == 32 || NMAX == 56 || NMAX == 64, "lu_factor_g: NMAX");
    typedef LugState<NMAX> St;
    constexpr int TS = St::TS, FR = St::FR;
    constexpr int NQ2 = (NMAX - 32) / 4;      // panel-2 registers per slot (6 / 8; 0 for NMAX = 32)
    const BR_GLOBAL double* J = g_ptr(J_);
    BR_GLOBAL double* wsg = g_ptr(ws);
    lane = launder_v(lane);
    n = g_uni(n);
    const int r = lane >> 4, c = lane & 15;
    // the saved J through a buffer of n columns (64 rows each): a column >= n, and a row that is
    // not a real one, is out of range and reads 0 (the offsets are in the VGPR: range-checked)
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc((void*)J, (short)0, n * (WAVE * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = lu_rsrc(wsg, NMAX * FR);            // factor columns M
    const __amdgpu_buffer_rsrc_t rd = lu_rsrc(wsg + NMAX * FR, WAVE);     // D^-1
    St S;
    auto& a = S.a;
#pragma unroll
    for (int t = 0; t < TS; ++t) S.pr[t] = g_pull(perm_io, c + 16 * t);
    // panel load: a[t][q] = (I - gamma J)[pr[t]][colbase + 4 q + r]; registers beyond the panel: 0
    auto load_panel = [&](auto CB, auto NQ) {
        constexpr int colbase = decltype(CB)::value, nqp = decltype(NQ)::value;
        const int rr = launder_v(r);
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int row = launder_v(S.pr[t]);
            const unsigned vb = (row < n) ? (unsigned)row * 8u + (unsigned)(colbase + rr) * (WAVE * 8) : LU_OOB;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (q < nqp) {
                    const double jv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, vb + 4u * q * (WAVE * 8), 0, 0));
                    a[t][q] = ((colbase + 4 * q + rr == row) ? 1.0 : 0.0) - gamma * jv;
                } else {
                    a[t][q] = 0.0;
                }
            }
        }
    };
    // panel 2 (after its load): the updates of steps 0..31, left-looking (multipliers re-read from M,
    // pivot-row values by the DPP broadcast), in two 16-step sub-blocks with a shifting frame; the
    // sub-block's rows are then final in panel 2 (U' = row * D^-1 stored)
    auto left_look = [&]() {
#pragma unroll 1
        for (int sb = 0; sb < 2; ++sb) {
            unsigned lo8[TS];
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                const int pos = c + 16 * (sb + t);
                lo8[t] = (sb + t < TS && pos < FR) ? (unsigned)pos * 8u : LU_OOB;
            }
            const int nsl = TS - sb;                                          // frame slots that exist
            double lc[2][TS];
            auto ldl = [&](double (&v)[TS], int k) {
#pragma unroll
                for (int t = 0; t < TS; ++t)
                    v[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lo8[t], k * (FR * 8), 0));
            };
            ldl(lc[0], 16 * sb);
            g_for<0, 16>([&](auto Ic) {
                constexpr int i = decltype(Ic)::value;
                if (i + 1 < 16) ldl(lc[(i + 1) & 1], 16 * sb + i + 1);
                double l[TS];
#pragma unroll
                for (int t = 0; t < TS; ++t) l[t] = lc[i & 1][t];
                l[0] = (launder_v(c) > i) ? l[0] : 0.0;                       // positions <= k: not updated
                asm volatile("s_nop 1");
                // every panel-2 register (columns >= n hold zeros: their updates are no-ops)
                const int nsl_ = g_uni(nsl);
                g_for<1, TS>([&](auto T) {
                    constexpr int t = TS - decltype(T)::value;
                    if (t < nsl_)
                        g_for<0, NQ2>([&](auto Q) { g_fnma<i>(a[t][decltype(Q)::value], a[0][decltype(Q)::value], l[t]); });
                });
                g_for<0, NQ2>([&](auto Q) { g_fnma_self<i>(a[0][decltype(Q)::value], l[0]); });
            });
            const double dl = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rd, (unsigned)(16 * sb + c) * 8u, 0, 0));
            const unsigned uo = (lo8[0] != LU_OOB) ? lo8[0] + (unsigned)r * (FR * 8) : LU_OOB;
#pragma unroll
            for (int q = 0; q < NQ2; ++q)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a[0][q] * dl), rs, uo, (32 + 4 * q) * (FR * 8), 0);
#pragma unroll
            for (int t = 0; t + 1 < TS; ++t)
#pragma unroll
                for (int q = 0; q < 8; ++q) a[t][q] = a[t + 1][q];
#pragma unroll
            for (int q = 0; q < 8; ++q) a[TS - 1][q] = 0.0;
        }
    };
    // block setup: store offsets of the frame's positions
    auto block_setup = [&](int blk) {
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int pos = c + 16 * (blk + t);
            S.so8[t] = (blk + t < TS && pos < n) ? (unsigned)pos * 8u : LU_OOB;
        }
    };
    // block end: U' of the block's rows in the panel's remaining columns, their D^-1; shift the frame
    auto block_end_store = [&](int kb, int nq) {
        const unsigned uo = (S.so8[0] != LU_OOB) ? S.so8[0] + (unsigned)r * (FR * 8) : LU_OOB;
        if (nq > 4) {
#pragma unroll
            for (int q = 4; q < 8; ++q)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a[0][q] * S.dinv0), rs, uo, (kb + 4 * q) * (FR * 8), 0);
        }
        if (r == 0) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, S.dinv0), rd, (unsigned)(kb + c) * 8u, 0, 0);
#pragma unroll
        for (int t = 0; t + 1 < TS; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) a[t][q] = a[t + 1][q + 4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[TS - 1][q] = 0.0;
        S.dinv0 = 0.0;
    };
    int fail = 0;
    BR_LUG_COUNT(0, 1);
    const int nblk = (n + 15) >> 4;
    const int np = (nblk > 2) ? 2 : 1;         // panels
    int pnl = 0, blk = 0;
#if BR_LUG_RESTART
    unsigned long long forced = 0;             // steps whose pivot is known to be on its position
    int dev = 0;
#pragma unroll 1
    for (;;) {                                 // panels, and restarts of a panel after an interchange
        if (pnl == 0) {
            load_panel(std::integral_constant<int, 0>{}, std::integral_constant<int, 8>{});
        } else if constexpr (NMAX > 32) {
            load_panel(std::integral_constant<int, 32>{}, std::integral_constant<int, NQ2>{});
            left_look();
        }
        S.dinv0 = 0.0;
        const int bend = (pnl == 0) ? (nblk < 2 ? nblk : 2) : nblk;
#pragma unroll 1
        for (blk = 2 * pnl; blk < bend; ++blk) {
            const int kb = 16 * blk;
            const int pend = (pnl == 0) ? (n < 32 ? n : 32) : n;               // end of this panel's columns
            const int nq = (pend - kb + 3) >> 2;                               // live registers (<= 8)
            const int ns = nblk - blk;                                         // live slots
            block_setup(blk);
#define BR_LUG_STEP(I)                                                                   \
    if (g_uni(kb) + I >= n) goto block_end;                                          \
    BR_LUG_COUNT(1, 1);                                                                  \
    if (!lug_step_rs<NMAX, I>(S, kb, c, r, nq, ns, forced, rs, xch)) { dev = I; goto pivot; }
            BR_LUG_STEP(0) BR_LUG_STEP(1) BR_LUG_STEP(2) BR_LUG_STEP(3)
            BR_LUG_STEP(4) BR_LUG_STEP(5) BR_LUG_STEP(6) BR_LUG_STEP(7)
            BR_LUG_STEP(8) BR_LUG_STEP(9) BR_LUG_STEP(10) BR_LUG_STEP(11)
            BR_LUG_STEP(12) BR_LUG_STEP(13) BR_LUG_STEP(14) BR_LUG_STEP(15)
#undef BR_LUG_STEP
        block_end:
            block_end_store(kb, nq);
        }
        if (++pnl >= np) break;
        continue;
    pivot:
        // ---- step k = 16 blk + dev failed the fast check: exact pivot; a tie on position k marks the
        // step, another position swaps places with k in the load order; the panel restarts
        {
            BR_LUG_COUNT(2, 1);
            const int k = 16 * blk + dev;
            int tp = 0;
            unsigned long long pb = 0;
            const int p = lug_exact_pivot<NMAX>(S, blk, dev, dev >> 2, dev & 3, c, n, tp, pb);
            if (p < 0 || pb == 0ull) {   // singular
                fail = k + 1;
                break;
            }
            const int cp = p & 15;
            if (tp == 0 && cp == dev) {
                BR_LUG_COUNT(3, 1);
                forced |= 1ull << k;
            } else {
                BR_LUG_COUNT(4, 1);
                BR_LUG_COUNT(5, k);
                lug_swap_order<NMAX>(S, blk, dev, tp, cp, c);
                if (pnl > 0) {   // multipliers of panel 1 (not redone) move with the rows
                    const int pos_p = cp + 16 * (blk + tp);
                    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's factor stores are done
                    if (lane < 32) {
                        BR_GLOBAL double* col = wsg + (size_t)lane * FR;
                        const double vk = col[k], vpp = col[pos_p];
                        col[k] = vpp;
                        col[pos_p] = vk;
                    }
                }
            }
        }
    }
#else
#pragma unroll 1
    for (;;) {                                 // panels
        if (pnl == 0) {
            load_panel(std::integral_constant<int, 0>{}, std::integral_constant<int, 8>{});
        } else if constexpr (NMAX > 32) {
            load_panel(std::integral_constant<int, 32>{}, std::integral_constant<int, NQ2>{});
            left_look();
        }
        S.dinv0 = 0.0;
        const int bend = (pnl == 0) ? (nblk < 2 ? nblk : 2) : nblk;
#pragma unroll 1
        for (blk = 2 * pnl; blk < bend; ++blk) {
            const int kb = 16 * blk;
            const int pend = (pnl == 0) ? (n < 32 ? n : 32) : n;               // end of this panel's columns
            const int nq = (pend - kb + 3) >> 2;                               // live registers (<= 8)
            const int ns = nblk - blk;                                         // live slots
            block_setup(blk);
#define BR_LUG_STEP(I)                                                                   \
    if (g_uni(kb) + I >= n) goto block_end;                                          \
    BR_LUG_COUNT(1, 1);                                                                  \
    if (!lug_step_ip<NMAX, I>(S, kb, blk, c, r, lane, n, nq, ns, rs, xch, wsg, fail)) goto lu_done;
            BR_LUG_STEP(0) BR_LUG_STEP(1) BR_LUG_STEP(2) BR_LUG_STEP(3)
            BR_LUG_STEP(4) BR_LUG_STEP(5) BR_LUG_STEP(6) BR_LUG_STEP(7)
            BR_LUG_STEP(8) BR_LUG_STEP(9) BR_LUG_STEP(10) BR_LUG_STEP(11)
            BR_LUG_STEP(12) BR_LUG_STEP(13) BR_LUG_STEP(14) BR_LUG_STEP(15)
#undef BR_LUG_STEP
        block_end:
            block_end_store(kb, nq);
        }
        if (++pnl >= np) break;
    }
lu_done:
#endif
    // padding: rows n..FR-1 of every column and columns n..NMAX-1 of M, D^-1 beyond the last block
    if (lane < FR) {
        const bool prow = lane >= n;
        for (int cc = 0; cc < NMAX; ++cc)
            if (prow || cc >= n) wsg[(size_t)cc * FR + lane] = 0.0;
    }
    if (lane >= 16 * nblk) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, 0.0), rd, (unsigned)lane * 8u, 0, 0);
    // step -> original row, in the row-per-lane form of perm_io (lane s: position s)
    {
        int v = lane;
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int x = g_pull(S.pr[t], c);
            v = (r == t) ? x : v;
        }
        perm_io = v;
    }
    return fail;
}

}  // namespace brhip
