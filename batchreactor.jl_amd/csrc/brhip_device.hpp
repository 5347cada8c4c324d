// brhip_device.hpp -- device side of libbrhip.so (gfx950, fp64).
//
// Execution model: ONE REACTOR PER WAVEFRONT (64 lanes), several reactors (waves) per
// workgroup; lane k <-> solution component k (gas species 0..ng-1, then surface coverages).
//
// LDS layout (few base addresses, so the hot loop keeps few SGPRs live):
//  * table image, staged once per workgroup from global memory (host-built, `img`):
//      [0,512) molwt[64] | [512,1024) sigma[64] | RX records (32 B / gas reaction) |
//      SX records (48 B / surface reaction) | SXE (4 doubles / surface reaction: coverage eps) |
//      TBE third-body entries (16 B: species, eff-1)
//  * per reactor block: [Ctl][V: Nordsieck + work vectors][SP: conc | accw | accs (64 each)]
//      [FOD: {k0/k_inf, log10 Fcent, c, n} per falloff reaction][SKD: {k, k*exp(cov)} per surface reaction]
//  * RXD: {kf, kr} per gas reaction, in the wave's global workspace slot (5.2 KB for GRI: kept
//    out of LDS so 12 reactors fit a CU instead of 8), prefetched at the start of each RHS
//  * T-dependent rate constants (RXD/FOD/SKD) are computed once per reactor: T is a per-reactor
//    constant (ConstantParams, src/BatchReactor.jl:14-17).
// Reactions are evaluated lane-parallel (reaction r on lane r mod 64); production rates are
// accumulated with fp64 LDS atomics (ds_add_f64, no return); reductions are DPP + readlane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace brhip {

constexpr double R_GAS = 8.31446261815324;   // RxnHelperUtils.R (src/BatchReactor.jl:338)
constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------
// mechanism description (host-built)
// ------------------------------------------------------------------------------------
struct DevMech {
    int ng, ns, n, nrg, nrs, ntb, nfo, ntbe, nset, conv;
    int nu4;                      // some gas reaction has 4 reactants or 4 products
    int cpl;                      // components per lane: 1 (n <= 64) or 2 (64 < n <= 128), see Lay
    double p_std, G;              // Pa ; site density mol/m2
    const uint4* img;             // LDS table image (global copy)
    int img_bytes;                // multiple of 16
    int sx_off, sxe_off, tbe_off; // byte offsets in the image
    int tbs_off;                  // third-body efficiency sets: one word (start | count << 20) each
    int fod_off, skd_off;         // byte offsets of FOD / SKD from the end of the species block
    int rblock_bytes;             // per-reactor LDS bytes from SP start (SP + FOD + SKD)
    // init only (T-dependent constants)
    const double* nasa;           // [ng][15]: Tmid, a_hi[7], a_lo[7]
    const double* g_par;          // [nrg][4]: A (SI), beta, Ea/R, Kc scale
    const int* g_dnu;             // [nrg]
    const double* fo_par;         // [nfo][8]: A0, b0, E0/R, a, T***, T*, T**, ntroe
    const double* s_par;          // [nrs][4]: A or s0, beta, Ea [J/mol], M_gas (stick)
    // Jacobian only
    const double* tb_eff;         // [nset][n] dense efficiencies
    const int* col_ptr;           // [n+1] Jacobian column lists
    const int* col_rx;            // combined reaction index (gas r, surface nrg+r)
    // gas-only fast Jacobian (jfast): mass-action column lists in the LDS image (cmp_off: int
    // [n+1] column starts, cmr_off: uint16 reaction per entry; reactant / product dependence
    // only), third-body dependence through the efficiency sets (ntb third-body reactions first)
    int jfast, ntbr, cmp_off, cmr_off;
    // per gas species j, the efficiency sets with eff_j != 1: tjp_off int [n+1] starts, tje_off
    // 16-byte entries {int set, pad, double eff - 1}
    int tjp_off, tje_off;
};

// The kernels' first argument is the DevMech (kernarg offset 0). The hot-path functions re-read
// its fields at the point of use through a laundered kernarg pointer (scalar loads from the
// kernarg segment), instead of keeping ~40 SGPRs of mechanism fields live across the whole
// integrator loop (which forced SGPR spills and serialised the LU / solve broadcasts).
extern __shared__ __attribute__((aligned(16))) char br_lds[];
template <class T>
__device__ __forceinline__ T karg_field(size_t off) {
    const char* p = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    typedef const __attribute__((address_space(4))) T cT;
    return *(cT*)(p + off);
}
#define MF(f) (::brhip::karg_field<decltype(::brhip::DevMech::f)>(offsetof(::brhip::DevMech, f)))
// RX records in the image: split into words 0..3 of every reaction, then words 4..7 (two arrays
// with a 16-byte stride: the b128 record reads of 64 consecutive reactions hit every LDS bank
// once; with the 32-byte stride of whole records two lanes share each bank)
template <class P>
struct RxRec {
    P a, b;
    __device__ __forceinline__ uint32_t operator[](int w) const { return w < 4 ? a[w] : b[w - 4]; }
};
template <class P>
__device__ __forceinline__ RxRec<P> rx_rec(P rx, int r) {
    return {rx + 4 * r, rx + 4 * MF(nrg) + 4 * r};
}

// RX record: w0 reactant species (4 x 8 bit; pad = SP_ONE, a slot holding 1.0, so the
// concentration products need no branches), w1 product species, w2 info (third-body
// efficiency set in bits 22..31), w3 pad, w4..w7 net-stoichiometry scatter list (byte offsets x6
// in w4..w6, nu nibbles | count << 24 in w7; see scatter())
__host__ __device__ inline int gi_nf(uint32_t v) { return v & 7; }
__host__ __device__ inline int gi_nr(uint32_t v) { return (v >> 3) & 7; }
__host__ __device__ inline int gi_rev(uint32_t v) { return (v >> 6) & 1; }
__host__ __device__ inline int gi_tb(uint32_t v) { return (v >> 7) & 3; }
__host__ __device__ inline int gi_troe(uint32_t v) { return (v >> 9) & 7; }
__host__ __device__ inline int gi_foidx(uint32_t v) { return (v >> 12) & 1023; }
__host__ __device__ inline int gi_tbidx(uint32_t v) { return (v >> 22) & 1023; }
// SX record: w0,w1 reactants (6 x 8 bit), w2,w3 products, w4 info, w5 coverage species (4 x 8),
// w6..w9 scatter list (as RX w4..w7), w10..w11 pad
__host__ __device__ inline int si_nf(uint32_t v) { return v & 7; }
__host__ __device__ inline int si_np(uint32_t v) { return (v >> 3) & 7; }
__host__ __device__ inline int si_stick(uint32_t v) { return (v >> 6) & 1; }
__host__ __device__ inline int si_ncov(uint32_t v) { return (v >> 7) & 7; }
__host__ __device__ inline int si_gas(uint32_t v) { return (v >> 10) & 255; }
__host__ __device__ inline int sp8(uint32_t w, int e) { return (w >> (8 * e)) & 255; }
constexpr int RX_WORDS = 8, SX_WORDS = 12, SXE_DOUBLES = 8;

// Components per lane: CPL = 1 for n <= 64 (lane k <-> component k); CPL = 2 for 64 < n <= 128
// (lane k <-> components k and k + 64, e.g. GRI gas + Ni surface, n = 66). Species-indexed LDS
// arrays are sized SPW = 64 (CPL = 1) or 80 (CPL = 2, n <= 72): see Lay.
template <int CPL>
struct Lay {
    // species slots: 64, or 80 for two components per lane (n <= 72; round 3: 128 before, the LDS
    // saved per reactor lets 12 gas+surface reactors share a CU instead of 11)
    static constexpr int SPW = CPL == 2 ? 80 : 64;
    // species block (doubles): conc[SPW], conc[ONE] = 1.0 (pad species of the packed records),
    // accw[SPW], accs[SPW], mc[64] third-body concentration per efficiency set
    static constexpr int CONC = 0, ONE = SPW, ACCW = SPW + 16, ACCS = 2 * SPW + 16, MC = 3 * SPW + 16;
    static constexpr int DOUBLES = 3 * SPW + 16 + 64, BYTES = DOUBLES * 8;
    static constexpr int IMG_RX = 16 * SPW;   // image: molwt[SPW] | sigma[SPW] | RX records ...
};

struct Tab {   // views of the staged table image
    const double* molwt;   // [SPW]
    const double* sigma;   // [SPW]
    const uint32_t* rx;    // RX_WORDS per gas reaction
    const uint32_t* sx;    // SX_WORDS per surface reaction
    const double* sxe;     // SXE_DOUBLES per surface reaction: coverage eps[4], site factor, pad
    const char* tbe;       // 16 B per third-body entry
    const uint32_t* tbs;   // per efficiency set: start | count << 20 into tbe
};
template <int CPL>
__device__ __forceinline__ Tab tab_view(const char* base, const DevMech& M) {
    Tab t;
    base = br_lds;
    t.molwt = reinterpret_cast<const double*>(base);
    t.sigma = t.molwt + Lay<CPL>::SPW;
    t.rx = reinterpret_cast<const uint32_t*>(base + Lay<CPL>::IMG_RX);
    t.sx = reinterpret_cast<const uint32_t*>(base + MF(sx_off));
    t.sxe = reinterpret_cast<const double*>(base + MF(sxe_off));
    t.tbe = base + MF(tbe_off);
    t.tbs = reinterpret_cast<const uint32_t*>(base + MF(tbs_off));
    return t;
}

// ------------------------------------------------------------------------------------
// sub-phase shader clocks (diagnostic build, BR_PHASE_CLOCKS): BR_SUB_T(t) starts a timer,
// BR_SUB_ADD(slot, t) adds its cycles to g_sub[slot] (one atomic from lane 0); read and reset
// from the host with br_diag_sub (brhip.hip). Slots: 0 LU panel 1, 1 LU panel 2, 2 LU gather,
// 3 ctl_post_rhs, 4..6 gas-only Jacobian: entry loop, column writes, multipliers (+ set passes);
// 7 begin_step; 8..10 ctl_post_solve: convergence + error test, complete + prepare next step,
// ignition / unstable / tstop checks; 11 RHS setup (conc, third-body sums), 12 RHS production.
// ------------------------------------------------------------------------------------
#if BR_PHASE_CLOCKS
// one row of 16 sums per resident wave (plain adds by the wave's lane 0: one device-wide atomic
// counter hit by every wave at every step saturated the memory-side atomic unit and slowed the
// whole kernel 2x)
constexpr int SUB_MAXW = 16384;
__device__ unsigned long long g_sub[SUB_MAXW][16];
__device__ __forceinline__ void sub_add(int slot, unsigned long long dt) {
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && w < SUB_MAXW) g_sub[w][slot] += dt;
}
#define BR_SUB_T(t) const unsigned long long t = clock64()
#define BR_SUB_ADD(slot, t) ::brhip::sub_add(slot, clock64() - (t))
#else
#define BR_SUB_T(t)
#define BR_SUB_ADD(slot, t)
#endif

// ------------------------------------------------------------------------------------
// wave primitives (DPP row reductions + readlane; no LDS)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double bcast(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// broadcast of a pivot-row element in the LU (a v_readlane pair; the LDS-crossbar form measured
// 78.2k vs 90.8k GRI reactors/s in round 2: its latency sits on the elimination chain)
__device__ __forceinline__ double bcast_lu(double v, int p) { return bcast(v, p); }
// uniform fp64 values: v_readfirstlane into SGPRs (scalar residency and scalar branches; fp64
// arithmetic and compares still run on the VALU)
__device__ __forceinline__ double uni(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// quad_perm[1,0,3,2]=0xB1, quad_perm[2,3,0,1]=0x4E, row_half_mirror=0x141, row_mirror=0x140:
// each step pairs lane i with a partner that pairs back with i, so both compute the same value.
// Across the four row results: row_bcast:15 adds row 0 into row 1 and row 2 into row 3,
// row_bcast:31 then row 1's total into row 3, and lane 63 is read: (r3 + r2) + (r1 + r0), equal
// to (r0 + r1) + (r2 + r3) since each add is commutative (bit-identical to four readlanes).
template <int CTRL, int RM>
__device__ __forceinline__ double dppd_rows(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, RM, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, RM, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_sum(double v) {
    v += dppd<0xB1>(v);
    v += dppd<0x4E>(v);
    v += dppd<0x141>(v);
    v += dppd<0x140>(v);
    v = v + dppd_rows<0x142, 0xA>(v);   // (rows 0, 2 add 0: unused)
    v = v + dppd_rows<0x143, 0xC>(v);
    return bcast(v, 63);
}
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dppd<0xB1>(v));
    v = fmax(v, dppd<0x4E>(v));
    v = fmax(v, dppd<0x141>(v));
    v = fmax(v, dppd<0x140>(v));
    v = fmax(v, dppd_rows<0x142, 0xA>(v));
    v = fmax(v, dppd_rows<0x143, 0xC>(v));
    return bcast(v, 63);
}

// sum / max over each 16-lane DPP row (the quad engine's reactor groups): the butterfly steps of
// wave_sum / wave_max without the cross-row ones; every lane of a row gets its row's value
__device__ __forceinline__ double row_sum(double v) {
    v += dppd<0xB1>(v);
    v += dppd<0x4E>(v);
    v += dppd<0x141>(v);
    v += dppd<0x140>(v);
    return v;
}
__device__ __forceinline__ double row_max(double v) {
    v = fmax(v, dppd<0xB1>(v));
    v = fmax(v, dppd<0x4E>(v));
    v = fmax(v, dppd<0x141>(v));
    v = fmax(v, dppd<0x140>(v));
    return v;
}
// the two 16-lane rows of each 32-lane half: v_permlane16_swap (gfx950) of a value with itself gives
// every lane its half's even-row value (.even) and odd-row value (.odd)
struct RowPair {
    double even, odd;
};
__device__ __forceinline__ RowPair row_pair(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)(b & 0xffffffffLL), (int)(b & 0xffffffffLL), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    RowPair r;
    r.even = __longlong_as_double(((long long)hi[0] << 32) | (unsigned int)lo[0]);
    r.odd = __longlong_as_double(((long long)hi[1] << 32) | (unsigned int)lo[1]);
    return r;
}
// sum / max over each 32-lane half (the pair engine's reactor groups): the row butterflies, then the
// two row results combined in the same order on every lane (even + odd)
__device__ __forceinline__ double half_sum(double v) {
    const RowPair p = row_pair(row_sum(v));
    return p.even + p.odd;
}
__device__ __forceinline__ double half_max(double v) {
    const RowPair p = row_pair(row_max(v));
    return fmax(p.even, p.odd);
}

// opaque copy of a uniform pointer: addresses derived from it cannot be hoisted out of the
// integrator's main loop (otherwise LICM keeps ~NMAX 64-bit column addresses live across the
// whole loop and the kernel spills)
// (the result is an explicit global-address-space pointer: global_load/store, not flat_*)
#define BR_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ BR_GLOBAL T* launder(T* p) {
    asm volatile("" : "+s"(p));
    return (BR_GLOBAL T*)p;
}
// opaque copy of a per-lane value (stops LICM from hoisting lane-dependent constants such as
// the identity-matrix entries of I - gamma*J out of the main loop)
__device__ __forceinline__ int launder_v(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// opaque copy of a uniform int (SGPR): comparisons against it are made where they are used
// instead of being hoisted out of the integrator loop as lane masks (which then spill)
__device__ __forceinline__ int launder_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}

// ------------------------------------------------------------------------------------
// per-reactor rate workspace (LDS)
// ------------------------------------------------------------------------------------
struct RView {
    double* sp;    // species block: conc[k] = sp[CONC+k], accw, accs, mc (see Lay)
    BR_GLOBAL double* rxd;   // kf = rxd[2r], kr = rxd[2r+1] (global workspace slot)
    double* fod;   // k0/k_inf, log10 Fcent, c, n per falloff reaction
    double* skd;   // k(T), k*exp(-sum eps theta/RT) (Jacobian) per surface reaction
};
__host__ __device__ inline int fod_off_bytes(int /*nrg*/) { return 0; }   // RXD is in global memory
__host__ __device__ inline int skd_off_bytes(int nrg, int nfo) { return fod_off_bytes(nrg) + 32 * nfo; }
__host__ __device__ inline int rblock_bytes(int nrg, int nfo, int nrs, int cpl) {
    return (cpl == 2 ? Lay<2>::BYTES : Lay<1>::BYTES) + skd_off_bytes(nrg, nfo) + 16 * nrs;
}
template <int CPL>
__device__ __forceinline__ RView rview(char* spbase, const DevMech& /*M*/, BR_GLOBAL double* rxd) {
    RView r;
    r.sp = reinterpret_cast<double*>(spbase);
    r.rxd = rxd;
    r.fod = reinterpret_cast<double*>(spbase + Lay<CPL>::BYTES + MF(fod_off));
    r.skd = reinterpret_cast<double*>(spbase + Lay<CPL>::BYTES + MF(skd_off));
    return r;
}

// fp64 LDS accumulate, relaxed, wavefront scope (ds_add_f64, no return)
__device__ __forceinline__ void lds_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// Net-stoichiometry scatter list of a reaction (4 packed words): w0..w2 hold the byte offsets
// (species * 8) of slots 0..5, two 16-bit fields per word, w3 the 4-bit signed nu of each slot |
// count << 24. Byte offsets: a slot's address is one add of the field to the array base (a
// select-word add) instead of a byte extract and a shift-add (round 3: the production loop's
// scatter is ~1/3 of the RHS's VALU).
__device__ __forceinline__ unsigned sl_off(uint32_t w, int hi) { return hi ? (w >> 16) : (w & 0xffffu); }
__device__ __forceinline__ int sl_nu(uint32_t w3, int e) { return ((int)(w3 << (28 - 4 * e))) >> 28; }
// acc[k] += nu_k * v over the list
__device__ __forceinline__ void scatter(double* acc, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, double v) {
    // the count extracted once (opaque copy): otherwise each slot test became a v_mov of the slot
    // number plus a byte-select compare
    const int cnt = launder_v((int)(w3 >> 24));
    const uint32_t ws[3] = {w0, w1, w2};
    char* const base = reinterpret_cast<char*>(acc);
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        if (e < cnt) {
            double* p = reinterpret_cast<double*>(base + sl_off(ws[e >> 1], e & 1));
            lds_add(p, (double)sl_nu(w3, e) * v);                // exact for small integer nu
        }
    }
}

// scatter() except for species `self`: its nu * v is returned instead of added (the caller sums
// it in a register and reduces over the wave: in a Jacobian column pass nearly every entry of
// column j touches species j, which made acc[j] the hot address of every atomic slot)
__device__ __forceinline__ double scatter_noself(double* acc, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, double v,
                                                 int self) {
    const int cnt = launder_v((int)(w3 >> 24));
    const uint32_t ws[3] = {w0, w1, w2};
    const unsigned self8 = (unsigned)self * 8u;
    char* const base = reinterpret_cast<char*>(acc);
    double sv = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        if (e < cnt) {
            const unsigned off = sl_off(ws[e >> 1], e & 1);
            const double t = (double)sl_nu(w3, e) * v;
            if (off == self8) sv += t;
            else lds_add(reinterpret_cast<double*>(base + off), t);
        }
    }
    return sv;
}

// stage the table image (all threads of the workgroup), then barrier
__device__ __forceinline__ void stage_tables(const DevMech& M, char* dst) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const int nv = MF(img_bytes) / 16;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) d[i] = MF(img)[i];
    __syncthreads();
}

// T-only constants (src/BatchReactor.jl:14-17: T is a per-reactor constant); g/RT scratch in accw
template <int CPL>
__device__ __forceinline__ void init_tconst(const DevMech& M, const Tab& tb, const RView& R, double T, int lane) {
    const double lT = log(T);
    double* grt = R.sp + Lay<CPL>::ACCW;
    if (lane == 0) R.sp[Lay<CPL>::ONE] = 1.0;
#pragma unroll 1
    for (int k = lane; k < MF(ng); k += WAVE) {
        const double* c = MF(nasa) + 15 * k;
        const double* a = (T < c[0]) ? c + 8 : c + 1;
        const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        const double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        grt[k] = h - s;
    }
    wave_sync();
    const double RT = R_GAS * T;
#pragma unroll 1
    for (int r = lane; r < MF(nrg); r += WAVE) {
        const auto rec = rx_rec(tb.rx, r);
        const uint32_t info = rec[2];
        const double* gp = MF(g_par) + 4 * r;
        const double kf = gp[0] * exp(gp[1] * lT - gp[2] / T);
        double kr = 0.0;
        if (gi_rev(info)) {
            double dg = 0.0;
            const int nf = gi_nf(info), nr = gi_nr(info);
            for (int e = 0; e < 4; ++e) if (e < nr) dg += grt[sp8(rec[1], e)];
            for (int e = 0; e < 4; ++e) if (e < nf) dg -= grt[sp8(rec[0], e)];
            double Kc = exp(-dg) * pow(MF(p_std) / RT, (double)MF(g_dnu)[r]);
            Kc *= gp[3];
            kr = kf / Kc;
        }
        R.rxd[2 * r] = kf;
        R.rxd[2 * r + 1] = kr;
        if (gi_tb(info) == 2) {
            const int fi = gi_foidx(info);
            const double* fp = MF(fo_par) + 8 * fi;
            double* fo = R.fod + 4 * fi;
            fo[0] = fp[0] * exp(fp[1] * lT - fp[2] / T) / kf;   // k0 / k_inf
            double fcv = 1.0;
            if (gi_troe(info)) {
                fcv = (1 - fp[3]) * exp(-T / fp[4]) + fp[3] * exp(-T / fp[5]);
                if (gi_troe(info) == 4) fcv += exp(-fp[6] / T);
            }
            const double lfc = log10(fcv);
            fo[1] = lfc;
            fo[2] = ((MF(conv) & BR_CONV_TROE_C4) ? -4.0 : -0.4) - 0.67 * lfc;
            fo[3] = 0.75 - 1.27 * lfc;
        }
    }
#pragma unroll 1
    for (int r = lane; r < MF(nrs); r += WAVE) {
        const uint32_t info = tb.sx[SX_WORDS * r + 4];
        const double* sp = MF(s_par) + 4 * r;
        double k;
        if (si_stick(info)) k = sp[0] * sqrt(RT / (2 * M_PI * sp[3]));
        else k = sp[0] * pow(T, sp[1]) * exp(-sp[2] / RT);
        R.skd[2 * r] = k;
    }
    // the RXD stores reach L2 and this CU's L1 is invalidated before any lane reads the slot
    // (it held the previous reactor's constants)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wave_sync();
}

// falloff: fac = Pr/(1+Pr)*F and d fac / d[M] (CHEMKIN Lindemann / Troe); fo[0] = k0/k_inf
// (T-only, so Pr = fo[0] [M] needs no division). Troe: log10 F = log10 Fcent / (1 + f1^2) with
// f1 = x / den, evaluated as log10 Fcent den^2 / (den^2 + x^2) (one division), F = exp10(...)
// instead of the generic pow(10, .) (same value to an ulp, about half the instructions).
__device__ __forceinline__ double troe_F(double Pr, const double* fo, double& x_out, double& den_out) {
    const double Prs = Pr > 1e-300 ? Pr : 1e-300;
    const double x = log10(Prs) + fo[2];
    const double den = fo[3] - 0.14 * x;
    const double d2 = den * den;
    x_out = x; den_out = den;
    return exp10(fo[1] * d2 / (d2 + x * x));
}
template <bool WANT_D>
__device__ __forceinline__ void falloff(const double* fo, bool troe, double Mc, double& fac, double& dfac) {
    const double k0r = fo[0];
    const double Pr = k0r * Mc;
    double F = 1.0, g = 0.0;
    if (troe) {
        double x, den;
        F = troe_F(Pr, fo, x, den);
        if (WANT_D) {
            const double lfc = fo[1], nn = fo[3];
            const double f1 = x / den;
            const double df1 = nn / (den * den);
            g = -lfc * 2 * f1 / ((1 + f1 * f1) * (1 + f1 * f1)) * df1;
        }
    }
    fac = Pr / (1 + Pr) * F;
    if (WANT_D) dfac = (F / ((1 + Pr) * (1 + Pr)) + F * g / (1 + Pr)) * k0r;
}

// third-body concentrations of the efficiency sets: mc[s] = Ctot + sum (eff-1) c over the set's
// list (one lane per set; the list entries are read 2 at a time so the loads overlap)
template <int CPL>
__device__ __forceinline__ void third_body_sets(const DevMech& M, const Tab& tb_, double* sp, double Ctot, int lane) {
    const Tab tb = tab_view<CPL>(br_lds, M);
    const double* conc = sp + Lay<CPL>::CONC;
#pragma unroll 1
    for (int t = lane; t < MF(nset); t += WAVE) {
        const uint32_t w = tb.tbs[t];
        const int b = w & 0xFFFFF, e = b + (int)(w >> 20);
        double s0 = Ctot, s1 = 0.0;
        int i = b;
#pragma unroll 1
        for (; i + 1 < e; i += 2) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            const double2 e1 = *reinterpret_cast<const double2*>(tb.tbe + 16 * (i + 1));
            const int k0 = __double_as_longlong(e0.x) & 0xFFFF, k1 = __double_as_longlong(e1.x) & 0xFFFF;
            s0 = fma(e0.y, conc[k0], s0);
            s1 = fma(e1.y, conc[k1], s1);
        }
        if (i < e) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            s0 = fma(e0.y, conc[__double_as_longlong(e0.x) & 0xFFFF], s0);
        }
        sp[Lay<CPL>::MC + t] = s0 + s1;
    }
}

// rates of progress, accumulated straight into the per-species production sums:
// accw[k] += nu_kr q_r (gas reactions), accs[k] += nu_kr q_r (surface reactions)
// the {kf, kr} pairs of a lane's first two gas reactions (lane, lane + 64), issued at the start of
// the RHS so their global-memory latency overlaps the concentration and third-body setup
struct KPre {
    double2 a, b;
};
__device__ __forceinline__ double2 kpair(const BR_GLOBAL double* rxd, int r) {
    return make_double2(rxd[2 * r], rxd[2 * r + 1]);   // one 16-byte load
}
__device__ __forceinline__ KPre rx_prefetch(const RView& R, int lane) {
    const int nrg = MF(nrg);
    KPre k;
    k.a = kpair(R.rxd, lane < nrg ? lane : 0);
    k.b = kpair(R.rxd, lane + WAVE < nrg ? lane + WAVE : 0);
    return k;
}
template <int CPL>
__device__ __forceinline__ void production(const DevMech& M, const Tab& tb_, const RView& R_, double RT, int lane,
                                           KPre kp) {
    typedef Lay<CPL> L;
    const Tab tb = tab_view<CPL>(br_lds, M);
    const RView R = R_;
    const bool xm = (MF(conv) & 2) != 0;
    const double* conc = R.sp + L::CONC;
    double* accw = R.sp + L::ACCW;
    double* accs = R.sp + L::ACCS;
    // net rate of progress of gas reaction r (mass action x third body / falloff)
    auto rate = [&](int r, const uint4& ra, const double2 k) -> double {
        const uint32_t info = ra.z;
        const int tbk = gi_tb(info);
        // branch-free mass-action products: unused slots point at conc[L::ONE] = 1; mechanisms
        // with at most 3 reactants / products per reaction (MF(nu4) == 0, GRI) skip the 4th slot
        double Pf = (conc[sp8(ra.x, 0)] * conc[sp8(ra.x, 1)]) * conc[sp8(ra.x, 2)];
        double Pb = (conc[sp8(ra.y, 0)] * conc[sp8(ra.y, 1)]) * conc[sp8(ra.y, 2)];
        if (MF(nu4)) { Pf *= conc[sp8(ra.x, 3)]; Pb *= conc[sp8(ra.y, 3)]; }
        double D = k.x * Pf - k.y * Pb;
        if (tbk) {
            const double Mc = R.sp[L::MC + gi_tbidx(info)];
            if (tbk == 1) D *= Mc;
            else {
                double fac, dfac;
                falloff<false>(R.fod + 4 * gi_foidx(info), gi_troe(info) != 0, Mc, fac, dfac);
                D *= fac;
                if (xm) D *= Mc * 1e-6;                                // [M] in mol/cm3
            }
        }
        return D;
    };
    // two reactions per lane and iteration (r and r + 64): their LDS gather chains overlap; the
    // next iteration's {kf, kr} loads are issued one iteration ahead
    const int nrg = MF(nrg);
    double2 kn0 = kp.a, kn1 = kp.b;
#pragma unroll 1
    for (int r = lane; r < nrg; r += 2 * WAVE) {
        const int r1 = r + WAVE;
        const bool has1 = r1 < nrg;
        const int q1 = has1 ? r1 : r;
        const double2 k0 = kn0, k1 = has1 ? kn1 : kn0;
        if (r + 2 * WAVE < nrg) kn0 = kpair(R.rxd, r + 2 * WAVE);
        if (r + 3 * WAVE < nrg) kn1 = kpair(R.rxd, r + 3 * WAVE);
        const auto rr0 = rx_rec(tb.rx, r), rr1 = rx_rec(tb.rx, q1);
        const uint4 ra0 = *reinterpret_cast<const uint4*>(rr0.a);
        const uint4 rb0 = *reinterpret_cast<const uint4*>(rr0.b);
        const uint4 ra1 = *reinterpret_cast<const uint4*>(rr1.a);
        const uint4 rb1 = *reinterpret_cast<const uint4*>(rr1.b);
        const double D0 = rate(r, ra0, k0);
        const double D1 = rate(q1, ra1, k1);
        scatter(accw, rb0.x, rb0.y, rb0.z, rb0.w, D0);
        if (has1) scatter(accw, rb1.x, rb1.y, rb1.z, rb1.w, D1);
    }
#pragma unroll 1
    for (int r = lane; r < MF(nrs); r += WAVE) {
        const uint32_t* rec = tb.sx + SX_WORDS * r;
        const int nc = si_ncov(rec[4]);
        const double* xe = tb.sxe + SXE_DOUBLES * r;
        // k(T) times the constant site factors (Gamma/sigma per surface reactant, 1 for sticking)
        double k = R.skd[2 * r] * xe[4];
        if (nc) {
            const uint32_t cs = rec[5];
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += xe[j] * conc[sp8(cs, j)];
            k *= exp(-s / RT);
        }
        // branch-free product over up to 6 reactants (pad slots = conc[L::ONE] = 1)
        const double P = ((conc[sp8(rec[0], 0)] * conc[sp8(rec[0], 1)]) * (conc[sp8(rec[0], 2)] * conc[sp8(rec[0], 3)])) *
                         (conc[sp8(rec[1], 0)] * conc[sp8(rec[1], 1)]);
        scatter(accs, rec[6], rec[7], rec[8], rec[9], k * P);
    }
}

// residual! (src/BatchReactor.jl:312-376) for the components of `lane` (lane + 64 s, s < CPL):
// du[s]; writes the diagnosed pressure to *p_out (save_data semantics).
template <int CPL>
__device__ __forceinline__ void rhs(const DevMech& M, const Tab& tb_, const RView& R_, double T, double Asv,
                                    double Asv_th, const double (&u)[CPL], int lane, double* p_out,
                                    double (&du)[CPL]) {
    typedef Lay<CPL> L;
    const Tab tb = tab_view<CPL>(br_lds, M);
    const RView R = R_;
    BR_SUB_T(rt0);
    const KPre kp = rx_prefetch(R, lane);
    const int ng = MF(ng), n = MF(n);
    // Y = u/rho, x = (Y/M)/sum(Y/M), p = rho R T / Mbar (:326-338 / :349-353) give the gas
    // concentrations c_k = p x_k / (R T) = u_k / M_k exactly; p = R T sum_k c_k
    double cg = 0.0, Mk[CPL];
#pragma unroll
    for (int s = 0; s < CPL; ++s) {
        const int k = lane + 64 * s;
        const bool gas = k < ng;
        Mk[s] = tb.molwt[k];
        const double c = gas ? u[s] / Mk[s] : u[s];
        if (k < n) { R.sp[L::CONC + k] = c; R.sp[L::ACCW + k] = 0.0; R.sp[L::ACCS + k] = 0.0; }
        cg += gas ? c : 0.0;
    }
    const double Ctot = wave_sum(cg);
    const double p = R_GAS * T * Ctot;
    if (MF(nset)) {
        wave_sync();
        third_body_sets<CPL>(M, tb, R.sp, Ctot, lane);
    }
    wave_sync();
    BR_SUB_ADD(11, rt0);
    BR_SUB_T(rt1);
    production<CPL>(M, tb, R, R_GAS * T, lane, kp);              // :344, :355
    wave_sync();
    BR_SUB_ADD(12, rt1);
    double w[CPL], sf[CPL];
#pragma unroll
    for (int s = 0; s < CPL; ++s) {
        const int k = lane + 64 * s;
        w[s] = k < n ? R.sp[L::ACCW + k] : 0.0;
        sf[s] = k < n ? R.sp[L::ACCS + k] : 0.0;
    }
    wave_sync();
    if (lane == 0) *p_out = p;
#pragma unroll
    for (int s = 0; s < CPL; ++s) {
        const int k = lane + 64 * s;
        if (k < ng) du[s] = (sf[s] * Asv + w[s]) * Mk[s];          // :345, :363-370
        else if (k < n) du[s] = sf[s] * Asv_th * tb.sigma[k] / MF(G);   // :367 / :370
        else du[s] = 0.0;
    }
}

// analytic Jacobian d(du)/du, written column by column to the per-reactor workspace
// Jsave[j*64 + k] = J[k][j] (coalesced). Column j is built from the reactions whose rate
// depends on component j (host-built column lists, incl. third-body reactions). The
// per-reaction multipliers (pre, D*dpre/d[M]) go through a global scratch `jscr` (2 per gas
// reaction), written by the reaction's lane and read back by any lane with L1-bypassing loads.
__device__ __forceinline__ double ld_l2(const BR_GLOBAL double* p) {
    return __hip_atomic_load((const double*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Gas-only analytic Jacobian (DevMech::jfast), after the multiplier loop of jacobian() left
// jscr[2r] = pre_r and jscr[2r+1] = D_r d(pre_r)/d[M] (pre = [M] or the falloff factor):
//   dq_r/dc_j = pre_r (kf_r d(prod_f)/dc_j - kr_r d(prod_b)/dc_j) + D_r dpre_r/d[M] eff_{s(r),j}.
// The third-body term is a product over the efficiency sets s: with w_s[k] = sum over the
// third-body reactions r of set s of nu_kr D_r dpre_r/d[M], its contribution to J[k][j] is
// sum_s w_s[k] eff_{s,j}: nset scatter passes and nset FMAs per entry (efficiencies by scalar
// loads) instead of a column-list entry for every (third-body reaction, species) pair. The
// mass-action part runs over reactant / product column lists staged in the LDS image, with
// (pre kf, pre kr) as one 16-byte load per entry, issued an iteration ahead.
constexpr int JF_MAXSET = 16;
__device__ __forceinline__ void jacobian_fast(const Tab& tb, const RView& R, int lane, bool xm, BR_GLOBAL double* Jsave,
                                              BR_GLOBAL double* jscr) {
    BR_SUB_T(jc0);
    typedef Lay<1> L;
    const double* conc = R.sp + L::CONC;
    double* accw = R.sp + L::ACCW;
    double* accs = R.sp + L::ACCS;
    double* mcb = R.sp + L::MC;
    const int n = MF(n), nset = MF(nset), ntb = MF(ntbr);
    // per-reaction multipliers: jscr[2r] = pre kf, jscr[2r+1] = pre kr; D dpre/d[M] of the
    // third-body reaction on this lane (r = lane < ntb <= 64: third-body reactions come first)
    double dcm = 0.0;
#pragma unroll 1
    for (int r = lane; r < MF(nrg); r += WAVE) {
        const auto rec = rx_rec(tb.rx, r);
        const uint32_t info = rec[2];
        const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
        const double kf = R.rxd[2 * r], kr = R.rxd[2 * r + 1];
        double pre = 1.0;
        if (tbk) {
            double Pf = 1.0, Pb = 1.0;
            for (int e = 0; e < 4; ++e) if (e < nf) Pf *= conc[sp8(rec[0], e)];
            for (int e = 0; e < 4; ++e) if (e < nr) Pb *= conc[sp8(rec[1], e)];
            const double D = kf * Pf - kr * Pb;
            const double Mc = R.sp[L::MC + gi_tbidx(info)];
            double coefM;
            if (tbk == 1) { pre = Mc; coefM = 1.0; }
            else {
                double fac, dfac;
                falloff<true>(R.fod + 4 * gi_foidx(info), gi_troe(info) != 0, Mc, fac, dfac);
                pre = fac * (xm ? Mc * 1e-6 : 1.0);
                coefM = dfac * (xm ? Mc * 1e-6 : 1.0) + (xm ? fac * 1e-6 : 0.0);
            }
            dcm = D * coefM;
        }
        jscr[2 * r] = pre * kf;
        jscr[2 * r + 1] = pre * kr;
    }
    __builtin_amdgcn_s_waitcnt(0);   // scratch stores complete before other lanes read them
    wave_sync();
    // w_s[lane] for every efficiency set
    double w[JF_MAXSET];
    const auto recl = rx_rec(tb.rx, lane < ntb ? lane : 0);
    const uint32_t tbset = gi_tbidx(recl[2]);
#pragma unroll
    for (int st = 0; st < JF_MAXSET; ++st) {
        w[st] = 0.0;
        if (st < nset) {
            if (lane < n) accw[lane] = 0.0;
            wave_sync();
            if (lane < ntb && (int)tbset == st) scatter(accw, recl[4], recl[5], recl[6], recl[7], dcm);
            wave_sync();
            w[st] = (lane < n) ? accw[lane] : 0.0;
            wave_sync();
        }
    }
    BR_SUB_ADD(6, jc0);
    const int* cp = reinterpret_cast<const int*>(reinterpret_cast<const char*>(br_lds) + MF(cmp_off));
    const uint16_t* cr = reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(br_lds) + MF(cmr_off));
    const int* tjp = reinterpret_cast<const int*>(reinterpret_cast<const char*>(br_lds) + MF(tjp_off));
    const char* tje = reinterpret_cast<const char*>(br_lds) + MF(tje_off);
    // third-body part of J[k][j] = sum_s w_s[k] eff_{s,j} = wsum[k] + sum over the sets with
    // eff_{s,j} != 1 of w_s[k] (eff_{s,j} - 1): no efficiency loads for the other columns
    double wsum = 0.0;
#pragma unroll
    for (int st = 0; st < JF_MAXSET; ++st) if (st < nset) wsum += w[st];
    const double Mk = tb.molwt[lane];
    const double rMl = 1.0 / tb.molwt[lane];   // 1/M_j, broadcast from lane j for column j
    // (L1-bypassing loads: other lanes wrote the multipliers in this call; the slot's L1 lines may
    // be stale.) The first entry of every pass is fetched while the previous pass writes its
    // columns, so no pass starts on a full L2 round trip.
    auto fetch = [&](int i, int ce, int& r, double2& pk) {
        r = (i < ce) ? (int)cr[i] : 0;
        pk = (i < ce) ? make_double2(ld_l2(jscr + 2 * r), ld_l2(jscr + 2 * r + 1)) : make_double2(0.0, 0.0);
    };
    int rq;
    double2 pq;
    fetch(uni(cp[0]) + lane, uni(cp[min(3, n)]), rq, pq);
#pragma unroll 1
    for (int j0 = 0; j0 < n; j0 += 3) {
        if (lane < n) { accw[lane] = 0.0; accs[lane] = 0.0; mcb[lane] = 0.0; }
        const int cb = uni(cp[j0]), c1 = uni(cp[min(j0 + 1, n)]), c2 = uni(cp[min(j0 + 2, n)]), ce = uni(cp[min(j0 + 3, n)]);
        wave_sync();
        BR_SUB_T(je0);
        double sf0 = 0.0, sf1 = 0.0, sf2 = 0.0;   // d(nu_j q)/dc_j of the entries of columns j0 .. j0+2
        int i = cb + lane;
        int r = rq;
        double2 pk = pq;
#pragma unroll 1
        for (; i < ce; i += WAVE) {
            const int in = i + WAVE;
            const int rn = (in < ce) ? (int)cr[in] : 0;
            const double2 pkn = (in < ce) ? make_double2(ld_l2(jscr + 2 * rn), ld_l2(jscr + 2 * rn + 1)) : make_double2(0.0, 0.0);
            const int j = j0 + (i >= c1) + (i >= c2);
            double* acc = (i >= c2) ? mcb : (i >= c1) ? accs : accw;
            const auto rec = rx_rec(tb.rx, r);
            const uint32_t info = rec[2];
            const int nf = gi_nf(info), nr = gi_nr(info);
            double d = 0.0;
#pragma unroll
            for (int e = 0; e < 4; ++e) if (e < nf && sp8(rec[0], e) == j) {
                double pr = pk.x;
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= conc[sp8(rec[0], e2)];
                d += pr;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) if (e < nr && sp8(rec[1], e) == j) {
                double pr = pk.y;
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= conc[sp8(rec[1], e2)];
                d -= pr;
            }
            const double sv = scatter_noself(acc, rec[4], rec[5], rec[6], rec[7], d, j);
            if (i >= c2) sf2 += sv;
            else if (i >= c1) sf1 += sv;
            else sf0 += sv;
            r = rn;
            pk = pkn;
        }
        wave_sync();
        BR_SUB_ADD(4, je0);
        BR_SUB_T(je1);
        if (j0 + 3 < n) fetch(uni(cp[j0 + 3]) + lane, uni(cp[min(j0 + 6, n)]), rq, pq);
        const double st0 = wave_sum(sf0), st1 = wave_sum(sf1), st2 = wave_sum(sf2);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int j = j0 + c;
            if (j < n) {
                const double* acc = c == 0 ? accw : c == 1 ? accs : mcb;
                double v = (lane < n ? acc[lane] : 0.0) + wsum;
                if (lane == j) v += (c == 0 ? st0 : c == 1 ? st1 : st2);
                const int t0 = uni(tjp[j]), t1 = uni(tjp[j + 1]);
                for (int e = t0; e < t1; ++e) {
                    const int se = uni(*reinterpret_cast<const int*>(tje + 16 * e));
                    double ws = 0.0;
#pragma unroll
                    for (int st = 0; st < JF_MAXSET; ++st) ws = (st == se) ? w[st] : ws;
                    v = fma(ws, *reinterpret_cast<const double*>(tje + 16 * e + 8), v);
                }
                Jsave[j * WAVE + lane] = (lane < n) ? Mk * v * bcast(rMl, j) : 0.0;
            }
        }
        wave_sync();
        BR_SUB_ADD(5, je1);
    }
}

template <int CPL>
__device__ __forceinline__ void jacobian(const DevMech& M, const Tab& tb_, const RView& R_, double T, double Asv,
                                         double Asv_th, const double (&u)[CPL], int lane, double* Jsave_,
                                         double* jscr_) {
    typedef Lay<CPL> L;
    constexpr int JW = CPL == 2 ? 80 : 64;   // Jacobian column stride (CPL = 2: CR2 rows, see lu_factor2)
    BR_GLOBAL double* Jsave = launder(Jsave_);
    BR_GLOBAL double* jscr = launder(jscr_);
    const Tab tb = tab_view<CPL>(br_lds, M);
    const RView R = R_;
    const double RT = R_GAS * T;
    const bool xm = (MF(conv) & 2) != 0;
    double* conc = R.sp + L::CONC;
    double* accw = R.sp + L::ACCW;
    double* accs = R.sp + L::ACCS;
    double cg = 0.0;
#pragma unroll
    for (int s = 0; s < CPL; ++s) {
        const int k = lane + 64 * s;
        const bool gas = k < MF(ng);
        const double c = gas ? u[s] / tb.molwt[k] : u[s];          // c_k = u_k/M_k = p x_k/(RT)
        if (k < MF(n)) conc[k] = c;
        cg += gas ? c : 0.0;
    }
    const double Ctot = wave_sum(cg);
    wave_sync();
    BR_SUB_T(jt0);
    if (MF(nset)) {
        third_body_sets<CPL>(M, tb, R.sp, Ctot, lane);
        wave_sync();
    }
    if constexpr (CPL == 1) {
        if (MF(jfast)) {
            jacobian_fast(tb, R, lane, xm, Jsave, jscr);
            return;
        }
    }
#pragma unroll 1
    for (int r = lane; r < MF(nrg); r += WAVE) {                   // per-reaction multipliers
        const auto rec = rx_rec(tb.rx, r);
        const uint32_t info = rec[2];
        const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
        const double kf = R.rxd[2 * r], kr = R.rxd[2 * r + 1];
        double Pf = 1.0, Pb = 1.0;
        for (int e = 0; e < 4; ++e) if (e < nf) Pf *= conc[sp8(rec[0], e)];
        for (int e = 0; e < 4; ++e) if (e < nr) Pb *= conc[sp8(rec[1], e)];
        const double D = kf * Pf - kr * Pb;
        double pre = 1.0, coefM = 0.0;
        if (tbk) {
            const double Mc = R.sp[L::MC + gi_tbidx(info)];
            if (tbk == 1) { pre = Mc; coefM = 1.0; }
            else {
                double fac, dfac;
                falloff<true>(R.fod + 4 * gi_foidx(info), gi_troe(info) != 0, Mc, fac, dfac);
                pre = fac * (xm ? Mc * 1e-6 : 1.0);
                coefM = dfac * (xm ? Mc * 1e-6 : 1.0) + (xm ? fac * 1e-6 : 0.0);
            }
        }
        jscr[2 * r] = pre;
        jscr[2 * r + 1] = D * coefM;
    }
#pragma unroll 1
    for (int r = lane; r < MF(nrs); r += WAVE) {
        const uint32_t* rec = tb.sx + SX_WORDS * r;
        const int nc = si_ncov(rec[4]);
        double k = R.skd[2 * r];
        if (nc) {
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += tb.sxe[SXE_DOUBLES * r + j] * conc[sp8(rec[5], j)];
            k *= exp(-s / RT);
        }
        R.skd[2 * r + 1] = k;
    }
    __builtin_amdgcn_s_waitcnt(0);   // scratch stores complete before other lanes read them
    wave_sync();
    if (CPL == 1 && MF(nrs) == 0) {
        // gas-only: three columns per pass (accumulators accw | accs | mc: the surface sums and the
        // third-body sums are idle here), over the concatenated column lists of j0..j0+2 (contiguous
        // in col_rx), so 18 passes with 3 wave barriers each instead of 53 for GRI
        double* mcb = R.sp + L::MC;
        const int n = MF(n);
        BR_SUB_ADD(6, jt0);
#pragma unroll 1
        for (int j0 = 0; j0 < n; j0 += 3) {
            if (lane < n) { accw[lane] = 0.0; accs[lane] = 0.0; mcb[lane] = 0.0; }
            wave_sync();
            const int* cp = MF(col_ptr);
            const int cb = cp[j0], c1 = cp[min(j0 + 1, n)], c2 = cp[min(j0 + 2, n)], ce = cp[min(j0 + 3, n)];
            BR_SUB_T(jt2);
#pragma unroll 1
            for (int i = cb + lane; i < ce; i += WAVE) {
                const int r = MF(col_rx)[i];
                const int j = j0 + (i >= c1) + (i >= c2);
                double* acc = (i >= c2) ? mcb : (i >= c1) ? accs : accw;
                const auto rec = rx_rec(tb.rx, r);
                const uint32_t info = rec[2];
                const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
                const double pre = ld_l2(jscr + 2 * r);
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nf && sp8(rec[0], e) == j) {
                    double pr = R.rxd[2 * r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= conc[sp8(rec[0], e2)];
                    d += pre * pr;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nr && sp8(rec[1], e) == j) {
                    double pr = R.rxd[2 * r + 1];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= conc[sp8(rec[1], e2)];
                    d -= pre * pr;
                }
                if (tbk && j < MF(ng)) d += ld_l2(jscr + 2 * r + 1) * MF(tb_eff)[gi_tbidx(info) * n + j];
                scatter(acc, rec[4], rec[5], rec[6], rec[7], d);
            }
            wave_sync();
            BR_SUB_ADD(4, jt2);
            BR_SUB_T(jt3);
            const double Mk = tb.molwt[lane];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int j = j0 + c;
                if (j < n) {
                    const double* acc = c == 0 ? accw : c == 1 ? accs : mcb;
                    const double w = lane < n ? acc[lane] : 0.0;
                    Jsave[j * JW + lane] = (lane < n) ? Mk * w / tb.molwt[j] : 0.0;
                }
            }
            wave_sync();
            BR_SUB_ADD(5, jt3);
        }
        return;
    }
#pragma unroll 1
    for (int j = 0; j < MF(n); ++j) {
#pragma unroll
        for (int s = 0; s < CPL; ++s) {
            const int k = lane + 64 * s;
            if (k < MF(n)) { accw[k] = 0.0; accs[k] = 0.0; }
        }
        wave_sync();
        const int cb = MF(col_ptr)[j], ce = MF(col_ptr)[j + 1];
#pragma unroll 1
        for (int i = cb + lane; i < ce; i += WAVE) {
            const int rr = MF(col_rx)[i];
            if (rr < MF(nrg)) {
                const int r = rr;
                const auto rec = rx_rec(tb.rx, r);
                const uint32_t info = rec[2];
                const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
                const double pre = ld_l2(jscr + 2 * r);
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nf && sp8(rec[0], e) == j) {
                    double pr = R.rxd[2 * r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= conc[sp8(rec[0], e2)];
                    d += pre * pr;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nr && sp8(rec[1], e) == j) {
                    double pr = R.rxd[2 * r + 1];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= conc[sp8(rec[1], e2)];
                    d -= pre * pr;
                }
                if (tbk && j < MF(ng)) d += ld_l2(jscr + 2 * r + 1) * MF(tb_eff)[gi_tbidx(info) * MF(n) + j];
                scatter(accw, rec[4], rec[5], rec[6], rec[7], d);
            } else {
                const int r = rr - MF(nrg);
                const uint32_t* rec = tb.sx + SX_WORDS * r;
                const uint32_t info = rec[4];
                const int nf = si_nf(info), nc = si_ncov(info);
                const bool stick = si_stick(info);
                const double k = R.skd[2 * r + 1];
                double cv[6], dc[6];
                int sp[6];
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    sp[e] = e < nf ? (e < 4 ? sp8(rec[0], e) : sp8(rec[1], e - 4)) : -1;
                    cv[e] = 1.0; dc[e] = 0.0;
                    if (e < nf) {
                        const int s = sp[e];
                        if (s < MF(ng)) { cv[e] = conc[s]; dc[e] = 1.0 / tb.molwt[s]; }
                        else if (stick) { cv[e] = conc[s]; dc[e] = 1.0; }
                        else { cv[e] = conc[s] * MF(G) / tb.sigma[s]; dc[e] = MF(G) / tb.sigma[s]; }
                    }
                }
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 6; ++e) if (sp[e] == j) {
                    double pr = k;
#pragma unroll
                    for (int e2 = 0; e2 < 6; ++e2) if (e2 != e && e2 < nf) pr *= cv[e2];
                    d += pr * dc[e];
                }
                if (nc) {
                    double P = 1.0;
#pragma unroll
                    for (int e = 0; e < 6; ++e) if (e < nf) P *= cv[e];
                    const double q = k * P;
                    for (int jj = 0; jj < 4; ++jj) if (jj < nc && sp8(rec[5], jj) == j)
                        d += q * (-tb.sxe[SXE_DOUBLES * r + jj] / RT);
                }
                scatter(accs, rec[6], rec[7], rec[8], rec[9], d);
            }
        }
        wave_sync();
#pragma unroll
        for (int s = 0; s < CPL; ++s) {
            const int k = lane + 64 * s;
            const bool act = k < MF(n);
            const double w = act ? accw[k] : 0.0;
            const double sf = act ? accs[k] : 0.0;
            const double Mk = tb.molwt[k];
            double v;
            if (k < MF(ng)) v = (j < MF(ng) ? Mk * w / tb.molwt[j] : 0.0) + Mk * Asv * sf;
            else v = Asv_th * tb.sigma[k] / MF(G) * sf;
            if (k < JW) Jsave[j * JW + k] = act ? v : 0.0;
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------------------------
// LU of A = I - gamma*J, row-per-lane (SUNDIALS denseGETRF semantics: partial pivoting on the
// first max |a_ik| in row order, multipliers l_ik = a_ik / a_kk, a_ij -= l_ik a_kj), without
// physical row swaps during the factorization (see LUWs for the stored form).
// Pivot search on the bit patterns of |a_ik| (monotone for non-negative doubles): a 32-bit
// DPP max over the high words, a second pass over the low words only when the high words tie,
// then, among candidates holding the max, the one with the lowest ORIGINAL row index = the first
// max in row order (the rows sit in lanes in the previous factorization's pivot order, lu_factor).
// ------------------------------------------------------------------------------------
// Wave max of a 32-bit value: 4 DPP steps inside each 16-lane row, then row_bcast:15 carries row r's
// max into row r + 1 (rows 1, 3) and row_bcast:31 row 1's into rows 2 and 3, so lane 63 holds the
// wave max; each step is one v_max_u32_dpp (written as inline asm: the compiler split the two
// row-masked steps into a v_mov, a v_mov_dpp and a v_max each). s_nop 1: the VALU-write ->
// DPP-read hazard of each step, and the readlane after the last.
__device__ __forceinline__ unsigned wave_umax(unsigned x) {
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
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "=&v"(r)
        : "v"(x));
    return __builtin_amdgcn_readlane(r, 63);
}
// a = a_ik, cm = 0x7fffffff on candidate rows (not pivoted yet), 0 elsewhere; prow = original row
// index held by this lane. hi = high word of |a_ik| on candidates, 0 elsewhere, so when the max is
// not 0 the lanes holding it are candidates (one compare for the ballot).
__device__ __forceinline__ int pivot_lane(double a, unsigned cm, int prow) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(a);
    const unsigned hi = (unsigned)(bits >> 32) & cm;
    const unsigned mh = wave_umax(hi);
    unsigned long long m = (mh != 0) ? __ballot(hi == mh) : __ballot(cm != 0);
    if (__builtin_popcountll(m) > 1) {
        const bool top = (mh != 0) ? (hi == mh) : (cm != 0);
        const unsigned lo = top ? (unsigned)bits : 0u;
        const unsigned ml = wave_umax(lo);
        const bool top2 = top && lo == ml;
        m = __ballot(top2);
        if (__builtin_popcountll(m) > 1) {   // an exact tie: the first in original row order
            const unsigned key = top2 ? ~(unsigned)prow : 0u;
            const unsigned mk = wave_umax(key);
            m = __ballot(top2 && key == mk);
        }
    }
    return m ? (int)__builtin_ctzll(m) : 0;
}
// Factor workspace (global, per reactor): ONE combined factor matrix, column-major, NMAX rows
// per column (round 3: 56 for GRI instead of 64: 12.5 % less factor footprint and solve traffic), rows in pivot-step order after lu_factor returns: column k holds L[s][k] on rows
// s > k, U'[s][k] = (D^-1 U)[s][k] on rows s < k and 0 on s = k; then D^-1 in step order.
// The forward sweep reads only rows below the diagonal and the backward sweep only rows above
// it (exec-masked loads skip whole 128-B lines), so a solve moves ~n^2 doubles instead of 2*n*64.
// (A packed-triangle layout -- each sweep reading one triangle front to back, 25.5 KB instead of
// ~29 KB per GRI solve from the fabric -- measured 2.7 % slower in round 3: its column segments
// start at arbitrary 8-B offsets, so every load instruction spans one more 128-B line.)
struct LUWs {
    BR_GLOBAL double* M;
    BR_GLOBAL double* D;
};
// raw buffer ops over the CPL = 1 factor matrix: the column base goes in soffset (scalar), the
// row in the per-lane offset; a lane that holds no row (lane >= FR) gets an out-of-range offset,
// so the buffer range check drops its stores and returns 0 for its loads (no exec masks, no
// address selects)
constexpr unsigned LU_OOB = 0x80000000u;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lu_rsrc(BR_GLOBAL double* M, int doubles) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)M, (short)0, doubles * 8, 0x00020000);
}
typedef __attribute__((address_space(3))) double LDSd;
typedef __attribute__((address_space(3))) int LDSi;

// right-looking steps k0..k1-1 on a left-aligned row segment a[0..W-1] (a[0] = column k0 on
// entry) whose columns end at `cend`: pivot search on a[0], column k of the factors (lane = the
// row it holds), rank-1 update of the live columns, shift by one (the k-loop stays rolled).
// Live columns go in chunks of BR_LU_CH (round 3: 4 instead of 8 = -61k VALU instructions per GRI
// reactor, +0.4 %; bit-identical).
#ifndef BR_LU_CH
#define BR_LU_CH 4
#endif
template <int W, int FR>
__device__ __forceinline__ void lu_rl_steps(double (&a)[W], int k0, int k1, int cend, int lane, int prow, int& pstep,
                                            double& dinv, int& fail, __amdgpu_buffer_rsrc_t rs) {
    constexpr int CH = BR_LU_CH;   // live-column granularity of the rank-1 update
    // factor columns hold FR = NMAX rows (lanes >= FR never hold a row: their stores are dropped)
    const unsigned fo8 = (lane < FR) ? (unsigned)lane * 8u : LU_OOB;
    static_assert(W % CH == 0, "W must be a multiple of the chunk");
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const bool cand = pstep < 0;
        // rows sit in the previous factorization's pivot order, so step k's pivot is usually on lane k:
        // when lane k is a candidate and no other candidate holds |a_ik| >= |a_kk|, lane k is the first
        // max |a| of denseGETRF and the DPP max passes are skipped (ties or a larger entry: the full
        // search). Round 6: bit-identical (scripts/bitcmp.py, GRI 4000 / surface 8000 reactors), GRI
        // +0.6 %, surface-only +0.0 %; the same fast path in the CPL = 2 LU measured -0.2 % on C5
        // (profiles/r06_lu_fastpiv_ab.json) and is not used there
        const double akk = bcast(a[0], k);
        const bool kcand = (__ballot(cand) >> k) & 1ull;
        const bool fast = kcand && __ballot(cand && lane != k && !(fabs(a[0]) < fabs(akk))) == 0;
        const int p = fast ? k : pivot_lane(a[0], cand ? 0x7fffffffu : 0u, prow);
        const double piv = fast ? akk : bcast(a[0], p);
        if (piv == 0.0 && !fail) fail = k + 1;
        const double rinv = 1.0 / piv;
        const bool isp = (lane == p);
        const bool rem = cand && !isp;
        const double l = rem ? a[0] * rinv : 0.0;
        const double fv = rem ? l : (cand ? 0.0 : a[0] * dinv);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, fv), rs, fo8, k * (FR * 8), 0);
        if (isp) { pstep = k; dinv = rinv; }
        const int live = cend - k;              // columns k..cend-1 are live in a[0..live-1]
#pragma unroll
        for (int c = 0; c < W; c += CH) {
            if (c < live) {
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    const int j = c + i;
                    if (j + 1 < W) a[j] = fma(-bcast_lu(a[j + 1], p), l, a[j + 1]);
                    else a[j] = 0.0;
                }
            }
        }
    }
}

// row order after factorization: lane s works on the pivot row of step s, i.e. original row
// perm[s] (perm = inverse of pstep); lanes >= n map to themselves
__device__ __forceinline__ int pivot_perm(int pstep, int lane, int n) {
    const int dst = (lane < n) ? pstep : lane;
    return __builtin_amdgcn_ds_permute(dst * 4, lane);
}
__device__ __forceinline__ double lane_pull(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src * 4, (int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_bpermute(src * 4, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// LU in two column panels of P = 32 (registers: 2P per lane, not 2n): panel 1 = columns
// 0..P-1 factored right-looking; panel 2 = columns P..n-1 first receives the P updates of panel
// 1 (left-looking: multipliers re-read from M, masked to rows not yet pivoted at that step;
// pivot-row values broadcast from the panel-2 registers of the pivot lane, in step order), then
// is factored right-looking. The arithmetic is exactly that of the unblocked right-looking LU.
// The rows are loaded into the lanes in the previous factorization's pivot order (perm_io: lane s
// holds original row perm_io[s]; the identity for a reactor's first LU): the rows of a stiff system
// keep their pivot order from one Newton matrix to the next, so every step's pivot then sits on
// the lane of its step, the factor matrix M comes out in pivot-step order as it is written, and
// the gather pass (a read and a write of the whole matrix, ~9 MB per GRI reactor) is skipped.
// Otherwise the rows of M are gathered into step order (in place) as before. D^-1 is stored in
// step order. Row placement does not change the arithmetic: each row gets the same FMAs, and ties
// in the pivot search go to the lowest original row. Returns 0 or k+1 for a zero pivot; perm_io:
// step s -> original row on return.
template <int NMAX>
__device__ __forceinline__ int lu_factor(const double* __restrict__ J_, double* __restrict__ ws, double gamma, int n,
                                         int lane, int& perm_io) {
    constexpr int P = NMAX < 32 ? NMAX : 32;
    constexpr int W2 = NMAX - P > 0 ? NMAX - P : 8;
    constexpr int CH = 8;
    static_assert(NMAX % CH == 0 && NMAX <= 64, "lu_factor: NMAX");
    const BR_GLOBAL double* J = launder(J_);
    BR_GLOBAL double* wsg = launder(ws);
    constexpr int FR = NMAX;   // factor column stride (rows): [M: NMAX columns of NMAX rows | D^-1: 64]
    const LUWs F{wsg, wsg + NMAX * FR};
    const __amdgpu_buffer_rsrc_t rs = lu_rsrc(wsg, NMAX * FR);   // the factor columns M
    lane = launder_v(lane);
    n = launder_s(n);
    // the saved J through a buffer of n columns: a column j >= n, and any lane that holds no row,
    // is out of range and reads 0 (no exec masks or per-column conditions; the column goes in the
    // per-lane offset, whose immediate part covers 8 columns)
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc((void*)J, (short)0, n * (WAVE * 8), 0x00020000);
    const int prow = launder_v(perm_io);      // original row held by this lane (lanes >= n: lane)
    const bool act = lane < n;
    const unsigned jo8 = act ? (unsigned)prow * 8u : LU_OOB;
    auto ldj = [&](int col) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, jo8 + col * (WAVE * 8), 0, 0));
    };
    int pstep = act ? -1 : 1024;
    double dinv = 0.0;
    int fail = 0;
    const int n1 = n < P ? n : P;
    BR_SUB_T(lt0);
    {
        double a[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const double jv = ldj(j);
            a[j] = ((j == prow) ? 1.0 : 0.0) - gamma * jv;
        }
        lu_rl_steps<P, FR>(a, 0, n1, n1, lane, prow, pstep, dinv, fail, rs);
    }
    BR_SUB_ADD(0, lt0);
    BR_SUB_T(lt1);
    if (NMAX > P && n > P) {
        double b[W2];
#pragma unroll
        for (int j = 0; j < W2; ++j) {
            const int col = P + j;
            const double jv = ldj(col);
            b[j] = ((col == prow) ? 1.0 : 0.0) - gamma * jv;
        }
        // multipliers of panel 1 re-read from M, one chunk of CH steps ahead (lanes >= FR read 0
        // through the buffer range check)
        const unsigned lo8 = (lane < FR) ? (unsigned)lane * 8u : LU_OOB;
        auto ldm = [&](double (&v)[CH], int c0) {
#pragma unroll
            for (int i = 0; i < CH; ++i)
                v[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lo8 + i * (FR * 8), c0 * (FR * 8), 0));
        };
        auto ll_chunk = [&](const double (&cur)[CH], int kb) {
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                const int k = kb + i;
                const unsigned long long m = __ballot(pstep == k);
                const int p = (int)__builtin_ctzll(m);
                const double l = ((unsigned)pstep > (unsigned)k) ? cur[i] : 0.0;   // not pivoted by step k
                // padding columns P + j >= n skipped; the bound is made opaque per step so each test
                // stays a scalar compare and branch (hoisted, the tests became lane masks with two
                // VALU ops per column and step to carry them)
                int nl = n - P;
                asm volatile("" : "+s"(nl));
#pragma unroll
                for (int j = 0; j < W2; ++j)
                    if (j + 8 < W2 || j < nl) b[j] = fma(-bcast_lu(b[j], p), l, b[j]);
            }
        };
        double cur[CH], nxt[CH];
        ldm(cur, 0);
#pragma unroll 1
        for (int kb = 0; kb < P; kb += CH) {
            if (kb + CH < P) ldm(nxt, kb + CH);
            ll_chunk(cur, kb);
#pragma unroll
            for (int i = 0; i < CH; ++i) cur[i] = nxt[i];
        }
        lu_rl_steps<W2, FR>(b, P, n, n, lane, prow, pstep, dinv, fail, rs);
    }
    BR_SUB_ADD(1, lt1);
    BR_SUB_T(lt2);
    constexpr int NC = NMAX / CH;
    int perm;
    if (__ballot(act && pstep != lane) == 0) {
        // pivots in lane order: M is in step order already; padding columns n..NMAX-1 are zeros
        perm = prow;
        if (lane < FR)
            for (int c = n; c < NMAX; ++c) F.M[c * FR + lane] = 0.0;
        F.D[lane] = dinv;
    } else {
        // rows into step order, in place: chunk c is gathered completely before it is stored, and
        // the gathers of chunk c+1 are in flight while chunk c is stored (columns >= n: zeros)
        const int q = pivot_perm(pstep, lane, n);   // lane holding the row of step `lane`
        perm = __builtin_amdgcn_ds_bpermute(q * 4, prow);
        double g[2][CH];
        auto gather = [&](double (&v)[CH], int c) {
#pragma unroll
            for (int i = 0; i < CH; ++i) v[i] = F.M[min(c + i, n - 1) * FR + min(q, FR - 1)];
        };
        gather(g[0], 0);
#pragma unroll
        for (int t = 0; t < NC; ++t) {
            if (t + 1 < NC) gather(g[(t + 1) & 1], (t + 1) * CH);
            __builtin_amdgcn_sched_barrier(0);
            if (lane < FR) {
#pragma unroll
                for (int i = 0; i < CH; ++i) F.M[(t * CH + i) * FR + lane] = (t * CH + i < n) ? g[t & 1][i] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        F.D[lane] = lane_pull(dinv, q);
    }
    BR_SUB_ADD(2, lt2);
    perm_io = perm;
    return fail;
}

// (The blocked LU with fp64 MFMA trailing updates, lu_factor_mf, measured and not adopted in round 4,
// lives in the variant library csrc/variants/brhip_lumf.hip -> libbrhip_lumf.so since round 6.)

// ---- triangular sweeps in DPP form: the columns go in blocks of 16, one block per 16-lane DPP
// row. Block b first runs its diagonal 16 x 16 part inside row b: r += -M[s][k] * r[k], with r[k]
// broadcast from lane k of the row by the DPP modifier of the FMA itself (v_fmac_f64
// row_newbcast) and the write limited to row b by the DPP row mask: one VALU op per column
// instead of two v_readlane + FMA, no exec change, no branch. The finished values of row b are
// then copied to every row through LDS (one write, one read) and the rows below (forward) /
// above (backward) apply the block's columns with the same DPP FMA on the copy. Every lane
// accumulates its columns in column order with fma(-M[s][k], r[k], r[s]), i.e. the arithmetic
// of a plain column-oriented substitution (bit-identical to the readlane form).
// r += -f * r[row base + K] in the rows of RM; the s_nop covers the VALU-write -> DPP-read
// hazard on r (the previous op of the chain wrote it)
template <int K, int RM>
__device__ __forceinline__ void dpp_fnma_self(double& r, double f) {
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, -%1 row_newbcast:%2 row_mask:%3 bank_mask:0xf"
                 : "+v"(r) : "v"(f), "i"(K), "i"(RM));
}
// r += -f * x[row base + K] in the rows of RM. x is the DPP-read operand: the first op of a chain
// (NOP) carries the s_nop itself, since LLVM's hazard recognizer does not see a DPP read inside
// inline asm and may place a VALU copy of x right before it; later ops of the chain read the same x
template <int K, int RM, bool NOP = false>
__device__ __forceinline__ void dpp_fnma(double& r, double x, double f) {
    if constexpr (NOP)
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:%4 bank_mask:0xf"
                     : "+v"(r) : "v"(x), "v"(f), "i"(K), "i"(RM));
    else
        asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:%4 bank_mask:0xf"
                     : "+v"(r) : "v"(x), "v"(f), "i"(K), "i"(RM));
}
template <bool FWD, int CW, int RM, int I>
__device__ __forceinline__ void dpp_diag(double& r, const double (&v)[16]) {
    if constexpr (I < CW) {
        constexpr int K = FWD ? I : CW - 1 - I;
        dpp_fnma_self<K, RM>(r, v[K]);
        dpp_diag<FWD, CW, RM, I + 1>(r, v);
    }
}
template <bool FWD, int CW, int RM, int I>
__device__ __forceinline__ void dpp_off(double& r, double x, const double (&v)[16]) {
    if constexpr (I < CW) {
        constexpr int K = FWD ? I : CW - 1 - I;
        dpp_fnma<K, RM, I == 0>(r, x, v[K]);
        dpp_off<FWD, CW, RM, I + 1>(r, x, v);
    }
}
// Diagonal-redirect loads: the step-ordered factor matrix holds an exact 0 at (k, k) and in every
// row >= n, so a lane that must not update in column k loads row k of that column: row =
// max(lane, k) in the forward sweep (rows > k update), min(lane, k) in the backward sweep (rows
// < k). The loaded factor is then the masked one, with no compare/select per column, and row k
// shares a 128-B line with the rows that do update except at 3 line boundaries. Raw buffer
// loads: per-lane offset in the VGPR (one v_max / v_min per column), the chunk's column base
// c * 512 B in soffset and the column within the chunk as the immediate (<= 3584 B).
// cache policy of the solve's factor loads (aux bits of the buffer load: 2 = nt, streaming). A
// factor line is re-read only by the wave's next solve, ~60k cycles later, after the XCD's other
// 511 waves have streamed ~17 MB through its 4 MB L2: it never survives there.
#ifndef BR_SOLVE_AUX
#define BR_SOLVE_AUX 0
#endif
// Each 8-column chunk is read through its own buffer descriptor: base = the chunk's first column,
// range = its columns < n. The range check covers the VGPR offset + immediate, not soffset. So the
// padding columns n..NMAX-1 (zeros) read 0 without a memory access: 3 of 56 columns at GRI's n = 53,
// 12 of 32 for the surface-only n = 20. No VALU cost; the descriptor is 4 SALU ops per chunk.
template <bool FWD, int FR>
__device__ __forceinline__ void tri_load_diag(double (&v)[8], const BR_GLOBAL double* wsg, int n, int c, unsigned ld8) {
    // ld8: the lane clamped to FR - 1 (lanes >= FR are never sources; they read row FR - 1)
    const int live = n - c < 0 ? 0 : (n - c > 8 ? 8 : n - c);
    const __amdgpu_buffer_rsrc_t rc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(wsg + c * FR), (short)0, live * (FR * 8), 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const unsigned k8 = (unsigned)(c + i) * 8u;
        const unsigned off = FWD ? max(ld8, k8) : min(ld8, k8);
        v[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, off + i * (FR * 8), 0, BR_SOLVE_AUX));
    }
}
// block T of a sweep (blocks of 16 columns, the last one NMAX % 16 wide if that is not 0),
// factor loads one block ahead; x64 = 64 doubles of LDS scratch
template <bool FWD, int NMAX, int T>
__device__ __forceinline__ void tri_block_dpp(const BR_GLOBAL double* wsg, int n, unsigned lane8, unsigned ld8, double& r,
                                              LDSd* x64, double (&v)[2][16]) {
    constexpr int NB = (NMAX + 15) / 16;
    if constexpr (T < NB) {
        constexpr int B = FWD ? T : NB - 1 - T;            // block = DPP row
        constexpr int CW = (16 * B + 16 > NMAX) ? NMAX - 16 * B : 16;
        auto load = [&](double (&d)[16], int blk) {
            tri_load_diag<FWD, NMAX>(*reinterpret_cast<double(*)[8]>(&d[0]), wsg, n, 16 * blk, ld8);
            if (16 * blk + 8 < NMAX) tri_load_diag<FWD, NMAX>(*reinterpret_cast<double(*)[8]>(&d[8]), wsg, n, 16 * blk + 8, ld8);
        };
        if constexpr (T == 0) load(v[0], B);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (T + 1 < NB) load(v[(T + 1) & 1], FWD ? B + 1 : B - 1);
        __builtin_amdgcn_sched_barrier(0);
        const double (&f)[16] = v[T & 1];
        dpp_diag<FWD, CW, 1 << B, 0>(r, f);
        constexpr int ROWS = FWD ? (0xF << (B + 1)) & 0xF : (1 << B) - 1;   // rows still to update
        if constexpr (ROWS != 0) {
            asm volatile("s_nop 1");                       // r: DPP-encoded VALU write (inline asm)
            x64[(lane8 >> 3)] = r;
            wave_sync();
            const double x = x64[16 * B + ((lane8 >> 3) & 15)];
            dpp_off<FWD, CW, ROWS, 0>(r, x, f);
            wave_sync();
        }
        tri_block_dpp<FWD, NMAX, T + 1>(wsg, n, lane8, ld8, r, x64, v);
    }
}
template <bool FWD, int NMAX>
__device__ __forceinline__ void tri_sweep_dpp(const BR_GLOBAL double* wsg, int n, int lane, double& r, LDSd* x64) {
    double v[2][16];
    tri_block_dpp<FWD, NMAX, 0>(wsg, n, (unsigned)lane * 8u, (unsigned)min(lane, NMAX - 1) * 8u, r, x64, v);
    asm volatile("s_nop 1");
}

// solve (I - gamma J) x = b with the factors of lu_factor: L y = P b, y' = D^-1 y, U' x = y'.
// `perm` from lu_factor; b and the returned x are in natural component order (the backward
// sweep leaves unknown s, i.e. column s, on lane s). x16: 64 doubles of LDS scratch.
template <int NMAX>
__device__ __forceinline__ double lu_solve(const double* __restrict__ ws, int n, int lane, int perm, double b,
                                           LDSd* x16) {
    static_assert(NMAX % 8 == 0 && NMAX <= 64, "lu_solve: NMAX");
    const BR_GLOBAL double* wsg = launder(ws);
    lane = launder_v(lane);
    // one buffer descriptor over factors + D^-1: every load of the solve is a buffer load, so the
    // waitcnt pass can count them in order (a global load among them forces vmcnt(0)); nothing
    // issued before the solve may still be pending either (a flat or scratch access of the
    // controller would make the counter out of order too), so drain it first
    __builtin_amdgcn_s_waitcnt(0x70);   // vmcnt(0) lgkmcnt(0)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)wsg, (short)0, (NMAX * NMAX + WAVE) * 8, 0x00020000);
    const double dinv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8, NMAX * NMAX * 8, 0));
    double r = lane_pull((lane < n) ? b : 0.0, perm);   // P b
    const int nu = __builtin_amdgcn_readfirstlane(n);
    tri_sweep_dpp<true, NMAX>(wsg, nu, lane, r, x16);
    r *= dinv;
    tri_sweep_dpp<false, NMAX>(wsg, nu, lane, r, x16);
    return (lane < n) ? r : 0.0;
}

// ------------------------------------------------------------------------------------
// 64 < n <= 72 (CPL = 2): lane holds positions lane and lane + 64. Same factorization semantics
// (first max |a_ik| in original row order, same multipliers and update order). Columns hold
// CR2 = 80 rows (5 lines: positions 64..79 are lanes 0..15 of the second slot; lanes 16..63 there
// never hold a row and never touch memory), not 128 (round 3: 37.5 % fewer bytes per factor and
// J column written). As for CPL = 1 the rows are loaded in the previous factorization's pivot
// order (prow: position -> original row), so when every pivot lands on its own position the
// factors are already in step order and the gather pass is skipped. The panels are 16 columns
// wide (registers: 2 x 16 per lane); the inverse permutation, P b and D^-1 go through LDS scratch
// (>= 160 doubles).
// ------------------------------------------------------------------------------------
constexpr int CR2 = 80;

// first max |a| over candidate positions; exact ties go to the lowest ORIGINAL row (prow)
__device__ __forceinline__ int pivot_row2(double v0, bool c0, double v1, bool c1, const int (&prow)[2]) {
    const unsigned long long b0 = (unsigned long long)__double_as_longlong(v0);
    const unsigned long long b1 = (unsigned long long)__double_as_longlong(v1);
    const unsigned h0 = c0 ? (unsigned)(b0 >> 32) : 0u, h1 = c1 ? (unsigned)(b1 >> 32) : 0u;
    const unsigned mh = wave_umax(max(h0, h1));
    bool t0 = c0 && h0 == mh, t1 = c1 && h1 == mh;
    unsigned long long m0 = __ballot(t0), m1 = __ballot(t1);
    if (__builtin_popcountll(m0) + __builtin_popcountll(m1) > 1) {
        const unsigned l0 = t0 ? (unsigned)b0 : 0u, l1 = t1 ? (unsigned)b1 : 0u;
        const unsigned ml = wave_umax(max(l0, l1));
        t0 = t0 && l0 == ml;
        t1 = t1 && l1 == ml;
        m0 = __ballot(t0);
        m1 = __ballot(t1);
        if (__builtin_popcountll(m0) + __builtin_popcountll(m1) > 1) {   // exact tie: lowest original row
            const unsigned k0 = t0 ? ~(unsigned)prow[0] : 0u, k1 = t1 ? ~(unsigned)prow[1] : 0u;
            const unsigned mk = wave_umax(max(k0, k1));
            m0 = __ballot(t0 && k0 == mk);
            m1 = __ballot(t1 && k1 == mk);
        }
    }
    return m0 ? (int)__builtin_ctzll(m0) : (m1 ? 64 + (int)__builtin_ctzll(m1) : 0);
}

template <int W>
__device__ __forceinline__ void lu_rl_steps2(double (&a)[2][W], int k0, int k1, int cend, int lane, int (&pstep)[2],
                                             double (&dinv)[2], int& fail, __amdgpu_buffer_rsrc_t rs, const int (&prow)[2]) {
    constexpr int CH = 8;
    static_assert(W % CH == 0, "W must be a multiple of 8");
    // the second slot's lanes 16..63 (positions 80..127, never rows) all address row 79: every
    // value they hold or write there is 0 (padding rows), so no memory op needs an exec mask;
    // factor stores as raw buffer ops (column base in soffset)
    const unsigned fo8[2] = {(unsigned)lane * 8u, (unsigned)min(64 + lane, CR2 - 1) * 8u};
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const int pr = pivot_row2(fabs(a[0][0]), pstep[0] < 0, fabs(a[1][0]), pstep[1] < 0, prow);
        const int p = pr & 63, ps = pr >> 6;
        const double piv = ps ? bcast(a[1][0], p) : bcast(a[0][0], p);
        if (piv == 0.0 && !fail) fail = k + 1;
        const double rinv = 1.0 / piv;
        double l[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const bool isp = (ps == s) && (lane == p);
            const bool rem = (pstep[s] < 0) && !isp;
            l[s] = rem ? a[s][0] * rinv : 0.0;
            const double fv = rem ? l[s] : ((pstep[s] >= 0) ? a[s][0] * dinv[s] : 0.0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, fv), rs, fo8[s], k * (CR2 * 8), 0);
            if (isp) { pstep[s] = k; dinv[s] = rinv; }
        }
        const int live = cend - k;
        auto upd = [&](auto S) {
            constexpr int src = decltype(S)::value;
#pragma unroll
            for (int c = 0; c < W; c += CH) {
                if (c < live) {
#pragma unroll
                    for (int i = 0; i < CH; ++i) {
                        const int j = c + i;
                        if (j + 1 < W) {
                            const double u = bcast_lu(a[src][j + 1], p);
                            a[0][j] = fma(-u, l[0], a[0][j + 1]);
                            a[1][j] = fma(-u, l[1], a[1][j + 1]);
                        } else {
                            a[0][j] = 0.0;
                            a[1][j] = 0.0;
                        }
                    }
                }
            }
        };
        if (ps) upd(std::integral_constant<int, 1>{});
        else upd(std::integral_constant<int, 0>{});
    }
}

// one 16-column panel starting at column C0: load (rows in prow order), left-looking updates by
// steps 0..C0-1 (multipliers from M in position order, masked to positions not yet pivoted at
// that step), right-looking factorization of its own columns; then the next panel
template <int NMAX, int C0>
__device__ __forceinline__ void lu2_panels(__amdgpu_buffer_rsrc_t rj, double gamma, int n, int lane, int (&pstep)[2],
                                           double (&dinv)[2], int& fail, __amdgpu_buffer_rsrc_t rs, const int (&prow)[2]) {
    if constexpr (C0 < NMAX) {
        constexpr int W = (NMAX - C0) < 16 ? (NMAX - C0) : 16;
        if (C0 < n) {
            const unsigned fo8[2] = {(unsigned)lane * 8u, (unsigned)min(64 + lane, CR2 - 1) * 8u};   // (see lu_rl_steps2)
            auto ldf = [&](int s, int col) {
                return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, fo8[s], col * (CR2 * 8), 0));
            };
            double a[2][W];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int row = prow[s];
                // J through a buffer of n columns: rows >= n and columns >= n are out of range (0)
                const unsigned jo8 = (row < n) ? (unsigned)row * 8u : LU_OOB;
#pragma unroll
                for (int j = 0; j < W; ++j) {
                    const int col = C0 + j;
                    const double jv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, jo8 + col * (CR2 * 8), 0, 0));
                    a[s][j] = ((col == row) ? 1.0 : 0.0) - gamma * jv;
                }
            }
            if (C0 > 0) {
                double n0 = ldf(0, 0), n1 = ldf(1, 0);
#pragma unroll 1
                for (int k = 0; k < C0; ++k) {
                    const double m0 = n0, m1 = n1;
                    const int kn = (k + 1 < C0) ? k + 1 : k;
                    n0 = ldf(0, kn);
                    n1 = ldf(1, kn);
                    const unsigned long long b0 = __ballot(pstep[0] == k), b1 = __ballot(pstep[1] == k);
                    const int p = b0 ? (int)__builtin_ctzll(b0) : (int)__builtin_ctzll(b1);
                    const double l0 = ((unsigned)pstep[0] > (unsigned)k) ? m0 : 0.0;
                    const double l1 = ((unsigned)pstep[1] > (unsigned)k) ? m1 : 0.0;
                    auto upd = [&](auto S) {
                        constexpr int src = decltype(S)::value;
#pragma unroll
                        for (int j = 0; j < W; ++j) {
                            const double u = bcast_lu(a[src][j], p);
                            a[0][j] = fma(-u, l0, a[0][j]);
                            a[1][j] = fma(-u, l1, a[1][j]);
                        }
                    };
                    if (b0) upd(std::integral_constant<int, 0>{});
                    else upd(std::integral_constant<int, 1>{});
                }
            }
            const int kend = (C0 + W < n) ? C0 + W : n;
            lu_rl_steps2<W>(a, C0, kend, kend, lane, pstep, dinv, fail, rs, prow);
        }
        lu2_panels<NMAX, C0 + 16>(rj, gamma, n, lane, pstep, dinv, fail, rs, prow);
    }
}

// perm_io[s]: on entry the original row loaded into position lane + 64 s (the previous
// factorization's step -> row map; identity for a reactor's first LU), on return this one's.
template <int NMAX>
__device__ __forceinline__ int lu_factor2(const double* __restrict__ J_, double* __restrict__ ws, LDSd* scr,
                                          double gamma, int n, int lane, int (&perm_io)[2]) {
    constexpr int CH = 4, NC = NMAX / CH;
    static_assert(NMAX % 8 == 0 && NMAX <= CR2 && NMAX > 64, "NMAX");
    const BR_GLOBAL double* J = launder(J_);
    BR_GLOBAL double* wsg = launder(ws);
    const LUWs F{wsg, wsg + NMAX * CR2};
    const __amdgpu_buffer_rsrc_t rs = lu_rsrc(wsg, NMAX * CR2);   // the factor columns M
    lane = launder_v(lane);
    n = launder_s(n);
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc((void*)J, (short)0, n * (CR2 * 8), 0x00020000);
    int pstep[2], prow[2];
    double dinv[2] = {0.0, 0.0};
    int fail = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int pos = lane + 64 * s;
        prow[s] = (pos < n) ? launder_v(perm_io[s]) : pos;
        pstep[s] = (pos < n) ? -1 : 1024;
    }
    lu2_panels<NMAX, 0>(rj, gamma, n, lane, pstep, dinv, fail, rs, prow);
    const int o1 = min(64 + lane, CR2 - 1);   // (see lu_rl_steps2)
    if (__ballot((lane < n && pstep[0] != lane) || (lane + 64 < n && pstep[1] != lane + 64)) == 0) {
        // every pivot on its own position: M is in step order already; D^-1 in step order
        // (columns >= n are not zeroed: lu_solve2 never reads them)
        F.D[lane] = dinv[0];
        F.D[o1] = dinv[1];
        perm_io[0] = prow[0];
        perm_io[1] = prow[1];
        return fail;
    }
    // inverse permutation through LDS: position of step s (positions >= n map to themselves),
    // and the original row / D^-1 of every position
    // (positions >= CR2 are padding and map to themselves, so the tables hold CR2 entries: 160
    // doubles of the scratch)
    LDSi* isc = (LDSi*)scr;            // [CR2] step -> position
    LDSi* rsc = (LDSi*)(scr + 40);     // [CR2] position -> original row
    LDSd* dsc = scr + 80;              // [CR2] position -> D^-1
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int pos = lane + 64 * s;
        if (pos < CR2) {
            isc[(pos < n) ? pstep[s] : pos] = pos;
            rsc[pos] = prow[s];
            dsc[pos] = dinv[s];
        }
    }
    wave_sync();
    int q[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int pos = lane + 64 * s;
        q[s] = (pos < CR2) ? isc[pos] : pos;
        perm_io[s] = (q[s] < CR2) ? rsc[q[s]] : pos;
    }
    F.D[lane] = dsc[q[0]];
    F.D[o1] = (q[1] < CR2) ? dsc[q[1]] : 0.0;
    wave_sync();
    // positions into step order, in place, chunks of CH columns double-buffered (columns >= n: zeros)
    double g[2][2][CH];
    auto gather = [&](double (&v)[2][CH], int c) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int col = (c + i < n) ? c + i : n - 1;
            v[0][i] = F.M[col * CR2 + q[0]];
            v[1][i] = F.M[col * CR2 + min(q[1], CR2 - 1)];
        }
    };
    gather(g[0], 0);
#pragma unroll
    for (int t = 0; t < NC; ++t) {
        if (t + 1 < NC) gather(g[(t + 1) & 1], (t + 1) * CH);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int col = t * CH + i;
            if (col < n) {   // (columns >= n: never read -- the solve's loads of them are out of range)
                F.M[col * CR2 + lane] = g[t & 1][0][i];
                F.M[col * CR2 + o1] = g[t & 1][1][i];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return fail;
}

// Triangular sweeps of the CPL = 2 factors in DPP form (64 < n <= NMAX = 72): r0 holds row lane, r1 row lane + 64
// (lanes 0..NMAX-65 real, the rest of DPP row 0 is zero padding). Column blocks 0..3 are rows 0..63 in r0
// (DPP row b), block 4 = columns 64..NMAX-1 is DPP row 0 of r1. Forward: block b's diagonal part in
// row b of r0, its finished values copied to every row through LDS, then the rows of r0 below it and
// the r1 rows (all below) apply it; block 4 last, inside r1. Backward: block 4 first inside r1, its
// values applied to every r0 row, then blocks 3..0 in r0 (r1 rows are below them: untouched).
// Factor loads: diagonal redirect (the step-ordered matrix is 0 at (k, k) and in every row >= n;
// first-half rows use max/min(row, k); second-half rows that cannot update are sent to k
// (backward) or, forward, clamped into the 128-B line of rows 64..79, whose rows >= n are zero).
// ncol (block 4 only): columns >= ncol (= n) are zero padding; their loads get an out-of-range offset
// and read 0 without touching memory (4.6 KB of the ~60 KB a solve reads at n = 66)
template <bool FWD, int CW, bool LIMIT = false>
__device__ __forceinline__ void tri2_load_blk(double (&v0)[16], double (&v1)[16], __amdgpu_buffer_rsrc_t rs, int c0,
                                              unsigned lane8, unsigned hi8, bool want0, bool want1, int ncol = 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i < CW) {
            const unsigned k8 = (unsigned)(c0 + i) * 8u;
            const int cb = (c0 + i) * CR2 * 8;
            const bool live = !LIMIT || c0 + i < ncol;
            if (want0) {
                const unsigned o0 = live ? (FWD ? max(lane8, k8) : min(lane8, k8)) : LU_OOB;
                v0[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, o0, cb, BR_SOLVE_AUX));
            }
            if (want1) {
                const unsigned o1 = live ? (FWD ? min(max(hi8, k8), 79u * 8u) : min(hi8, k8)) : LU_OOB;
                v1[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, o1, cb, BR_SOLVE_AUX));
            }
        }
    }
}
template <int NMAX>
__device__ __forceinline__ void tri_sweeps2_dpp(__amdgpu_buffer_rsrc_t rs, int lane, double (&r)[2], const double (&dv)[2],
                                                LDSd* x64, int n) {
    static_assert(NMAX > 64 && NMAX <= 72, "CPL = 2 DPP sweeps: 64 < NMAX <= 72");
    constexpr int W1 = NMAX - 64;
    const unsigned lane8 = (unsigned)lane * 8u, hi8 = lane8 + 512u;
    const int xl = lane & 15;
    // slot-0 factors double-buffered (the next block's in flight during this one), slot-1 factors
    // (rows 64..79) loaded at the start of their own block and consumed after its diagonal part:
    // 96 instead of 128 VGPRs of buffers (the kernel's peak; 3 waves/SIMD need <= 168)
    double v0[2][16], v1[16];
    // ---- forward: blocks 0..3 (r0), then block 4 (r1)
    tri2_load_blk<true, 16>(v0[0], v1, rs, 0, lane8, hi8, true, false);
    auto fwd_blk = [&](auto B_) {
        constexpr int B = decltype(B_)::value;
        double (&f0)[16] = v0[B & 1];
        __builtin_amdgcn_sched_barrier(0);
        tri2_load_blk<true, 16>(v0[B & 1], v1, rs, 16 * B, lane8, hi8, false, true);
        if constexpr (B < 3) tri2_load_blk<true, 16>(v0[(B + 1) & 1], v1, rs, 16 * (B + 1), lane8, hi8, true, false);
        __builtin_amdgcn_sched_barrier(0);
        dpp_diag<true, 16, 1 << B, 0>(r[0], f0);
        asm volatile("s_nop 1");
        x64[lane] = r[0];
        wave_sync();
        const double x = x64[16 * B + xl];
        if constexpr (B < 3) dpp_off<true, 16, (0xF << (B + 1)) & 0xF, 0>(r[0], x, f0);
        dpp_off<true, 16, 0x1, 0>(r[1], x, v1);
        wave_sync();
    };
    fwd_blk(std::integral_constant<int, 0>{});
    fwd_blk(std::integral_constant<int, 1>{});
    fwd_blk(std::integral_constant<int, 2>{});
    fwd_blk(std::integral_constant<int, 3>{});
    tri2_load_blk<true, W1, true>(v0[0], v1, rs, 64, lane8, hi8, false, true, n);
    dpp_diag<true, W1, 0x1, 0>(r[1], v1);               // block 4
    asm volatile("s_nop 1");
    r[0] *= dv[0];
    r[1] *= dv[1];
    // ---- backward: block 4 (r1) first, then blocks 3..0 (r0)
    tri2_load_blk<false, W1, true>(v0[0], v1, rs, 64, lane8, hi8, true, true, n);
    __builtin_amdgcn_sched_barrier(0);
    tri2_load_blk<false, 16>(v0[1], v1, rs, 48, lane8, hi8, true, false);
    __builtin_amdgcn_sched_barrier(0);
    dpp_diag<false, W1, 0x1, 0>(r[1], v1);
    asm volatile("s_nop 1");
    x64[lane] = r[1];
    wave_sync();
    {
        const double x = x64[xl];
        dpp_off<false, W1, 0xF, 0>(r[0], x, v0[0]);
    }
    wave_sync();
    auto bwd_blk = [&](auto B_, auto BUF_) {
        constexpr int B = decltype(B_)::value, BUF = decltype(BUF_)::value;
        double (&f0)[16] = v0[BUF];
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (B > 0) tri2_load_blk<false, 16>(v0[BUF ^ 1], v1, rs, 16 * (B - 1), lane8, hi8, true, false);
        __builtin_amdgcn_sched_barrier(0);
        dpp_diag<false, 16, 1 << B, 0>(r[0], f0);
        if constexpr (B > 0) {
            asm volatile("s_nop 1");
            x64[lane] = r[0];
            wave_sync();
            const double x = x64[16 * B + xl];
            dpp_off<false, 16, (1 << B) - 1, 0>(r[0], x, f0);
            wave_sync();
        }
    };
    bwd_blk(std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{});
    bwd_blk(std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{});
    bwd_blk(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    bwd_blk(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    asm volatile("s_nop 1");
}

template <int NMAX>
__device__ __forceinline__ void lu_solve2(const double* __restrict__ ws, LDSd* scr, int n, int lane,
                                          const int (&perm)[2], double (&b)[2]) {
    const BR_GLOBAL double* wsg = launder(ws);
    lane = launder_v(lane);
    LDSd* dsc = scr + 64;   // [CR2] (scr[0..63]: the sweeps' copy row)
#pragma unroll
    for (int s = 0; s < 2; ++s)
        if (lane + 64 * s < CR2) dsc[lane + 64 * s] = (lane + 64 * s < n) ? b[s] : 0.0;
    wave_sync();
    double r[2] = {dsc[perm[0]], (perm[1] < CR2) ? dsc[perm[1]] : 0.0};   // P b
    wave_sync();
    static_assert(NMAX > 64 && NMAX <= 72, "lu_solve2: NMAX");
    // (all solve loads are buffer loads: drain first so the waitcnt pass can count them in order)
    __builtin_amdgcn_s_waitcnt(0x70);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)wsg, (short)0, (NMAX + 1) * CR2 * 8, 0x00020000);
    const double dv[2] = {
        __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8, NMAX * CR2 * 8, 0)),
        __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, min(lane, CR2 - 65) * 8 + 512, NMAX * CR2 * 8, 0))};
    tri_sweeps2_dpp<NMAX>(rs, lane, r, dv, scr, __builtin_amdgcn_readfirstlane(n));
    b[0] = (lane < n) ? r[0] : 0.0;
    b[1] = (lane + 64 < n) ? r[1] : 0.0;
}

}  // namespace brhip
