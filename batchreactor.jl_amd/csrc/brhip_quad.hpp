// brhip_quad.hpp -- FOUR REACTORS PER WAVE integrator for small gas-phase mechanisms (n <= 16
// components, no surface species; e.g. H2/O2, n = 9, the C2 ensemble). Included by brhip.hip after
// the controller: it runs the same CVODE 5.x restatement (begin_step / ctl_post_rhs /
// ctl_post_solve, src/BatchReactor.jl:138-141,:210) with the controller instantiated for 16-lane
// reactor groups (GW = 16).
//
// Why: one reactor per wave leaves 55 of 64 lanes idle for H2/O2 (n = 9, 27 reactions) in the LU
// and solve and pays the ~1k-instruction step controller per reactor; one reactor per lane
// (k_lane) keeps a reactor's whole state in one lane's registers (436 registers, 1 wave/SIMD,
// spills, 2.6 MB of memory traffic per reactor) and runs every controller branch of 64 diverging
// reactors. Here reactor g of a wave sits on the 16-lane DPP row g, lane gl = lane & 15 holds
// component gl: the controller is shared by 4 reactors (4-way divergence), reductions are DPP row
// butterflies, the LU factors live in registers (one row per lane), the solve needs no memory.
//
// Per reactor (LDS): [Ctl | V: NVEC x 16 doubles | species block: conc[0..15], acc[16..31],
// mc[32..63], 1.0 at [64] (the records' pad species SP_ONE = 64) | kd: {kf, kr} per reaction | fod:
// {k0/kinf, log10 Fcent, c, n} per falloff reaction]. Global: the saved Jacobian, 16 x 16
// column-major per reactor slot. Mechanism tables as for the wavefront engine (LDS image).
#pragma once

namespace quad {
constexpr int G = 16;                               // lanes per reactor
constexpr int SP_CONC = 0, SP_ACC = 16, SP_MC = 32, SP_ONE_Q = 64, SP_DOUBLES = 66;
constexpr int MAX_SETS = 32;                        // mc[32..63]
__host__ __device__ inline int vbytes() { return NVEC * G * 8; }
__host__ __device__ inline int block_bytes(int nrg, int nfo) {
    const int b = CTL_BYTES + vbytes() + SP_DOUBLES * 8 + 16 * nrg + 32 * nfo;
    return (b + 15) / 16 * 16;
}
__host__ __device__ inline int kd_off() { return CTL_BYTES + vbytes() + SP_DOUBLES * 8; }
}  // namespace quad

// max of a 32-bit value over each 16-lane DPP row (every lane gets its row's max)
__device__ __forceinline__ unsigned row_umax(unsigned x) {
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

// T-only constants of one group's reactor (init_tconst for the quad layout): {kf, kr} per gas
// reaction into kd, falloff constants into fod; g/RT per species in the acc slots (scratch)
template <int NM>
__device__ __forceinline__ void q_init_tconst(const Tab& tb, double* sp, double* kd, double* fod, double T, int gl) {
    const double lT = log(T);
    double* grt = sp + quad::SP_ACC;
    const int ng = MF(ng), nrg = MF(nrg);
    if (gl == 0) sp[quad::SP_ONE_Q] = 1.0;
    if (gl < ng) {
        const double* c = MF(nasa) + 15 * gl;
        const double* a = (T < c[0]) ? c + 8 : c + 1;
        const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        const double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        grt[gl] = h - s;
    }
    wave_sync();
    const double RT = R_GAS * T;
#pragma unroll 1
    for (int r = gl; r < nrg; r += quad::G) {
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
        kd[2 * r] = kf;
        kd[2 * r + 1] = kr;
        if (gi_tb(info) == 2) {
            const int fi = gi_foidx(info);
            const double* fp = MF(fo_par) + 8 * fi;
            double* fo = fod + 4 * fi;
            fo[0] = fp[0] * exp(fp[1] * lT - fp[2] / T) / kf;
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
    wave_sync();
}

// the mass-action part kf prod(c_f) - kr prod(c_b) of gas reaction r of a group (products in the
// wavefront engine's order; pad slots read conc[SP_ONE_Q] = 1), the reactant / product
// concentrations kept for the Jacobian
__device__ __forceinline__ double q_mass_action(const double* sp, const double* kd, uint32_t w0, uint32_t w1, int r,
                                                double (&cf)[4], double (&cb)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        cf[e] = sp[quad::SP_CONC + sp8(w0, e)];
        cb[e] = sp[quad::SP_CONC + sp8(w1, e)];
    }
    double Pf = (cf[0] * cf[1]) * cf[2], Pb = (cb[0] * cb[1]) * cb[2];
    if (MF(nu4)) { Pf *= cf[3]; Pb *= cb[3]; }
    return kd[2 * r] * Pf - kd[2 * r + 1] * Pb;
}

// residual! (src/BatchReactor.jl:312-376) for a gas-only group: du of component gl; the pressure
// of this evaluation to *p_out (save_data semantics)
template <int NM>
__device__ __forceinline__ double q_rhs(const Tab& tb, double* sp, const double* kd, const double* fod, double T, double u,
                                        int gl, double* p_out) {
    const int n = MF(n), nrg = MF(nrg), nset = MF(nset);
    const double Mk = tb.molwt[gl];
    const double c = gl < n ? u / Mk : 0.0;                         // c_k = u_k / M_k (p x_k / RT)
    sp[quad::SP_CONC + gl] = c;
    sp[quad::SP_ACC + gl] = 0.0;
    const double Ctot = row_sum(c);
    const double p = R_GAS * T * Ctot;
    wave_sync();
    const double* conc = sp + quad::SP_CONC;
#pragma unroll 1
    for (int t = gl; t < nset; t += quad::G) {                      // third-body sums per efficiency set
        const uint32_t w = tb.tbs[t];                                // (pairing as third_body_sets)
        const int b = w & 0xFFFFF, e = b + (int)(w >> 20);
        double s0 = Ctot, s1 = 0.0;
        int i = b;
#pragma unroll 1
        for (; i + 1 < e; i += 2) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            const double2 e1 = *reinterpret_cast<const double2*>(tb.tbe + 16 * (i + 1));
            s0 = fma(e0.y, conc[__double_as_longlong(e0.x) & 0xFFFF], s0);
            s1 = fma(e1.y, conc[__double_as_longlong(e1.x) & 0xFFFF], s1);
        }
        if (i < e) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            s0 = fma(e0.y, conc[__double_as_longlong(e0.x) & 0xFFFF], s0);
        }
        sp[quad::SP_MC + t] = s0 + s1;
    }
    wave_sync();
    double* acc = sp + quad::SP_ACC;
    const bool xm = (MF(conv) & 2) != 0;
#pragma unroll 1
    for (int r = gl; r < nrg; r += quad::G) {                        // reaction r on lane r mod 16
        const auto rr = rx_rec(tb.rx, r);
        const uint4 ra = *reinterpret_cast<const uint4*>(rr.a);
        const uint4 rb = *reinterpret_cast<const uint4*>(rr.b);
        double cf[4], cb[4];
        double D = q_mass_action(sp, kd, ra.x, ra.y, r, cf, cb);
        const int tbk = gi_tb(ra.z);
        if (tbk) {                                                   // as production()'s rate
            const double Mc = sp[quad::SP_MC + gi_tbidx(ra.z)];
            if (tbk == 1) D *= Mc;
            else {
                double fac, dfac;
                falloff<false>(fod + 4 * gi_foidx(ra.z), gi_troe(ra.z) != 0, Mc, fac, dfac);
                D *= fac;
                if (xm) D *= Mc * 1e-6;                              // [M] in mol/cm3
            }
        }
        scatter(acc, rb.x, rb.y, rb.z, rb.w, D);
    }
    wave_sync();
    const double w = acc[gl];
    wave_sync();
    if (gl == 0) *p_out = p;
    return gl < n ? w * Mk : 0.0;                                    // :363-370 (gas only)
}

// Analytic Jacobian d(du)/du of a gas-only group, row gl per lane (jr[j] = J[gl][j]), at the state
// of the RHS just evaluated (its concentrations and third-body sums are still in the species
// block): J[k][j] = M_k / M_j * sum_r nu_kr dq_r/dc_j (same terms as the wavefront engine and the
// oracle's jac_tc: mass-action partial products, third-body / falloff d[M] columns; the M_k / M_j
// factor applied once per entry). Reactions in a uniform loop (every group evaluates reaction r
// for its own state); the sparse partials go to their column through a scalar switch.
template <int NM>
__device__ __forceinline__ void q_jac(const Tab& tb, const double* sp, const double* kd, const double* fod, int gl,
                                      double (&jr)[NM]) {
    const int n = MF(n), nrg = MF(nrg);
    const bool xm = (MF(conv) & 2) != 0;
#pragma unroll
    for (int j = 0; j < NM; ++j) jr[j] = 0.0;
    const unsigned gl8 = (unsigned)gl * 8u;
#pragma unroll 1
    for (int r = 0; r < nrg; ++r) {
        const auto rr = rx_rec(tb.rx, r);
        const uint32_t w0 = uni((int)rr[0]), w1 = uni((int)rr[1]), info = uni((int)rr[2]);
        const uint32_t s0 = uni((int)rr[4]), s1 = uni((int)rr[5]), s2 = uni((int)rr[6]), s3 = uni((int)rr[7]);
        double cf[4], cb[4];
        const double D = q_mass_action(sp, kd, w0, w1, r, cf, cb);
        double pre = 1.0, coefM = 0.0;
        const int tbk = gi_tb(info);
        if (tbk) {
            const double Mc = sp[quad::SP_MC + gi_tbidx(info)];
            if (tbk == 1) { pre = Mc; coefM = 1.0; }
            else {
                double fac, dfac;
                falloff<true>(fod + 4 * gi_foidx(info), gi_troe(info) != 0, Mc, fac, dfac);
                const double xs = xm ? Mc * 1e-6 : 1.0;             // [M] in mol/cm3 (reference)
                pre = fac * xs;
                coefM = dfac * xs + (xm ? fac * 1e-6 : 0.0);
            }
        }
        // this row's net stoichiometric coefficient in reaction r
        const int cnt = (int)(s3 >> 24);
        const uint32_t sw[3] = {s0, s1, s2};
        double nu = 0.0;
#pragma unroll
        for (int e = 0; e < 6; ++e)
            if (e < cnt && sl_off(sw[e >> 1], e & 1) == gl8) nu += (double)sl_nu(s3, e);
        // third-body / falloff: d q / d c_j = D coefM eff_j (all gas species)
        if (gi_tb(info)) {
            const double dm = nu * D * coefM;
            const double* eff = MF(tb_eff) + (size_t)gi_tbidx(info) * MF(n);
#pragma unroll
            for (int j = 0; j < NM; ++j) if (j < n) jr[j] = fma(dm, eff[j], jr[j]);
        }
        // mass-action partials: slot e of the forward (backward) product
        const double kf = kd[2 * r], kr = kd[2 * r + 1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            double pf = kf * pre, pb = -kr * pre;
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2)
                if (e2 != e) { pf *= cf[e2]; pb *= cb[e2]; }
            const int kfs = (int)((w0 >> (8 * e)) & 255), kbs = (int)((w1 >> (8 * e)) & 255);
            const double vf = nu * pf, vb = nu * pb;
#pragma unroll
            for (int j = 0; j < NM; ++j) {
                if (j == kfs) jr[j] += vf;   // (kfs, kbs uniform: scalar branches; pad slot 64 matches no j)
                if (j == kbs) jr[j] += vb;
            }
        }
    }
    const double Mk = tb.molwt[gl];
#pragma unroll
    for (int j = 0; j < NM; ++j) jr[j] = (gl < n && j < n) ? jr[j] * (Mk / tb.molwt[j]) : 0.0;
}

// compile-time loop: f(std::integral_constant<int, K>) for K = B .. E-1
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}
// value of lane K of this lane's 16-lane row (DPP row_newbcast: a VALU move, no LDS crossbar)
template <int K>
__device__ __forceinline__ double row_bcast(double v) { return dppd<0x150 + K>(v); }

// group pivot of step k: the first max |a| (bit patterns: a 32-bit max over the high words, then
// over the low words, then the lowest lane) among candidate lanes of the row; returns that lane
// within the group. SUNDIALS denseGETRF takes the first row of largest |a_ik| in the current
// (already interchanged) row order -- the lane order here.
__device__ __forceinline__ int q_pivot(double a, bool cand, int gl) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(a) & 0x7fffffffffffffffull;
    const unsigned hi = cand ? (unsigned)(bits >> 32) : 0u;
    const unsigned mh = row_umax(hi);
    const bool top = cand && hi == mh;
    const unsigned lo = top ? (unsigned)bits : 0u;
    const unsigned ml = row_umax(lo);
    const bool top2 = top && lo == ml;
    const unsigned key = top2 ? ~(unsigned)gl : 0u;
    return (int)(~row_umax(key));
}

// LU of A = I - gamma J with partial pivoting as SUNDIALS denseGETRF (src/BatchReactor.jl:204-210:
// CVODE's dense linear solver), one row per lane in registers, rows interchanged physically (lane
// = current row position): after the factorization lane s holds row s of the factors (L's
// multipliers in a[k < s], U in a[k >= s]), dinv = 1 / u_ss, and orig = the original row now at
// lane s (the accumulated interchanges, applied to b by q_solve). Interchanges are bpermutes of the
// two rows' registers, issued only when some group of the wave needs one; the pivot row's values
// reach the row by DPP row broadcasts. Returns 0 or k+1 (zero pivot at step k, as denseGETRF).
template <int NM>
__device__ __forceinline__ int q_lu(const double (&jr)[NM], double gamma, int n, int gl, double (&a)[NM], int& orig,
                                    double& dinv) {
    const int gb = (int)(threadIdx.x & 48);
#pragma unroll
    for (int j = 0; j < NM; ++j) a[j] = ((j == gl && gl < n) ? 1.0 : 0.0) - gamma * jr[j];
    orig = gl;
    dinv = 0.0;
    int fail = 0;
    sfor<0, NM>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < n) {
            const int p = q_pivot(a[k], gl >= k && gl < n, gl);
            if (__ballot(p != k) != 0) {                           // interchange rows k and p
                const int src = gb + (gl == k ? p : (gl == p ? k : gl));
#pragma unroll
                for (int j = 0; j < NM; ++j) a[j] = lane_pull(a[j], src);
                orig = __builtin_amdgcn_ds_bpermute(src * 4, orig);
            }
            const double pv = row_bcast<k>(a[k]);
            if (pv == 0.0 && fail == 0) fail = k + 1;
            const double rinv = 1.0 / pv;
            const bool below = gl > k;
            const double l = below ? a[k] * rinv : 0.0;                // denseGETRF: a_ik *= 1 / a_kk
            if (below) a[k] = l;
            if (gl == k) dinv = rinv;
#pragma unroll
            for (int j = k + 1; j < NM; ++j)
                if (j < n) a[j] = fma(-row_bcast<k>(a[j]), l, a[j]);
        }
    });
    return fail;
}

// solve (I - gamma J) x = b with q_lu's factors (denseGETRS): b interchanged (P b: one bpermute),
// forward with the unit L, backward with U; each step's pivot value reaches the row by a DPP
// broadcast from the compile-time lane k. b and x in component order (lane gl).
template <int NM>
__device__ __forceinline__ double q_solve(const double (&a)[NM], int orig, double dinv, int n, int gl, double b) {
    const int gb = (int)(threadIdx.x & 48);
    double y = lane_pull(gl < n ? b : 0.0, gb + orig);
    sfor<0, NM>([&](auto kc) {                                        // L y = P b
        constexpr int k = decltype(kc)::value;
        if (k + 1 < n) {
            const double yk = row_bcast<k>(y);
            y = fma(-((gl > k) ? a[k] : 0.0), yk, y);
        }
    });
    double x = 0.0;
    sfor<0, NM>([&](auto kc) {                                        // U x = y, k = n-1 .. 0
        constexpr int k = NM - 1 - decltype(kc)::value;
        if (k < n) {
            if (gl == k) x = y * dinv;
            const double xk = row_bcast<k>(x);
            y = fma(-((gl < k) ? a[k] : 0.0), xk, y);
        }
    });
    return gl < n ? x : 0.0;
}

// the controller entry points for 16-lane groups (BR_QCTL_NOINLINE: out of line, so their register
// allocation is separate from the hot loop's)
#ifndef BR_QCTL_NOINLINE
#define BR_QCTL_NOINLINE 0
#endif
#if BR_QCTL_NOINLINE
#define BR_QCTL_ATTR __noinline__
#else
#define BR_QCTL_ATTR __forceinline__
#endif
__device__ BR_QCTL_ATTR int q_post_rhs(LCtl* C, VT<1, 16>& V, int gl, const double (&f)[1], double (&b)[1]) {
    return ctl_post_rhs<1, 16>(C, V, gl, f, b);
}
__device__ BR_QCTL_ATTR int q_post_solve(LCtl* C, VT<1, 16>& V, int gl, double (&delta)[1], int lu_fail) {
    return ctl_post_solve<1, 16>(C, V, gl, delta, lu_fail);
}

#ifndef BR_QWPB
#define BR_QWPB 4   // waves per workgroup (16 reactors); tables staged once per workgroup
#endif
#ifndef BR_QWPE
#define BR_QWPE 3   // waves per SIMD the register allocation targets (<= 168 VGPRs)
#endif

// the quad integrator kernel: persistent grid, every group takes reactor indices from o.work
template <int NM>
__global__ __launch_bounds__(64 * BR_QWPB) __attribute__((amdgpu_waves_per_eu(BR_QWPE))) void k_quad(DevMech M, int N, const double* __restrict__ Tv,
                                                        double* __restrict__ U, const double* __restrict__ tfv, KOpts o,
                                                        double* __restrict__ stats, double* __restrict__ Jws) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    stage_tables(M, smem_raw);
    const Tab tb = tab_view<1>(smem_raw, M);
    const int lane = threadIdx.x & 63, gl = lane & 15;
    const int grp = (int)(threadIdx.x >> 4);                          // group within the workgroup
    const int slot = blockIdx.x * (BR_QWPB * 4) + grp;                // workspace slot of this group
    const int RB = quad::block_bytes(MF(nrg), MF(nfo));
    char* rbase = smem_raw + M.img_bytes + (size_t)grp * RB;
    LCtl* C = (LCtl*)rbase;
    VA<1, quad::G> V{(LDbl*)(rbase + CTL_BYTES), gl};
    double* sp = reinterpret_cast<double*>(rbase + CTL_BYTES + quad::vbytes());
    double* kd = reinterpret_cast<double*>(rbase + quad::kd_off());
    double* fod = kd + 2 * MF(nrg);
    BR_GLOBAL double* Jq = launder(Jws) + (size_t)slot * (quad::G * quad::G);
    const int n = MF(n);
    double* p_last = reinterpret_cast<double*>(rbase);                // Ctl::p_last is the first field
    // this group's reactor: the first one from the work counter
    auto take = [&]() -> int {
        int v = 0;
        if (gl == 0) v = atomicAdd(o.work, 1);
        return __builtin_amdgcn_ds_bpermute((int)(threadIdx.x & 48) * 4, v);
    };
    int rid = take();
    double T = 0.0;
    bool fresh = true;
    int dqj = -1;   // >= 0: building column dqj of the DQ Jacobian
    double a[NM];
    int orig = gl;
    double dinv = 0.0;
#pragma unroll
    for (int j = 0; j < NM; ++j) a[j] = 0.0;
    unsigned long long cyc0 = 0;
#if BR_PHASE_CLOCKS   // diagnostic build: this group's shader clocks per phase (br_stats cyc_*)
    unsigned long long q_rhs_c = 0, q_jac_c = 0, q_lu_c = 0, q_sol_c = 0, q_ctl_c = 0, q_all = 0;
#define QCLK(v) const unsigned long long v = clock64()
#define QACC(acc, v) acc += clock64() - v
#else
#define QCLK(v)
#define QACC(acc, v)
#endif
    for (;;) {
        if (__ballot(rid < N) == 0) break;
        if (rid < N) {
            if (fresh) {                                              // ---- CVodeInit for reactor rid
                fresh = false;
                cyc0 = wall_clock64();
#if BR_PHASE_CLOCKS
                q_rhs_c = q_jac_c = q_lu_c = q_sol_c = q_ctl_c = 0;
                q_all = clock64();
#endif
                T = Tv[rid];
                C->a_rtol = o.rtol; C->a_atol = o.atol; C->a_hmax_inv = o.hmax_inv; C->a_ufac = o.ufac;
                C->a_max_steps = o.max_steps; C->a_trace_cap = 0; C->a_trace = nullptr; C->a_rid = rid; C->a_n = n;
                C->a_ign = o.ign; C->a_nout = o.nout; C->a_tout = o.tout; C->a_yout = o.yout;
                q_init_tconst<NM>(tb, sp, kd, fod, T, gl);
                const bool act = gl < n;
                const double u0 = act ? U[(size_t)rid * n + gl] : 0.0;
#pragma unroll
                for (int j = 0; j < NVEC; ++j) V.at(j, 0) = 0.0;
                V.at(0, 0) = u0;
                V.at(V_Y, 0) = u0;
                V.at(V_EWT, 0) = act ? 1.0 / (o.rtol * fabs(u0) + o.atol) : 1.0;
                const double su = row_sum(act ? fabs(u0) : 0.0);
#pragma unroll
                for (int i = 0; i < QMAX + 2; ++i) C->tau[i] = 0.0;
#pragma unroll
                for (int i = 0; i < 6; ++i) C->tq[i] = 0.0;
#pragma unroll
                for (int i = 0; i <= QMAX; ++i) C->l[i] = 0.0;
                C->tn = 0.0; C->h = 0.0; C->rl1 = 0.0; C->gamma = 0.0; C->gamrat = 1.0; C->gammap = 0.0; C->crate = 1.0;
                C->delp = 0.0; C->hprime = 0.0; C->hscale = 0.0; C->eta = 1.0; C->etamax = ETAMX1; C->acnrm = 0.0;
                C->saved_tq5 = 0.0; C->saved_t = 0.0; C->tol = 0.0; C->hg = 0.0; C->hub = 0.0; C->hlb = 0.0; C->hnew = 0.0;
                C->tstop = tfv[rid];
                C->ulimit = o.ufac > 0.0 ? o.ufac * su : INFINITY;
                C->q = 1; C->qprime = 1; C->L = 2; C->qwait = 2;
                C->nst = 0; C->nfe = 0; C->nsetups = 0; C->nje = 0; C->nni = 0; C->ncfn = 0; C->netf = 0; C->nstlp = 0;
                C->nstlj = 0; C->ncf = 0; C->nef = 0; C->nstloc = 0; C->status = 0; C->m_it = 0; C->convfail = 0;
                C->count1 = 0; C->phase = PH_F0; C->callSetup = 0; C->jbad = 0; C->jcur_nls = 0; C->hnewOK = 0;
                C->newj = 0; C->p_last = 0.0;
                C->iout = 0; C->ign_t = 0.0; C->ign_rate = -INFINITY; C->t_ign = NAN; C->ign_x = 0.0; C->ign_dt = NAN;
                C->dq_mininc = 1.0; C->nfe_dq = 0;
                if (o.ign >= 0) {
                    double uv[1] = {u0};
                    C->ign_x = mole_frac_of<1, quad::G>(uv, gl, o.ign);
                }
                if (o.nout) {                                         // outputs at t <= 0: the initial state
                    int io = 0;
                    while (io < o.nout && !(o.tout[io] > 0.0)) {
                        if (act) o.yout[((size_t)rid * o.nout + io) * n + gl] = u0;
                        ++io;
                    }
                    C->iout = io;
                }
                wave_sync();
            }
            // ---- one RHS for this group's reactor, then its controller. dqj >= 0: this RHS is at
            // y + inc_dqj e_dqj, column dqj of CVODE's DQ Jacobian (cvLsDenseDQJac, k_integrate's
            // dq_* steps with 16-lane groups)
            double yv = V.at(V_Y, 0);
            if (dqj >= 0) {
                double inc[1];
                dq_incs<1, quad::G>(C, V, gl, inc);
                if (gl == dqj) yv += inc[0];
            }
            QCLK(c_r);
            const double fv = q_rhs<NM>(tb, sp, kd, fod, T, yv, gl, p_last);
            QACC(q_rhs_c, c_r);
            double f[1] = {fv}, b[1];
            int act_code;
            bool jac_ready = false;
            QCLK(c_c);
            if (dqj >= 0) {
                double inc[1];
                dq_incs<1, quad::G>(C, V, gl, inc);
                const double ii = 1.0 / gbcast<quad::G>(inc[0], dqj);
                Jq[dqj * quad::G + gl] = ii * fv - ii * V.at(V_TEMP, 0);
                C->nfe_dq = C->nfe_dq + 1;
                if (++dqj < n) {
                    act_code = A_RHS;
                } else {
                    dqj = -1;
                    dq_newton_rhs<1, quad::G>(C, V, gl, b);
                    act_code = A_SETUP;
                    jac_ready = true;
                }
            } else {
                act_code = q_post_rhs(C, V, gl, f, b);
                if (act_code == A_SETUP && o.dq_jac && C->newj) {
                    dq_begin<1, quad::G>(C, V, gl, f);
                    dqj = 0;
                    act_code = A_RHS;
                }
            }
            QACC(q_ctl_c, c_c);
            int lu_fail = 0;
            if (act_code == A_SETUP) {
                if (!jac_ready && C->newj) {                          // analytic Jacobian at y, saved
                    QCLK(c_j);
                    double jr[NM];
                    q_jac<NM>(tb, sp, kd, fod, gl, jr);
#pragma unroll
                    for (int j = 0; j < NM; ++j) Jq[j * quad::G + gl] = jr[j];
                    QACC(q_jac_c, c_j);
                }
                QCLK(c_l);
                double jr[NM];
#pragma unroll
                for (int j = 0; j < NM; ++j) jr[j] = Jq[j * quad::G + gl];
                lu_fail = q_lu<NM>(jr, C->gamma, n, gl, a, orig, dinv);
                QACC(q_lu_c, c_l);
            }
            if (act_code == A_SOLVE || act_code == A_SETUP) {
                QCLK(c_s);
                double delta[1] = {0.0};
                if (!lu_fail) delta[0] = q_solve<NM>(a, orig, dinv, n, gl, b[0]);
                QACC(q_sol_c, c_s);
                QCLK(c_p);
                act_code = q_post_solve(C, V, gl, delta, lu_fail);
                QACC(q_ctl_c, c_p);
            }
            if (act_code == A_DONE) {                                 // ---- results, next reactor
                const int status = C->status;
                const double u_out = status ? V.at(0, 0) : V.at(V_Y, 0);
                if (gl < n) U[(size_t)rid * n + gl] = u_out;
                if (stats && gl == 0) {
                    double* st = stats + (size_t)rid * BR_NSTAT;
                    st[0] = C->nst; st[1] = C->nfe; st[2] = C->nje; st[3] = C->nsetups; st[4] = C->nni;
                    st[5] = C->ncfn; st[6] = C->netf; st[7] = (double)status;
                    st[8] = (double)(wall_clock64() - cyc0);
#if BR_PHASE_CLOCKS
                    st[9] = (double)q_rhs_c; st[10] = (double)q_jac_c; st[11] = (double)q_lu_c; st[12] = (double)q_sol_c;
                    st[14] = (double)q_ctl_c; st[15] = (double)(clock64() - q_all);
#else
                    st[9] = st[10] = st[11] = st[12] = st[14] = st[15] = 0.0;
#endif
                    st[13] = C->tn;
                    st[16] = o.ign >= 0 ? (double)C->t_ign : NAN; st[17] = o.ign >= 0 ? (double)C->ign_rate : NAN;
                    st[18] = o.ign >= 0 ? (double)C->ign_dt : NAN; st[19] = C->nfe_dq;
                }
                rid = take();
                fresh = true;
            }
        }
    }
}
