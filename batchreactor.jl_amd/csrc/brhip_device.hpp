// brhip_device.hpp -- device side of libbrhip.so (gfx950, fp64).
//
// Execution model: ONE REACTOR PER WAVEFRONT (64 lanes), several reactors (waves) per
// workgroup; lane k <-> solution component k (gas species 0..ng-1, then surface coverages).
//  * The compact mechanism tables (reaction species packs, production CSR, third-body
//    efficiencies) are staged ONCE PER WORKGROUP into LDS and shared by its waves.
//  * T-dependent rate constants live in a per-reactor LDS block (T is a per-reactor
//    constant: ConstantParams, src/BatchReactor.jl:14-17), as does the BDF controller state.
//  * Reactions are evaluated lane-parallel (reaction r on lane r mod 64) and accumulated
//    into the species production sums with fp64 LDS atomics (ds_add_f64, wave-private).
//  * Reductions are DPP row reductions + 4 v_readlane (no LDS round trips).
//  * The Newton matrix I - gamma*J is factored ROW-PER-LANE in registers (a[NMAX]); the
//    pivot row of each LU step is found by a DPP argmax and broadcast with v_readlane; no row
//    swaps; the pivot order is recovered with a ballot. J and the LU factors are kept in a
//    per-reactor HBM workspace (coalesced [column][lane]) so the step loop's register file
//    stays small.
// Waves of one workgroup never synchronise with each other after the table staging.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace brhip {

constexpr double R_GAS = 8.31446261815324;   // RxnHelperUtils.R (src/BatchReactor.jl:338)
constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------
// mechanism description (global memory pointers) and the LDS table layout
// ------------------------------------------------------------------------------------
struct DevMech {
    int ng, ns, n, nrg, nrs, nr, conv;
    int ntb, nfo, ntbe;
    double p_std, G;              // Pa ; site density mol/m2
    // words staged to LDS (uint32): [rx_sp nrg][rx_pr nrg][rx_info nrg][sx_sp 2*nrs][sx_pr 2*nrs]
    // [sx_info nrs][tb_ptr ntb+1][tb_sp ntbe]  then doubles [tb_de ntbe]
    const uint32_t* tab;          // packed words
    int tab_words;                // number of uint32 words (16-byte multiple)
    const double* tab_d;          // tb_de
    // global-only (init / Jacobian)
    const double* molwt;          // [n] (1 for surface)
    const double* sigma;          // [n] (1 for gas)
    const double* nasa;           // [ng*15]
    const double* g_arr;          // [3][nrg]
    const double* g_kcs;          // [nrg]
    const int* g_dnu;             // [nrg]
    const double* fo_low;         // [3][nfo]
    const double* fo_troe;        // [4][nfo]
    const int* fo_ntroe;          // [nfo]
    const double* tb_eff;         // [ntb][n] dense (Jacobian)
    const double* s_arr;          // [3][nrs]
    const uint32_t* s_cov_sp;     // [nrs] 4 x 8-bit species
    const double* s_cov_eps;      // [4][nrs]
    const int* col_ptr;           // [n+1] Jacobian column lists
    const int* col_rx;            // combined reaction index (gas r, surface nrg+r)
};

// rx_info bit fields
__host__ __device__ inline int gi_nf(uint32_t v) { return v & 7; }
__host__ __device__ inline int gi_nr(uint32_t v) { return (v >> 3) & 7; }
__host__ __device__ inline int gi_rev(uint32_t v) { return (v >> 6) & 1; }
__host__ __device__ inline int gi_tb(uint32_t v) { return (v >> 7) & 3; }
__host__ __device__ inline int gi_tbidx(uint32_t v) { return (v >> 9) & 1023; }
__host__ __device__ inline int gi_foidx(uint32_t v) { return (v >> 19) & 1023; }
// sx_info bit fields
__host__ __device__ inline int si_nf(uint32_t v) { return v & 7; }
__host__ __device__ inline int si_np(uint32_t v) { return (v >> 3) & 7; }
__host__ __device__ inline int si_stick(uint32_t v) { return (v >> 6) & 1; }
__host__ __device__ inline int si_ncov(uint32_t v) { return (v >> 7) & 7; }
__host__ __device__ inline int si_gas(uint32_t v) { return (v >> 10) & 255; }
__host__ __device__ inline int sp8(uint32_t w, int e) { return (w >> (8 * e)) & 255; }

struct Tab {   // LDS views
    const uint32_t *rx_sp, *rx_pr, *rx_info, *rx_sc, *sx_sp, *sx_pr, *sx_info, *sx_sc, *tb_ptr, *tb_sp;
    const double* tb_de;
};

__host__ __device__ inline int tab_words(int nrg, int nrs, int ntb, int ntbe) {
    int w = 6 * nrg + 8 * nrs + (ntb + 1) + ntbe;
    return (w + 3) & ~3;   // 16-byte multiple
}
__device__ __forceinline__ Tab tab_view(const uint32_t* base, const DevMech& M) {
    Tab t;
    const uint32_t* p = base;
    t.rx_sp = p; p += M.nrg;
    t.rx_pr = p; p += M.nrg;
    t.rx_info = p; p += M.nrg;
    t.rx_sc = p; p += 3 * M.nrg;
    t.sx_sp = p; p += 2 * M.nrs;
    t.sx_pr = p; p += 2 * M.nrs;
    t.sx_info = p; p += M.nrs;
    t.sx_sc = p; p += 3 * M.nrs;
    t.tb_ptr = p; p += M.ntb + 1;
    t.tb_sp = p;
    t.tb_de = reinterpret_cast<const double*>(base + M.tab_words);
    return t;
}
__host__ __device__ inline size_t tab_bytes(const DevMech& M) {
    return ((size_t)M.tab_words * 4 + (size_t)M.ntbe * 8 + 15) & ~(size_t)15;
}

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
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ double bcast(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double uni(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// quad_perm[1,0,3,2]=0xB1, quad_perm[2,3,0,1]=0x4E, row_half_mirror=0x141, row_mirror=0x140:
// each step pairs lane i with a partner that pairs back with i, so both compute the same value.
__device__ __forceinline__ double wave_sum(double v) {
    v += dppd<0xB1>(v);
    v += dppd<0x4E>(v);
    v += dppd<0x141>(v);
    v += dppd<0x140>(v);
    return (bcast(v, 0) + bcast(v, 16)) + (bcast(v, 32) + bcast(v, 48));
}
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dppd<0xB1>(v));
    v = fmax(v, dppd<0x4E>(v));
    v = fmax(v, dppd<0x141>(v));
    v = fmax(v, dppd<0x140>(v));
    return fmax(fmax(bcast(v, 0), bcast(v, 16)), fmax(bcast(v, 32), bcast(v, 48)));
}
template <int CTRL>
__device__ __forceinline__ void argmax_step(double& v, int& i) {
    const double ov = dppd<CTRL>(v);
    const int oi = dppi<CTRL>(i);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}
// lane of the largest v (lowest lane on ties); uniform
__device__ __forceinline__ int wave_argmax(double v) {
    int i = (int)threadIdx.x & 63;
    argmax_step<0xB1>(v, i);
    argmax_step<0x4E>(v, i);
    argmax_step<0x141>(v, i);
    argmax_step<0x140>(v, i);
    double bv = bcast(v, 0);
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double rv = bcast(v, r);
        const int ri = __builtin_amdgcn_readlane(i, r);
        if (rv > bv || (rv == bv && ri < bi)) { bv = rv; bi = ri; }
    }
    return uni(bi);
}

// ------------------------------------------------------------------------------------
// per-reactor LDS workspace
// ------------------------------------------------------------------------------------
struct Smem {
    double* kf;    // [nrg]
    double* kr;    // [nrg]
    double* jpre;  // [nrg]  Jacobian: multiplier of dD
    double* jdm;   // [nrg]  Jacobian: D * d(pre)/d[M]
    double* accw;  // [max(n, ng)] production by gas reactions (also g/RT scratch at init)
    double* accs;  // [n]    production by surface reactions
    double* ks;    // [nrs]
    double* sk;    // [nrs]
    double* k0;    // [nfo]
    double* lfc;   // [nfo]  log10(Fcent)
    double* tcc;   // [nfo]  Troe c
    double* tnn;   // [nfo]  Troe n
    double* conc;  // [n]    gas concentrations (mol/m3) then coverages
    double* mc;    // [ntb]
};

__host__ __device__ inline int accw_len(int n, int ng) { return n > ng ? n : ng; }
__host__ __device__ inline size_t reactor_doubles(const DevMech& M) {
    size_t d = (size_t)4 * M.nrg + accw_len(M.n, M.ng) + M.n + 2 * (size_t)M.nrs + 4 * (size_t)M.nfo + M.n + M.ntb;
    return (d + 1) & ~(size_t)1;   // 16-byte multiple
}
__device__ __forceinline__ Smem carve(double* p, const DevMech& M) {
    Smem s;
    s.kf = p; p += M.nrg;
    s.kr = p; p += M.nrg;
    s.jpre = p; p += M.nrg;
    s.jdm = p; p += M.nrg;
    s.accw = p; p += accw_len(M.n, M.ng);
    s.accs = p; p += M.n;
    s.ks = p; p += M.nrs;
    s.sk = p; p += M.nrs;
    s.k0 = p; p += M.nfo;
    s.lfc = p; p += M.nfo;
    s.tcc = p; p += M.nfo;
    s.tnn = p; p += M.nfo;
    s.conc = p; p += M.n;
    s.mc = p;
    return s;
}

// fp64 LDS accumulate, relaxed, wavefront scope (ds_add_f64; deterministic inside one wave)
__device__ __forceinline__ void lds_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// acc[k] += nu_k * v over a reaction's net-stoichiometry scatter list (3 packed words)
__device__ __forceinline__ void scatter(double* acc, const uint32_t* sc, double v) {
    const uint32_t w0 = sc[0], w1 = sc[1], w2 = sc[2];
    const int cnt = (w1 >> 16) & 255;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        if (e < cnt) {
            const int k = e < 4 ? sp8(w0, e) : sp8(w1, e - 4);
            const int nu = ((int)(w2 << (28 - 4 * e))) >> 28;   // sign-extended nibble
            lds_add(&acc[k], nu == 1 ? v : (nu == -1 ? -v : nu * v));
        }
    }
}

// stage the packed tables (all threads of the workgroup), then barrier
__device__ __forceinline__ void stage_tables(const DevMech& M, uint32_t* dst) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int i = t; i < M.tab_words; i += nt) dst[i] = M.tab[i];
    double* dd = reinterpret_cast<double*>(dst + M.tab_words);
    for (int i = t; i < M.ntbe; i += nt) dd[i] = M.tab_d[i];
    __syncthreads();
}

// T-only constants (src/BatchReactor.jl:14-17: T is a per-reactor constant)
__device__ __forceinline__ void init_tconst(const DevMech& M, const Tab& tb, Smem& S, double T, int lane) {
    const double lT = log(T);
    for (int k = lane; k < M.ng; k += WAVE) {   // g/RT per species into qb (scratch)
        const double* c = M.nasa + 15 * k;
        const double* a = (T < c[0]) ? c + 8 : c + 1;
        const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        const double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        S.accw[k] = h - s;
    }
    wave_sync();
    const double RT = R_GAS * T;
    for (int r = lane; r < M.nrg; r += WAVE) {
        const uint32_t info = tb.rx_info[r];
        const double A = M.g_arr[r], b = M.g_arr[M.nrg + r], EoR = M.g_arr[2 * M.nrg + r];
        const double kf = A * exp(b * lT - EoR / T);
        double kr = 0.0;
        if (gi_rev(info)) {
            double dg = 0.0;
            const int nf = gi_nf(info), nr = gi_nr(info);
            const uint32_t fw = tb.rx_sp[r], rw = tb.rx_pr[r];
            for (int e = 0; e < 4; ++e) if (e < nr) dg += S.accw[sp8(rw, e)];
            for (int e = 0; e < 4; ++e) if (e < nf) dg -= S.accw[sp8(fw, e)];
            double Kc = exp(-dg) * pow(M.p_std / RT, (double)M.g_dnu[r]);
            Kc *= M.g_kcs[r];
            kr = kf / Kc;
        }
        S.kf[r] = kf;
        S.kr[r] = kr;
        if (gi_tb(info) == 2) {
            const int fi = gi_foidx(info);
            const double A0 = M.fo_low[fi], b0 = M.fo_low[M.nfo + fi], E0 = M.fo_low[2 * M.nfo + fi];
            S.k0[fi] = A0 * exp(b0 * lT - E0 / T);
            double fcv = 1.0;
            if (M.fo_ntroe[fi]) {
                const double ta = M.fo_troe[fi], t3 = M.fo_troe[M.nfo + fi], t1 = M.fo_troe[2 * M.nfo + fi];
                const double t2 = M.fo_troe[3 * M.nfo + fi];
                fcv = (1 - ta) * exp(-T / t3) + ta * exp(-T / t1);
                if (M.fo_ntroe[fi] == 4) fcv += exp(-t2 / T);
            }
            const double lfc = log10(fcv);
            S.lfc[fi] = lfc;
            S.tcc[fi] = -0.4 - 0.67 * lfc;
            S.tnn[fi] = 0.75 - 1.27 * lfc;
        }
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const uint32_t info = tb.sx_info[r];
        const double A = M.s_arr[r], b = M.s_arr[M.nrs + r], Ea = M.s_arr[2 * M.nrs + r];
        double k;
        if (si_stick(info)) k = A * sqrt(RT / (2 * M_PI * M.molwt[si_gas(info)]));
        else k = A * pow(T, b) * exp(-Ea / RT);
        S.ks[r] = k;
    }
    wave_sync();
}

// falloff: fac = Pr/(1+Pr)*F and d fac / d[M]
template <bool WANT_D>
__device__ __forceinline__ void falloff(const DevMech& M, const Smem& S, int r, int fi, double Mc, double& fac,
                                        double& dfac) {
    const double kinf = S.kf[r], k0 = S.k0[fi];
    const double Pr = k0 * Mc / kinf;
    double F = 1.0, g = 0.0;
    if (M.fo_ntroe[fi]) {
        const double Prs = Pr > 1e-300 ? Pr : 1e-300;
        const double lfc = S.lfc[fi];
        const double L = log10(Prs);
        const double cc = S.tcc[fi], nn = S.tnn[fi];
        const double den = nn - 0.14 * (L + cc);
        const double f1 = (L + cc) / den;
        const double lF = lfc / (1 + f1 * f1);
        F = pow(10.0, lF);
        if (WANT_D) {
            const double df1 = nn / (den * den);
            g = -lfc * 2 * f1 / ((1 + f1 * f1) * (1 + f1 * f1)) * df1;
        }
    }
    fac = Pr / (1 + Pr) * F;
    if (WANT_D) dfac = (F / ((1 + Pr) * (1 + Pr)) + F * g / (1 + Pr)) * (k0 / kinf);
}

// third-body concentrations [M]_t = Ctot + sum (eff-1) c   (conc in S.conc)
__device__ __forceinline__ void third_body(const DevMech& M, const Tab& tb, Smem& S, double Ctot, int lane) {
    for (int t = lane; t < M.ntb; t += WAVE) {
        double s = Ctot;
        const int e = tb.tb_ptr[t + 1];
        for (int i = tb.tb_ptr[t]; i < e; ++i) s += tb.tb_de[i] * S.conc[tb.tb_sp[i]];
        S.mc[t] = s;
    }
}

// rates of progress, accumulated straight into the per-species production sums:
// accw[k] += nu_kr q_r (gas reactions), accs[k] += nu_kr q_r (surface reactions)
__device__ __forceinline__ void production(const DevMech& M, const Tab& tb, Smem& S, double RT, int lane) {
    const bool xm = (M.conv & 2) != 0;
    for (int r = lane; r < M.nrg; r += WAVE) {
        const uint32_t info = tb.rx_info[r], fw = tb.rx_sp[r], rw = tb.rx_pr[r];
        const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
        double Pf = 1.0, Pb = 1.0;
#pragma unroll
        for (int e = 0; e < 4; ++e) if (e < nf) Pf *= S.conc[sp8(fw, e)];
#pragma unroll
        for (int e = 0; e < 4; ++e) if (e < nr) Pb *= S.conc[sp8(rw, e)];
        double D = S.kf[r] * Pf - S.kr[r] * Pb;
        if (tbk == 1) D *= S.mc[gi_tbidx(info)];
        else if (tbk == 2) {
            const double Mc = S.mc[gi_tbidx(info)];
            double fac, dfac;
            falloff<false>(M, S, r, gi_foidx(info), Mc, fac, dfac);
            D *= fac;
            if (xm) D *= Mc;
        }
        scatter(S.accw, tb.rx_sc + 3 * r, D);
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const uint32_t info = tb.sx_info[r];
        const int nf = si_nf(info), np = si_np(info), nc = si_ncov(info);
        const bool stick = si_stick(info);
        double k = S.ks[r];
        if (nc) {
            const uint32_t cs = M.s_cov_sp[r];
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += M.s_cov_eps[j * M.nrs + r] * S.conc[sp8(cs, j)];
            k *= exp(-s / RT);
        }
        double P = 1.0;
        const uint32_t w0 = tb.sx_sp[2 * r], w1 = tb.sx_sp[2 * r + 1];
#pragma unroll
        for (int e = 0; e < 6; ++e) if (e < nf) {
            const int sp = e < 4 ? sp8(w0, e) : sp8(w1, e - 4);
            if (sp < M.ng || stick) P *= S.conc[sp];
            else P *= S.conc[sp] * M.G / M.sigma[sp];
        }
        scatter(S.accs, tb.sx_sc + 3 * r, k * P);
    }
}

// residual! (src/BatchReactor.jl:312-376) for component `lane`; returns du_lane and the
// diagnosed pressure (save_data semantics).
__device__ __noinline__ double rhs(const DevMech& M, const Tab& tb, Smem& S, double T, double Asv, double Asv_th,
                                    double u, int lane, double Mk, double* p_out) {
    const bool gas = lane < M.ng;
    const bool act = lane < M.n;
    const double rho = wave_sum(gas ? u : 0.0);                 // :326
    const double Y = u / rho;                                    // :328
    const double t = gas ? Y / Mk : 0.0;
    const double ssum = wave_sum(t);
    const double x = gas ? t / ssum : 0.0;                       // massfrac_to_molefrac!
    const double Mb = wave_sum(gas ? x * Mk : 0.0);              // average_molwt
    const double p = rho * R_GAS * T / Mb;                       // :338 / :353
    const double c = gas ? p * x / (R_GAS * T) : u;
    if (act) { S.conc[lane] = c; S.accw[lane] = 0.0; S.accs[lane] = 0.0; }
    const double Ctot = M.ntb ? wave_sum(gas ? c : 0.0) : 0.0;
    wave_sync();
    third_body(M, tb, S, Ctot, lane);
    wave_sync();
    production(M, tb, S, R_GAS * T, lane);                      // :344, :355
    wave_sync();
    const double w = act ? S.accw[lane] : 0.0;
    const double s = act ? S.accs[lane] : 0.0;
    wave_sync();
    if (lane == 0) *p_out = p;
    if (gas) return (s * Asv + w) * Mk;                          // :345, :363-370
    if (!act) return 0.0;
    return s * Asv_th * M.sigma[lane] / M.G;                    // :367 / :370
}

// analytic Jacobian d(du)/du, written column by column to the per-reactor workspace
// Jsave[j*64 + k] = J[k][j] (coalesced). Column j is built from the reactions whose rate
// depends on component j (host-built column lists, incl. third-body reactions).
__device__ __forceinline__ void jacobian(const DevMech& M, const Tab& tb, Smem& S, double T, double Asv,
                                         double Asv_th, double u, int lane, double Mk, double* Jsave) {
    const bool gas = lane < M.ng;
    const bool act = lane < M.n;
    const double RT = R_GAS * T;
    const bool xm = (M.conv & 2) != 0;
    const double c = gas ? u / Mk : u;                           // c_k = u_k/M_k = p x_k/(RT)
    if (act) S.conc[lane] = c;
    const double Ctot = M.ntb ? wave_sum(gas ? c : 0.0) : 0.0;
    wave_sync();
    third_body(M, tb, S, Ctot, lane);
    wave_sync();
    for (int r = lane; r < M.nrg; r += WAVE) {                   // per-reaction multipliers
        const uint32_t info = tb.rx_info[r], fw = tb.rx_sp[r], rw = tb.rx_pr[r];
        const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
        double Pf = 1.0, Pb = 1.0;
        for (int e = 0; e < 4; ++e) if (e < nf) Pf *= S.conc[sp8(fw, e)];
        for (int e = 0; e < 4; ++e) if (e < nr) Pb *= S.conc[sp8(rw, e)];
        const double D = S.kf[r] * Pf - S.kr[r] * Pb;
        double pre = 1.0, coefM = 0.0;
        if (tbk == 1) { pre = S.mc[gi_tbidx(info)]; coefM = 1.0; }
        else if (tbk == 2) {
            const double Mc = S.mc[gi_tbidx(info)];
            double fac, dfac;
            falloff<true>(M, S, r, gi_foidx(info), Mc, fac, dfac);
            pre = fac * (xm ? Mc : 1.0);
            coefM = dfac * (xm ? Mc : 1.0) + (xm ? fac : 0.0);
        }
        S.jpre[r] = pre;
        S.jdm[r] = D * coefM;
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const uint32_t info = tb.sx_info[r];
        const int nc = si_ncov(info);
        double k = S.ks[r];
        if (nc) {
            const uint32_t cs = M.s_cov_sp[r];
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += M.s_cov_eps[j * M.nrs + r] * S.conc[sp8(cs, j)];
            k *= exp(-s / RT);
        }
        S.sk[r] = k;
    }
    for (int j = 0; j < M.n; ++j) {
        if (act) { S.accw[lane] = 0.0; S.accs[lane] = 0.0; }
        wave_sync();
        const int cb = M.col_ptr[j], ce = M.col_ptr[j + 1];
        for (int i = cb + lane; i < ce; i += WAVE) {
            const int rr = M.col_rx[i];
            if (rr < M.nrg) {
                const int r = rr;
                const uint32_t info = tb.rx_info[r], fw = tb.rx_sp[r], rw = tb.rx_pr[r];
                const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
                const double pre = S.jpre[r];
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nf && sp8(fw, e) == j) {
                    double pr = S.kf[r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= S.conc[sp8(fw, e2)];
                    d += pre * pr;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nr && sp8(rw, e) == j) {
                    double pr = S.kr[r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= S.conc[sp8(rw, e2)];
                    d -= pre * pr;
                }
                if (tbk && j < M.ng) d += S.jdm[r] * M.tb_eff[gi_tbidx(info) * M.n + j];
                scatter(S.accw, tb.rx_sc + 3 * r, d);
            } else {
                const int r = rr - M.nrg;
                const uint32_t info = tb.sx_info[r];
                const int nf = si_nf(info), np = si_np(info), nc = si_ncov(info);
                const bool stick = si_stick(info);
                const double k = S.sk[r];
                const uint32_t w0 = tb.sx_sp[2 * r], w1 = tb.sx_sp[2 * r + 1];
                double cv[6], dc[6];
                int sp[6];
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    sp[e] = e < nf ? (e < 4 ? sp8(w0, e) : sp8(w1, e - 4)) : -1;
                    cv[e] = 1.0; dc[e] = 0.0;
                    if (e < nf) {
                        const int s = sp[e];
                        if (s < M.ng) { cv[e] = S.conc[s]; dc[e] = 1.0 / M.molwt[s]; }
                        else if (stick) { cv[e] = S.conc[s]; dc[e] = 1.0; }
                        else { cv[e] = S.conc[s] * M.G / M.sigma[s]; dc[e] = M.G / M.sigma[s]; }
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
                    const uint32_t cs = M.s_cov_sp[r];
                    for (int jj = 0; jj < 4; ++jj) if (jj < nc && sp8(cs, jj) == j)
                        d += q * (-M.s_cov_eps[jj * M.nrs + r] / RT);
                }
                scatter(S.accs, tb.sx_sc + 3 * r, d);
            }
        }
        wave_sync();
        const double w = act ? S.accw[lane] : 0.0;
        const double s = act ? S.accs[lane] : 0.0;
        double v;
        if (gas) v = (j < M.ng ? Mk * w / M.molwt[j] : 0.0) + Mk * Asv * s;
        else v = Asv_th * M.sigma[act ? lane : 0] / M.G * s;
        Jsave[j * WAVE + lane] = act ? v : 0.0;
        wave_sync();
    }
}

// ------------------------------------------------------------------------------------
// LU of I - gamma*J, row-per-lane (SUNDIALS denseGETRF semantics: partial pivoting on max
// |a_ik|, multipliers mult = 1/a_kk, a_ij -= a_kj * l_ik), without physical row swaps.
// Rolled over k: each lane keeps the live part of its row left-aligned in registers
// (a[0] = current column) and shifts it by one per step, so the code stays a few KB (the
// fully unrolled form is ~NMAX^2 blocks and thrashes the instruction cache). Finished
// columns go to LU[k*64 + lane]. Returns fail (0 or k+1 for a zero pivot) and this lane's
// pivot step in `pstep` (-> the row order).
// ------------------------------------------------------------------------------------
template <int NMAX>
__device__ __noinline__ int lu_factor_mem(const double* __restrict__ J, double* __restrict__ LU, double gamma, int n,
                                          int lane, int* pstep_out) {
    constexpr int CH = 8;
    static_assert(NMAX % CH == 0, "NMAX must be a multiple of 8");
    double a[NMAX];
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
        a[j] = -gamma * J[j * WAVE + lane];
        if (j == lane) a[j] += 1.0;
    }
    int pstep = (lane < n) ? -1 : NMAX + 1;
    int fail = 0;
    for (int k = 0; k < n; ++k) {
        const double v = (pstep < 0) ? fabs(a[0]) : -1.0;
        const int p = wave_argmax(v);
        const double piv = bcast(a[0], p);
        if (piv == 0.0 && !fail) fail = k + 1;
        if (lane == p) pstep = k;
        const bool rem = pstep < 0;
        const double mult = 1.0 / piv;
        const double l = a[0] * mult;
        LU[k * WAVE + lane] = rem ? l : a[0];
        const int live = n - k;                 // columns k..n-1 are live; a[0..live-1]
#pragma unroll
        for (int c = 0; c < NMAX; c += CH) {
            if (c < live) {
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    const int j = c + i;
                    if (j + 1 < NMAX) {
                        const double apj = bcast(a[j + 1], p);
                        a[j] = rem ? a[j + 1] - apj * l : a[j + 1];
                    } else {
                        a[j] = 0.0;
                    }
                }
            }
        }
    }
    for (int k = n; k < NMAX; ++k) LU[k * WAVE + lane] = (k == lane) ? 1.0 : 0.0;
    *pstep_out = pstep;
    return fail;
}

__device__ __forceinline__ int pivot_lane(int pstep, int k) {
    const unsigned long long m = __ballot(pstep == k);
    return __builtin_ctzll(m);
}

// solve (LU) x = b with the factors stored column-major per lane: LU[k*64 + lane] = a_lane[k].
// Rolled over chunks of 8 columns; the next chunk's loads are issued before the current
// chunk's dependent chain, so the chain does not wait on memory.
template <int NMAX>
__device__ __noinline__ double lu_solve_mem(const double* __restrict__ LU, int n, int lane, int pstep, double b) {
    constexpr int CH = 8;
    double r = b;
    double cur[CH], nxt[CH];
    const int nch = (n + CH - 1) / CH;
#pragma unroll
    for (int i = 0; i < CH; ++i) cur[i] = LU[i * WAVE + lane];
    for (int cb = 0; cb < nch; ++cb) {
        const int c = cb * CH;
        if (cb + 1 < nch) {
#pragma unroll
            for (int i = 0; i < CH; ++i) nxt[i] = LU[(c + CH + i) * WAVE + lane];
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int k = c + i;
            if (k < n) {
                const int p = pivot_lane(pstep, k);
                const double yk = bcast(r, p);
                if (pstep > k && lane < n) r = r - cur[i] * yk;
            }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) cur[i] = nxt[i];
    }
    const int c_last = (nch - 1) * CH;
#pragma unroll
    for (int i = 0; i < CH; ++i) cur[i] = LU[(c_last + i) * WAVE + lane];
    for (int cb = nch - 1; cb >= 0; --cb) {
        const int c = cb * CH;
        if (cb > 0) {
#pragma unroll
            for (int i = 0; i < CH; ++i) nxt[i] = LU[(c - CH + i) * WAVE + lane];
        }
#pragma unroll
        for (int i = CH - 1; i >= 0; --i) {
            const int k = c + i;
            if (k < n) {
                const int p = pivot_lane(pstep, k);
                if (lane == p) r = r / cur[i];
                const double xk = bcast(r, p);
                if (pstep < k) r = r - cur[i] * xk;
            }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) cur[i] = nxt[i];
    }
    // lane p holds x_{pstep(p)}: push it to lane pstep(p)
    const int dst = (lane < n) ? pstep : lane;
    const long long bits = __double_as_longlong(r);
    const int lo = __builtin_amdgcn_ds_permute(dst * 4, (int)(bits & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_permute(dst * 4, (int)(bits >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

}  // namespace brhip
