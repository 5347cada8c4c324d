// brhip_device.hpp -- device side of libbrhip.so (gfx950, fp64).
//
// Execution model: ONE REACTOR PER WAVEFRONT (64 lanes), lane k <-> solution component k
// (gas species 0..ng-1, then surface coverages). Reactions are evaluated lane-parallel
// (reaction r on lane r mod 64), species production is a per-lane ELL gather. The Newton
// matrix I - gamma*J is held ROW-PER-LANE in registers (a[NMAX]); LU pivots are found by a
// wave argmax and the pivot row is broadcast with v_readlane, so no row swaps and no LDS
// traffic in the factorisation. Mechanism tables are read-only in global memory (L1/L2
// resident); T-dependent rate constants live in LDS per reactor (T is constant:
// ConstantParams, src/BatchReactor.jl:14-17).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace brhip {

constexpr double R_GAS = 8.31446261815324;   // RxnHelperUtils.R (src/BatchReactor.jl:338)
constexpr int WAVE = 64;

struct DevMech {
    int ng, ns, n, nrg, nrs, conv;
    int ntb, nfo, ell_len;
    double p_std, G;            // Pa ; site density mol/m2
    const double* molwt;        // [n] (1 for surface)
    const double* sigma;        // [n] (1 for gas)
    const double* nasa;         // [ng*15]
    const int* g_f;             // [4][nrg]
    const int* g_r;             // [4][nrg]
    const int* g_info;          // [nrg]
    const double* g_arr;        // [3][nrg]
    const double* g_kcs;        // [nrg]
    const int* g_dnu;           // [nrg]
    const double* fo_low;       // [3][nfo]
    const double* fo_troe;      // [4][nfo]
    const int* fo_ntroe;        // [nfo]
    const int* tb_ptr;          // [ntb+1]
    const int* tb_sp;           // sparse (eff - 1) entries
    const double* tb_de;
    const double* tb_eff;       // [ntb][n] dense
    const int* s_f;             // [6][nrs]
    const int* s_info;          // [nrs]
    const double* s_arr;        // [3][nrs]
    const int* s_gas;           // [nrs]
    const int* s_cov_sp;        // [4][nrs]
    const double* s_cov_eps;    // [4][nrs]
    const int* ell_r;           // [ell_len][n]
    const double* ell_nu;       // [ell_len][n]
};

// g_info bit fields
__host__ __device__ inline int gi_nf(int v) { return v & 7; }
__host__ __device__ inline int gi_nr(int v) { return (v >> 3) & 7; }
__host__ __device__ inline int gi_rev(int v) { return (v >> 6) & 1; }
__host__ __device__ inline int gi_tb(int v) { return (v >> 7) & 3; }
__host__ __device__ inline int gi_tbidx(int v) { return (v >> 9) & 1023; }
__host__ __device__ inline int gi_foidx(int v) { return (v >> 19) & 1023; }
// s_info bit fields
__host__ __device__ inline int si_nf(int v) { return v & 7; }
__host__ __device__ inline int si_np(int v) { return (v >> 3) & 7; }
__host__ __device__ inline int si_stick(int v) { return (v >> 6) & 1; }
__host__ __device__ inline int si_ncov(int v) { return (v >> 7) & 7; }

// ------------------------------------------------------------------------------------
// wave primitives
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;  // bitwise identical in every lane (commutative pairwise butterfly)
}
__device__ __forceinline__ double uni(double v) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
    int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double bcast(double v, int lane) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// ------------------------------------------------------------------------------------
// per-reactor LDS workspace
// ------------------------------------------------------------------------------------
struct Smem {
    double* kf;    // [nrg]
    double* kr;    // [nrg]
    double* k0;    // [nfo]
    double* fc;    // [nfo]
    double* ks;    // [nrs]
    double* conc;  // [n]   gas concentrations (mol/m3) then coverages
    double* qb;    // [nrg + nrs] rates of progress / column derivatives
    double* mc;    // [ntb]
    double* jpre;  // [nrg]
    double* jdm;   // [nrg]
    double* sk;    // [nrs]
    int* pivl;     // [64]
};

__host__ __device__ inline int qb_len(int ng, int nrg, int nrs) { return nrg + nrs > ng ? nrg + nrs : ng; }
__host__ __device__ inline size_t smem_bytes(int ng, int n, int nrg, int nrs, int ntb, int nfo) {
    size_t d = (size_t)4 * nrg + 2 * (size_t)nrs + qb_len(ng, nrg, nrs) + 2 * (size_t)nfo + n + ntb;
    return d * sizeof(double) + 64 * sizeof(int) + 64;
}

__device__ __forceinline__ Smem carve(double* base, const DevMech& M) {
    Smem s;
    double* p = base;
    s.kf = p; p += M.nrg;
    s.kr = p; p += M.nrg;
    s.jpre = p; p += M.nrg;
    s.jdm = p; p += M.nrg;
    s.qb = p; p += qb_len(M.ng, M.nrg, M.nrs);
    s.ks = p; p += M.nrs;
    s.sk = p; p += M.nrs;
    s.k0 = p; p += M.nfo;
    s.fc = p; p += M.nfo;
    s.conc = p; p += M.n;
    s.mc = p; p += M.ntb;
    s.pivl = (int*)p;
    return s;
}

// T-only constants (src/BatchReactor.jl:14-17: T is a per-reactor constant)
__device__ __forceinline__ void init_tconst(const DevMech& M, Smem& S, double T, int lane) {
    // g/RT per species into qb (scratch)
    const double lT = log(T);
    for (int k = lane; k < M.ng; k += WAVE) {
        const double* c = M.nasa + 15 * k;
        const double* a = (T < c[0]) ? c + 8 : c + 1;
        double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        S.qb[k] = h - s;
    }
    __syncthreads();
    const double RT = R_GAS * T;
    for (int r = lane; r < M.nrg; r += WAVE) {
        const int info = M.g_info[r];
        const double A = M.g_arr[r], b = M.g_arr[M.nrg + r], EoR = M.g_arr[2 * M.nrg + r];
        double kf = A * exp(b * lT - EoR / T);
        double kr = 0.0;
        if (gi_rev(info)) {
            double dg = 0.0;
            const int nf = gi_nf(info), nr = gi_nr(info);
            for (int e = 0; e < 4; ++e) if (e < nr) dg += S.qb[M.g_r[e * M.nrg + r]];
            for (int e = 0; e < 4; ++e) if (e < nf) dg -= S.qb[M.g_f[e * M.nrg + r]];
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
                const double ta = M.fo_troe[fi], t3 = M.fo_troe[M.nfo + fi], t1 = M.fo_troe[2 * M.nfo + fi], t2 = M.fo_troe[3 * M.nfo + fi];
                fcv = (1 - ta) * exp(-T / t3) + ta * exp(-T / t1);
                if (M.fo_ntroe[fi] == 4) fcv += exp(-t2 / T);
            }
            S.fc[fi] = fcv;
        }
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const int info = M.s_info[r];
        const double A = M.s_arr[r], b = M.s_arr[M.nrs + r], Ea = M.s_arr[2 * M.nrs + r];
        double k;
        if (si_stick(info)) k = A * sqrt(RT / (2 * M_PI * M.molwt[M.s_gas[r]]));
        else k = A * pow(T, b) * exp(-Ea / RT);
        S.ks[r] = k;
    }
    __syncthreads();
}

// falloff: fac = Pr/(1+Pr)*F and d fac / d[M]
__device__ __forceinline__ void falloff(const DevMech& M, const Smem& S, int r, int fi, double Mc, double& fac, double& dfac, bool want_d) {
    const double kinf = S.kf[r], k0 = S.k0[fi];
    const double Pr = k0 * Mc / kinf;
    double F = 1.0, g = 0.0;
    if (M.fo_ntroe[fi]) {
        const double Prs = Pr > 1e-300 ? Pr : 1e-300;
        const double lfc = log10(S.fc[fi]);
        const double L = log10(Prs);
        const double cc = -0.4 - 0.67 * lfc, nn = 0.75 - 1.27 * lfc;
        const double den = nn - 0.14 * (L + cc);
        const double f1 = (L + cc) / den;
        const double lF = lfc / (1 + f1 * f1);
        F = pow(10.0, lF);
        if (want_d) {
            const double df1 = nn / (den * den);
            g = -lfc * 2 * f1 / ((1 + f1 * f1) * (1 + f1 * f1)) * df1;
        }
    }
    fac = Pr / (1 + Pr) * F;
    if (want_d) dfac = (F / ((1 + Pr) * (1 + Pr)) + F * g / (1 + Pr)) * (k0 / kinf);
}

// third-body concentrations [M]_t = sum_k eff_tk c_k  (conc in S.conc, Ctot = sum gas c)
__device__ __forceinline__ void third_body(const DevMech& M, Smem& S, double Ctot, int lane) {
    for (int t = lane; t < M.ntb; t += WAVE) {
        double s = Ctot;
        for (int i = M.tb_ptr[t]; i < M.tb_ptr[t + 1]; ++i) s += M.tb_de[i] * S.conc[M.tb_sp[i]];
        S.mc[t] = s;
    }
}

// rates of progress into S.qb (gas 0..nrg-1, surface nrg..)
__device__ __forceinline__ void rates_of_progress(const DevMech& M, Smem& S, double RT, int lane) {
    const bool xm = (M.conv & 2) != 0;
    for (int r = lane; r < M.nrg; r += WAVE) {
        const int info = M.g_info[r];
        const int nf = gi_nf(info), nr = gi_nr(info), tb = gi_tb(info);
        double Pf = 1.0, Pb = 1.0;
#pragma unroll
        for (int e = 0; e < 4; ++e) if (e < nf) Pf *= S.conc[M.g_f[e * M.nrg + r]];
#pragma unroll
        for (int e = 0; e < 4; ++e) if (e < nr) Pb *= S.conc[M.g_r[e * M.nrg + r]];
        double D = S.kf[r] * Pf - S.kr[r] * Pb;
        if (tb == 1) D *= S.mc[gi_tbidx(info)];
        else if (tb == 2) {
            const double Mc = S.mc[gi_tbidx(info)];
            double fac, dfac;
            falloff(M, S, r, gi_foidx(info), Mc, fac, dfac, false);
            D *= fac;
            if (xm) D *= Mc;
        }
        S.qb[r] = D;
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const int info = M.s_info[r];
        const int nf = si_nf(info), nc = si_ncov(info);
        const bool stick = si_stick(info);
        double k = S.ks[r];
        if (nc) {
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += M.s_cov_eps[j * M.nrs + r] * S.conc[M.s_cov_sp[j * M.nrs + r]];
            k *= exp(-s / RT);
        }
        double P = 1.0;
        for (int e = 0; e < 6; ++e) if (e < nf) {
            const int sp = M.s_f[e * M.nrs + r];
            if (sp < M.ng || stick) P *= S.conc[sp];
            else P *= S.conc[sp] * M.G / M.sigma[sp];
        }
        S.qb[M.nrg + r] = k * P;
    }
}

// ELL gather of the production terms for component `lane`: w (gas rxns), s (surface rxns)
__device__ __forceinline__ void gather(const DevMech& M, const Smem& S, int lane, double& w, double& s) {
    w = 0.0; s = 0.0;
    if (lane >= M.n) return;
    for (int m = 0; m < M.ell_len; ++m) {
        const int r = M.ell_r[m * M.n + lane];
        if (r < 0) break;
        const double v = M.ell_nu[m * M.n + lane] * S.qb[r];
        if (r < M.nrg) w += v; else s += v;
    }
}

// residual! (src/BatchReactor.jl:312-376) for component `lane`; returns du_lane.
// Also returns the diagnosed pressure and mole fraction (save_data semantics).
__device__ __forceinline__ double rhs(const DevMech& M, Smem& S, double T, double Asv, double Asv_th, double u,
                             int lane, double Mk, double& p_out, double& x_out) {
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
    if (act) S.conc[lane] = c;
    const double Ctot = wave_sum(gas ? c : 0.0);
    __syncthreads();
    third_body(M, S, Ctot, lane);
    __syncthreads();
    rates_of_progress(M, S, R_GAS * T, lane);                   // :344, :355
    __syncthreads();
    double w, s;
    gather(M, S, lane, w, s);
    __syncthreads();
    p_out = p; x_out = x;
    if (gas) return (s * Asv + w) * Mk;                          // :345, :363-370
    if (!act) return 0.0;
    return s * Asv_th * M.sigma[lane] / M.G;                    // :367 / :370
}

// analytic Jacobian d(du)/du: lane k receives row k in a[0..NMAX-1]
template <int NMAX>
__device__ __forceinline__ void jacobian(const DevMech& M, Smem& S, double T, double Asv, double Asv_th, double u,
                                int lane, double Mk, double (&a)[NMAX]) {
    const bool gas = lane < M.ng;
    const bool act = lane < M.n;
    const double RT = R_GAS * T;
    const bool xm = (M.conv & 2) != 0;
    const double c = gas ? u / Mk : u;                           // c_k = u_k/M_k = p x_k/(RT)
    if (act) S.conc[lane] = c;
    const double Ctot = wave_sum(gas ? c : 0.0);
    __syncthreads();
    third_body(M, S, Ctot, lane);
    __syncthreads();
    // pre-pass: per-reaction multipliers
    for (int r = lane; r < M.nrg; r += WAVE) {
        const int info = M.g_info[r];
        const int nf = gi_nf(info), nr = gi_nr(info), tb = gi_tb(info);
        double Pf = 1.0, Pb = 1.0;
        for (int e = 0; e < 4; ++e) if (e < nf) Pf *= S.conc[M.g_f[e * M.nrg + r]];
        for (int e = 0; e < 4; ++e) if (e < nr) Pb *= S.conc[M.g_r[e * M.nrg + r]];
        const double D = S.kf[r] * Pf - S.kr[r] * Pb;
        double pre = 1.0, coefM = 0.0;
        if (tb == 1) { pre = S.mc[gi_tbidx(info)]; coefM = 1.0; }
        else if (tb == 2) {
            const double Mc = S.mc[gi_tbidx(info)];
            double fac, dfac;
            falloff(M, S, r, gi_foidx(info), Mc, fac, dfac, true);
            pre = fac * (xm ? Mc : 1.0);
            coefM = dfac * (xm ? Mc : 1.0) + (xm ? fac : 0.0);
        }
        S.jpre[r] = pre;
        S.jdm[r] = D * coefM;
    }
    for (int r = lane; r < M.nrs; r += WAVE) {
        const int info = M.s_info[r];
        const int nc = si_ncov(info);
        double k = S.ks[r];
        if (nc) {
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += M.s_cov_eps[j * M.nrs + r] * S.conc[M.s_cov_sp[j * M.nrs + r]];
            k *= exp(-s / RT);
        }
        S.sk[r] = k;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NMAX; ++i) a[i] = 0.0;
    for (int j = 0; j < M.n; ++j) {
        {
            for (int r = lane; r < M.nrg; r += WAVE) {
                const int info = M.g_info[r];
                const int nf = gi_nf(info), nr = gi_nr(info), tb = gi_tb(info);
                int fe[4], re[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) { fe[e] = e < nf ? M.g_f[e * M.nrg + r] : -1; re[e] = e < nr ? M.g_r[e * M.nrg + r] : -1; }
                double d = 0.0;
                const double pre = S.jpre[r];
#pragma unroll
                for (int e = 0; e < 4; ++e) if (fe[e] == j) {
                    double pr = S.kf[r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= S.conc[fe[e2]];
                    d += pre * pr;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) if (re[e] == j) {
                    double pr = S.kr[r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= S.conc[re[e2]];
                    d -= pre * pr;
                }
                if (tb && j < M.ng) d += S.jdm[r] * M.tb_eff[gi_tbidx(info) * M.n + j];
                S.qb[r] = d;
            }
            for (int r = lane; r < M.nrs; r += WAVE) {
                const int info = M.s_info[r];
                const int nf = si_nf(info), nc = si_ncov(info);
                const bool stick = si_stick(info);
                const double k = S.sk[r];
                double cv[6], dc[6];
                int sp[6];
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    sp[e] = e < nf ? M.s_f[e * M.nrs + r] : -1;
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
                    for (int jj = 0; jj < 4; ++jj) if (jj < nc && M.s_cov_sp[jj * M.nrs + r] == j)
                        d += q * (-M.s_cov_eps[jj * M.nrs + r] / RT);
                }
                S.qb[M.nrg + r] = d;
            }
            __syncthreads();
            double w, s;
            gather(M, S, lane, w, s);
            double v;
            const bool jgas = j < M.ng;
            if (gas) v = (jgas ? Mk * w / M.molwt[j] : 0.0) + Mk * Asv * s;
            else v = Asv_th * M.sigma[act ? lane : 0] / M.G * s;
            v = act ? v : 0.0;
#pragma unroll
            for (int i = 0; i < NMAX; ++i) if (i == j) a[i] = v;
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------
// LU of the row-per-lane matrix (SUNDIALS denseGETRF semantics: partial pivoting on
// max |a_ik|, multipliers mult = 1/a_kk, a_ij -= a_kj * l_ik), without physical swaps.
// pstep = pivot step at which this lane's row was chosen. Returns 0 or k+1 if singular.
// ------------------------------------------------------------------------------------
template <int NMAX>
__device__ __forceinline__ int lu_factor(double (&a)[NMAX], int n, int lane, int& pstep, int* pivl) {
    pstep = -1;
    int fail = 0;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        if (k < n) {
            double v = (lane < n && pstep < 0) ? fabs(a[k]) : -1.0;
            int idx = lane;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const double ov = __shfl_xor(v, o, WAVE);
                const int oi = __shfl_xor(idx, o, WAVE);
                if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
            }
            const int p = uni(idx);
            const double piv = bcast(a[k], p);
            if (piv == 0.0 && !fail) fail = k + 1;
            if (lane == p) pstep = k;
            if (lane == 0) pivl[k] = p;
            const bool rem = (lane < n) && (pstep < 0);
            const double mult = 1.0 / piv;
            const double l = a[k] * mult;
            if (rem) a[k] = l;
#pragma unroll
            for (int j = k + 1; j < NMAX; ++j) {
                if (j < n) {
                    const double apj = bcast(a[j], p);
                    if (rem) a[j] = a[j] - apj * l;
                }
            }
        }
    }
    __syncthreads();
    return fail;
}

template <int NMAX>
__device__ __forceinline__ double lu_solve(const double (&a)[NMAX], int n, int lane, int pstep, const int* pivl, double b) {
    double r = b;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        if (k < n) {
            const int p = uni(pivl[k]);
            const double yk = bcast(r, p);
            if (lane < n && pstep > k) r = r - a[k] * yk;
        }
    }
#pragma unroll
    for (int k = NMAX - 1; k >= 0; --k) {
        if (k < n) {
            const int p = uni(pivl[k]);
            if (lane == p) r = r / a[k];
            const double xk = bcast(r, p);
            if (lane < n && pstep < k) r = r - a[k] * xk;
        }
    }
    const int src = (lane < n) ? pivl[lane] : lane;
    return __shfl(r, src, WAVE);
}

}  // namespace brhip
