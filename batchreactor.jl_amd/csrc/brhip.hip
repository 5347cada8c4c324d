// brhip.hip -- libbrhip.so: C-ABI (include/brhip.h) + the batched CVODE-style BDF kernel.
//
// The integrator restates SUNDIALS CVODE 5.x (the solver behind CVODE_BDF() in
// src/BatchReactor.jl:138-141,:210): Nordsieck BDF orders 1..5, modified Newton with
// maxcor 3, Jacobian reuse (msbp 20 / msbj 51 / dgmax 0.3/0.2), WRMS error test, cvHin
// initial step, tstop clamping and dense output at tstop. The Jacobian is analytic
// (brhip_device.hpp) instead of CVODE's difference quotients.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/brhip.h"
#include "brhip_device.hpp"

using namespace brhip;

namespace {

constexpr int QMAX = 5;
constexpr double HLB_FACTOR = 100.0, HUB_FACTOR = 0.1, H_BIAS = 0.5;
constexpr int MAX_ITERS = 4;
constexpr double ETAMX1 = 10000.0, ETAMX2 = 10.0, ETAMX3 = 10.0, ETAMXF = 0.2, ETAMIN = 0.1, ETACF = 0.25;
constexpr double ADDON = 1e-6, BIAS1 = 6.0, BIAS2 = 6.0, BIAS3 = 10.0, ONEPSM = 1.000001;
constexpr int SMALL_NST = 10, MXNCF = 10, MXNEF = 7, MXNEF1 = 3, SMALL_NEF = 2, LONG_WAIT = 10;
constexpr int NLS_MAXCOR = 3, MSBP = 20, LS_MSBJ = 51;
constexpr double CRDOWN = 0.3, DGMAX = 0.3, RDIV = 2.0, CORTES = 0.1, THRESH = 1.5, FUZZ = 100.0, LS_DGMAX = 0.2;
constexpr double UROUND = 2.220446049250313e-16;
enum { FIRST_CALL = 0, PREV_CONV_FAIL = 1, PREV_ERR_FAIL = 2 };
enum { NO_FAILURES = 0, FAIL_BAD_J = 1, FAIL_OTHER = 2 };

struct KOpts {
    double rtol, atol, hmax_inv, ufac;
    int max_steps, trace_cap;
};

// per-reactor controller state (LDS)
struct Ctl {
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double hprime, hscale, eta, etamax, gammap, crate, delp, acnrm, saved_tq5, p_last;
    int q, qprime, L, qwait;
    int cnt[12];
    int pstep[64];
};
constexpr int CTL_BYTES = (sizeof(Ctl) + 15) / 16 * 16;

template <int K>
__device__ __forceinline__ double getv(const double (&a)[K], int i) {
    double v = 0.0;
#pragma unroll
    for (int t = 0; t < K; ++t) if (t == i) v = a[t];
    return v;
}
template <int K>
__device__ __forceinline__ void setv(double (&a)[K], int i, double v) {
#pragma unroll
    for (int t = 0; t < K; ++t) if (t == i) a[t] = v;
}

// LDS layout of a workgroup: [packed tables][reactor 0: Ctl | Smem | Nordsieck zs]...
constexpr int ZS_VECS = QMAX + 4;   // z[0..QMAX], ewt, acor, tempv
__host__ __device__ inline size_t reactor_bytes(const DevMech& M) {
    return CTL_BYTES + reactor_doubles(M) * 8 + (size_t)ZS_VECS * WAVE * 8;
}
struct LaneVec {   // component `lane` of vector j at p[j*64]
    double* p;
    __device__ __forceinline__ double& operator[](int j) const { return p[j * WAVE]; }
};
__host__ __device__ inline size_t wg_lds_bytes(const DevMech& M, int rpb) { return tab_bytes(M) + rpb * reactor_bytes(M); }

struct WaveCtx {
    int wave, lane, rid;
    Tab tb;
    char* rbase;   // this wave's reactor block
};
__device__ __forceinline__ WaveCtx wave_ctx(const DevMech& M, char* smem, int rpb) {
    WaveCtx w;
    w.wave = threadIdx.x >> 6;
    w.lane = threadIdx.x & 63;
    w.rid = blockIdx.x * rpb + w.wave;
    stage_tables(M, reinterpret_cast<uint32_t*>(smem));
    w.tb = tab_view(reinterpret_cast<const uint32_t*>(smem), M);
    w.rbase = smem + tab_bytes(M) + (size_t)w.wave * reactor_bytes(M);
    return w;
}

// ------------------------------------------------------------------------------------
// the integrator: one reactor per 64-lane workgroup
// ------------------------------------------------------------------------------------
#ifndef BR_WPE
#define BR_WPE 2
#endif
template <int NMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BR_WPE, 8))) void k_integrate(
    DevMech M, int N, int rpb, const double* __restrict__ Tv, const double* __restrict__ Asvv, double* __restrict__ U,
    const double* __restrict__ tfv, KOpts o, double* __restrict__ stats, double* __restrict__ Jws,
    double* __restrict__ trace) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx(M, smem_raw, rpb);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    const Tab& tb = W.tb;
    double* smem = reinterpret_cast<double*>(W.rbase);
    const int n = M.n;
    const bool act = lane < n;
    Smem S = carve(smem + CTL_BYTES / 8, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    const double tstop = tfv[rid];
    const double Mk = act ? M.molwt[lane] : 1.0;
    double* Jsave = Jws + (size_t)rid * 2 * NMAX * WAVE;   // J, then the LU factors
    double* LUsave = Jsave + NMAX * WAVE;

    init_tconst(M, tb, S, T, lane);

    // Nordsieck history and long-lived work vectors (this lane's component) live in the
    // reactor's LDS block: zs[j*64 + lane]; y/ftemp/delta stay in registers
    double* zs = smem + CTL_BYTES / 8 + reactor_doubles(M);
    const LaneVec z{zs + lane};
    double& ewt = zs[(QMAX + 1) * WAVE + lane];
    double& acor = zs[(QMAX + 2) * WAVE + lane];
    double& tempv = zs[(QMAX + 3) * WAVE + lane];
#pragma unroll
    for (int j = 0; j <= QMAX; ++j) z[j] = 0.0;
    ewt = 1.0; acor = 0.0; tempv = 0.0;
    double y = 0.0, ftemp = 0.0, delta = 0.0;
    int pstep = -1;
    // uniform controller state: kept in LDS (one copy per reactor) to free VGPRs for the
    // row-per-lane Newton matrix; every lane reads/writes the same values.
    Ctl& C = *reinterpret_cast<Ctl*>(smem);
    double (&tau)[QMAX + 2] = C.tau;
    double (&tq)[6] = C.tq;
    double (&l)[QMAX + 1] = C.l;
#pragma unroll
    for (int i = 0; i < QMAX + 2; ++i) tau[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) tq[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
    double tn = 0.0, h = 0.0, rl1 = 0.0, gamma = 0.0, gamrat = 1.0;
    double& hprime = C.hprime; double& hscale = C.hscale; double& eta = C.eta; double& etamax = C.etamax;
    double& gammap = C.gammap; double& crate = C.crate; double& delp = C.delp; double& acnrm = C.acnrm;
    double& saved_tq5 = C.saved_tq5;
    hprime = 0.0; hscale = 0.0; eta = 1.0; etamax = ETAMX1; gammap = 0.0; crate = 1.0; delp = 0.0; acnrm = 0.0;
    saved_tq5 = 0.0;
    int& q = C.q; int& qprime = C.qprime; int& L = C.L; int& qwait = C.qwait;
    q = 1; qprime = 1; L = 2; qwait = 2;
    int& nst = C.cnt[0]; int& nfe = C.cnt[1]; int& nsetups = C.cnt[2]; int& nje = C.cnt[3]; int& nni = C.cnt[4];
    int& ncfn = C.cnt[5]; int& netf = C.cnt[6]; int& nstlp = C.cnt[7]; int& nstlj = C.cnt[8];
    int& jcur = C.cnt[9];
#pragma unroll
    for (int i = 0; i < 10; ++i) C.cnt[i] = 0;
    double& p_last = C.p_last;
    const double hmin = 0.0;
    // phase cycle counters (lane 0 accumulates)
    unsigned long long cyc_rhs = 0, cyc_jac = 0, cyc_lu = 0, cyc_sol = 0;
    const unsigned long long cyc0 = wall_clock64();
    wave_sync();

    z[0] = act ? U[(size_t)rid * n + lane] : 0.0;
    const double ulimit = o.ufac * uni(wave_sum(act ? fabs(z[0]) : 0.0));

    auto F = [&](double yv) __attribute__((always_inline)) -> double {
        const unsigned long long c0 = clock64();
        const double r = rhs(M, tb, S, T, Asv, Asv_th, yv, lane, Mk, &p_last);
        cyc_rhs += clock64() - c0;
        return r;
    };
    auto wrms = [&](double v) __attribute__((always_inline)) -> double {
        const double t = act ? v * ewt : 0.0;
        return uni(sqrt(wave_sum(t * t) / n));
    };
    auto set_ewt = [&]() __attribute__((always_inline)) { ewt = act ? 1.0 / (o.rtol * fabs(z[0]) + o.atol) : 1.0; };

    auto rescale = [&]() __attribute__((always_inline)) {
        double factor = eta;
#pragma unroll
        for (int j = 1; j <= QMAX; ++j) if (j <= q) { z[j] *= factor; factor *= eta; }
        h = hscale * eta; hscale = h;
    };
    auto predict = [&]() __attribute__((always_inline)) {
        tn += h;
        if ((tn - tstop) * h > 0) tn = tstop;
#pragma unroll
        for (int k = 1; k <= QMAX; ++k)
#pragma unroll
            for (int j = QMAX; j >= k; --j)
                if (j <= q && k <= q) z[j - 1] += z[j];
    };
    auto restore = [&](double saved_t) __attribute__((always_inline)) {
        tn = saved_t;
#pragma unroll
        for (int k = 1; k <= QMAX; ++k)
#pragma unroll
            for (int j = QMAX; j >= k; --j)
                if (j <= q && k <= q) z[j - 1] -= z[j];
    };
    auto cvset = [&]() __attribute__((always_inline)) {
        double xi_inv = 1.0, xistar_inv = 1.0;
        l[0] = 1.0; l[1] = 1.0;
#pragma unroll
        for (int i = 2; i <= QMAX; ++i) l[i] = 0.0;
        double alpha0 = -1.0, alpha0_hat = -1.0, hsum = h;
        if (q > 1) {
#pragma unroll
            for (int j = 2; j < QMAX; ++j) {
                if (j < q) {
                    hsum += tau[j - 1];
                    xi_inv = h / hsum;
                    alpha0 -= 1.0 / j;
#pragma unroll
                    for (int i = QMAX; i >= 1; --i) if (i <= j) l[i] += l[i - 1] * xi_inv;
                }
            }
            alpha0 -= 1.0 / q;
            xistar_inv = -l[1] - alpha0;
            hsum += getv(tau, q - 1);
            xi_inv = h / hsum;
            alpha0_hat = -l[1] - xi_inv;
#pragma unroll
            for (int i = QMAX; i >= 1; --i) if (i <= q) l[i] += l[i - 1] * xistar_inv;
        }
        // cvSetTqBDF
        const double A1 = 1.0 - alpha0_hat + alpha0;
        const double A2 = 1.0 + q * A1;
        const double lq = getv(l, q);
        tq[2] = fabs(A1 / (alpha0 * A2));
        tq[5] = fabs(A2 * xistar_inv / (lq * xi_inv));
        if (qwait == 1) {
            if (q > 1) {
                const double C = xistar_inv / lq;
                const double A3 = alpha0 + 1.0 / q;
                const double A4 = alpha0_hat + xi_inv;
                const double Cpinv = (1.0 - A4 + A3) / A3;
                tq[1] = fabs(C * Cpinv);
            } else tq[1] = 1.0;
            hsum += getv(tau, q);
            xi_inv = h / hsum;
            const double A5 = alpha0 - (1.0 / (q + 1));
            const double A6 = alpha0_hat - xi_inv;
            const double Cppinv = (1.0 - A6 + A5) / A2;
            tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
        }
        tq[4] = CORTES / tq[2];
        rl1 = 1.0 / l[1];
        gamma = h * rl1;
        if (nst == 0) gammap = gamma;
        gamrat = (nst > 0) ? gamma / gammap : 1.0;
    };
    auto adjust_order = [&](int dq) __attribute__((always_inline)) {
        if (q == 2 && dq != 1) return;
        if (dq == 1) {  // cvIncreaseBDF
#pragma unroll
            for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
            l[2] = 1.0;
            double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = hscale;
            if (q > 1) {
#pragma unroll
                for (int j = 1; j < QMAX; ++j) {
                    if (j < q) {
                        hsum += tau[j + 1];
                        const double xi = hsum / hscale;
                        prod *= xi;
                        alpha0 -= 1.0 / (j + 1);
                        alpha1 += 1.0 / xi;
#pragma unroll
                        for (int i = QMAX; i >= 2; --i) if (i <= j + 2) l[i] = l[i] * xiold + l[i - 1];
                        xiold = xi;
                    }
                }
            }
            const double A1 = (-alpha0 - alpha1) / prod;
            const double zL = A1 * z[QMAX];   // zn[L] = A1 * zn[indx_acor], indx_acor = qmax
#pragma unroll
            for (int j = 2; j <= QMAX; ++j) if (j <= q) z[j] += l[j] * zL;
#pragma unroll
            for (int j = 1; j <= QMAX; ++j) if (j == q + 1) z[j] = zL;
        } else {        // cvDecreaseBDF
#pragma unroll
            for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
            l[2] = 1.0;
            double hsum = 0.0;
#pragma unroll
            for (int j = 1; j <= QMAX - 2; ++j) {
                if (j <= q - 2) {
                    hsum += tau[j];
                    const double xi = hsum / hscale;
#pragma unroll
                    for (int i = QMAX; i >= 2; --i) if (i <= j + 2) l[i] = l[i] * xi + l[i - 1];
                }
            }
            double zq = 0.0;
#pragma unroll
            for (int j = 0; j <= QMAX; ++j) if (j == q) zq = z[j];
#pragma unroll
            for (int j = 2; j < QMAX; ++j) if (j < q) z[j] -= l[j] * zq;
        }
    };
    // cvLsSetup: A = I - gamma*J (J fresh or saved) and factor it
    auto lsetup = [&](int convfail) __attribute__((always_inline)) -> int {
        const double dgamma = fabs(gamma / gammap - 1.0);
        const bool jbad = (nst == 0) || (nst > nstlj + LS_MSBJ) || ((convfail == FAIL_BAD_J) && (dgamma < LS_DGMAX)) ||
                          (convfail == FAIL_OTHER);
        if (!jbad) {
            jcur = 0;
        } else {
            jcur = 1; nje++; nstlj = nst;
            const unsigned long long c0 = clock64();
            jacobian(M, tb, S, T, Asv, Asv_th, y, lane, Mk, Jsave);
            cyc_jac += clock64() - c0;
        }
        const unsigned long long c1 = clock64();
        const int rc = lu_factor_mem<NMAX>(Jsave, LUsave, gamma, n, lane, &C.pstep[lane]);
        pstep = C.pstep[lane];
        cyc_lu += clock64() - c1;
        return rc;
    };
    // cvNls with SUNNonlinSol_Newton semantics
    auto nls = [&](int nflag) __attribute__((always_inline)) -> int {
        const int convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? NO_FAILURES : FAIL_OTHER;
        bool callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (nst == 0) ||
                         (nst >= nstlp + MSBP) || (fabs(gamrat - 1.0) > DGMAX);
        acor = 0.0;
        const double tol = tq[4];
        bool jbad = false;
        int jc = 0;
        int m = 0;
        for (;;) {
            y = z[0] + acor;
            ftemp = F(y);
            nfe++;
            delta = (rl1 * z[1] + acor) - gamma * ftemp;
            if (m == 0 && callSetup) {
                const int lr = lsetup(jbad ? FAIL_BAD_J : convfail);
                nsetups++;
                jc = jcur;
                gamrat = 1.0; gammap = gamma; crate = 1.0; nstlp = nst;
                if (lr) { y = z[0] + acor; return 2; }
            }
            nni++;
            delta = -delta;
            {
                const unsigned long long c0 = clock64();
                delta = lu_solve_mem<NMAX>(LUsave, n, lane, pstep, delta);
                cyc_sol += clock64() - c0;
            }
            if (gamrat != 1.0) delta *= 2.0 / (1.0 + gamrat);
            acor += delta;
            const double del = wrms(delta);
            if (m > 0) crate = fmax(CRDOWN * crate, del / delp);
            const double dcon = del * fmin(1.0, crate) / tol;
            if (dcon <= 1.0) {
                acnrm = (m == 0) ? del : wrms(acor);
                y = z[0] + acor;
                jcur = 0;
                return 0;
            }
            bool fail = (m >= 1) && (del > RDIV * delp);
            if (!fail) {
                delp = del;
                m++;
                if (m >= NLS_MAXCOR) fail = true;
            }
            if (fail) {
                if (!jc) { callSetup = true; jbad = true; acor = 0.0; m = 0; continue; }
                break;
            }
        }
        y = z[0] + acor;
        return 1;
    };

    // ---- CVodeInit + first call ----
    set_ewt();
    z[1] = F(z[0]);
    nfe++;
    {   // cvHin
        const double tout = tstop;
        const double tdist = fabs(tout - tn);
        const double tround = UROUND * fmax(fabs(tn), fabs(tout));
        const double hlb = HLB_FACTOR * tround;
        const double ratio = act ? fabs(z[1]) / (HUB_FACTOR * fabs(z[0]) + 1.0 / ewt) : 0.0;
        const double hub_inv = uni(wave_max(ratio));
        double hub = HUB_FACTOR * tdist;
        if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
        double hg = sqrt(hlb * hub);
        if (hub < hlb) {
            h = hg;
        } else {
            bool hnewOK = false;
            double hnew = hg;
            for (int count1 = 1; count1 <= MAX_ITERS; ++count1) {
                y = hg * z[1] + z[0];
                tempv = F(y);
                nfe++;
                tempv = (tempv - z[1]) * (1.0 / hg);
                const double yddnrm = wrms(tempv);
                if (hnewOK || count1 == MAX_ITERS) { hnew = hg; break; }
                hnew = (yddnrm * hub * hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * hub);
                const double hrat = hnew / hg;
                if ((hrat > 0.5) && (hrat < 2.0)) hnewOK = true;
                if ((count1 > 1) && (hrat > 2.0)) { hnew = hg; hnewOK = true; }
                hg = hnew;
            }
            double h0 = H_BIAS * hnew;
            if (h0 < hlb) h0 = hlb;
            if (h0 > hub) h0 = hub;
            h = h0;
        }
    }
    if (o.hmax_inv > 0) { const double rh = fabs(h) * o.hmax_inv; if (rh > 1.0) h /= rh; }
    if ((tn + h - tstop) * h > 0.0) h = (tstop - tn) * (1.0 - 4.0 * UROUND);
    hscale = h; hprime = h;
    if (trace) {
        double* row = trace + (size_t)rid * (o.trace_cap + 1) * (n + 4);
        if (lane == 0) { row[0] = 0.0; row[1] = h; row[2] = 1.0; row[3] = p_last; }
        if (act) row[4 + lane] = z[0];
    }
    z[1] *= h;

    int status = 0;
    int nstloc = 0;
    double u_out = z[0];
    for (;;) {
        if (nst > 0) set_ewt();
        if (nstloc >= o.max_steps) { status = BR_ERR_MAXSTEPS; break; }
        // ---- cvStep ----
        const double saved_t = tn;
        int ncf = 0, nef = 0, nflag = FIRST_CALL;
        double dsm = 0.0;
        int kflag = 0;
        if ((nst > 0) && (hprime != h)) {
            if (qprime != q) { adjust_order(qprime - q); q = qprime; L = q + 1; qwait = L; }
            rescale();
        }
        for (;;) {
            predict();
            cvset();
            const int r = nls(nflag);
            if (r != 0) {
                ncfn++;
                restore(saved_t);
                ncf++;
                etamax = 1.0;
                if ((fabs(h) <= hmin * ONEPSM) || (ncf == MXNCF)) { kflag = BR_ERR_CONV; break; }
                eta = fmax(ETACF, hmin / fabs(h));
                nflag = PREV_CONV_FAIL;
                rescale();
                continue;
            }
            dsm = acnrm * tq[2];
            if (dsm <= 1.0) break;
            nef++; netf++; nflag = PREV_ERR_FAIL;
            restore(saved_t);
            if ((fabs(h) <= hmin * ONEPSM) || (nef == MXNEF)) { kflag = BR_ERR_ERRTEST; break; }
            etamax = 1.0;
            if (nef <= MXNEF1) {
                eta = 1.0 / (pow(BIAS2 * dsm, 1.0 / L) + ADDON);
                eta = fmax(ETAMIN, fmax(eta, hmin / fabs(h)));
                if (nef >= SMALL_NEF) eta = fmin(eta, ETAMXF);
                rescale();
                continue;
            }
            if (q > 1) {
                eta = fmax(ETAMIN, hmin / fabs(h));
                adjust_order(-1);
                L = q; q--; qwait = L;
                rescale();
                continue;
            }
            eta = fmax(ETAMIN, hmin / fabs(h));
            h *= eta; hscale = h; qwait = LONG_WAIT;
            tempv = F(z[0]);
            nfe++;
            z[1] = h * tempv;
        }
        if (kflag) { status = kflag; break; }
        // cvCompleteStep
        nst++;
#pragma unroll
        for (int i = QMAX + 1; i >= 2; --i) if (i <= q) tau[i] = tau[i - 1];
        if ((q == 1) && (nst > 1)) tau[2] = tau[1];
        tau[1] = h;
#pragma unroll
        for (int j = 0; j <= QMAX; ++j) if (j <= q) z[j] += l[j] * acor;
        qwait--;
        if ((qwait == 1) && (q != QMAX)) { z[QMAX] = acor; saved_tq5 = tq[5]; }
        // cvPrepareNextStep
        if (etamax == 1.0) {
            qwait = qwait > 2 ? qwait : 2;
            qprime = q; hprime = h; eta = 1.0;
        } else {
            const double etaq = 1.0 / (pow(BIAS2 * dsm, 1.0 / L) + ADDON);
            bool choose = (qwait == 0);
            if (!choose) { eta = etaq; qprime = q; }
            else {
                qwait = 2;
                double etaqm1 = 0.0, etaqp1 = 0.0;
                if (q > 1) {
                    double zq = 0.0;
#pragma unroll
                    for (int j = 0; j <= QMAX; ++j) if (j == q) zq = z[j];
                    const double ddn = wrms(zq) * tq[1];
                    etaqm1 = 1.0 / (pow(BIAS1 * ddn, 1.0 / q) + ADDON);
                }
                if (q != QMAX && saved_tq5 != 0.0) {
                    const double cquot = (tq[5] / saved_tq5) * pow(h / tau[2], (double)L);
                    tempv = acor - cquot * z[QMAX];
                    const double dup = wrms(tempv) * tq[3];
                    etaqp1 = 1.0 / (pow(BIAS3 * dup, 1.0 / (L + 1)) + ADDON);
                }
                const double etam = fmax(etaqm1, fmax(etaq, etaqp1));
                if (etam < THRESH) { eta = 1.0; qprime = q; }
                else if (etam == etaq) { eta = etaq; qprime = q; }
                else if (etam == etaqm1) { eta = etaqm1; qprime = q - 1; }
                else { eta = etaqp1; qprime = q + 1; z[QMAX] = acor; }
            }
            // cvSetEta
            if (eta < THRESH) { eta = 1.0; hprime = h; }
            else {
                eta = fmin(eta, etamax);
                eta /= fmax(1.0, fabs(h) * o.hmax_inv * eta);
                hprime = h * eta;
            }
        }
        etamax = (nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
        acor *= tq[2];
        nstloc++;
        if (o.ufac > 0.0) {   // runaway state (br_opts.unstable_factor)
            const double mx = uni(wave_max(act ? fabs(z[0]) : 0.0));
            if (!(mx <= ulimit)) { status = BR_ERR_UNSTABLE; break; }
        }
        if (trace && nst <= o.trace_cap) {   // per-step sample buffer (save_data rows)
            double* row = trace + ((size_t)rid * (o.trace_cap + 1) + nst) * (n + 4);
            if (lane == 0) { row[0] = tn; row[1] = h; row[2] = (double)q; row[3] = p_last; }
            if (act) row[4 + lane] = z[0];
        }
        // CVode ONE_STEP + tstop handling
        const double troundoff = FUZZ * UROUND * (fabs(tn) + fabs(h));
        if (fabs(tn - tstop) <= troundoff) {
            // CVodeGetDky(tstop, 0)
            const double s = (tstop - tn) / h;
            double yv = 0.0;
#pragma unroll
            for (int j = QMAX; j >= 0; --j) {
                if (j == q) yv = z[j];
                else if (j < q) yv = z[j] + s * yv;
            }
            u_out = yv;
            if (trace && nst <= o.trace_cap) {
                double* row = trace + ((size_t)rid * (o.trace_cap + 1) + nst) * (n + 4);
                if (lane == 0) row[0] = tstop;
                if (act) row[4 + lane] = yv;
            }
            break;
        }
        if ((tn + hprime - tstop) * h > 0.0) {
            hprime = (tstop - tn) * (1.0 - 4.0 * UROUND);
            eta = hprime / h;
        }
    }
    if (status) u_out = z[0];
    if (act) U[(size_t)rid * n + lane] = u_out;
    if (stats && lane == 0) {
        double* st = stats + (size_t)rid * BR_NSTAT;
        st[0] = (double)nst; st[1] = (double)nfe; st[2] = (double)nje; st[3] = (double)nsetups;
        st[4] = (double)nni; st[5] = (double)ncfn; st[6] = (double)netf; st[7] = (double)status;
        st[8] = (double)(wall_clock64() - cyc0); st[9] = (double)cyc_rhs; st[10] = (double)cyc_jac;
        st[11] = (double)cyc_lu; st[12] = (double)cyc_sol; st[13] = tn;
    }
}

// ------------------------------------------------------------------------------------
// parity kernels: rates, rhs, jacobian (one reactor per wave)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rates(DevMech M, int N, int rpb, const double* Tv, const double* pv,
                                               const double* X, const double* TH, double* W_, double* SD) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx(M, smem_raw, rpb);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    Smem S = carve(reinterpret_cast<double*>(W.rbase) + CTL_BYTES / 8, M);
    const double T = Tv[rid], p = pv[rid];
    init_tconst(M, W.tb, S, T, lane);
    double c = 0.0;
    if (lane < M.ng) c = p * X[(size_t)rid * M.ng + lane] / (R_GAS * T);
    else if (lane < M.n) c = TH ? TH[(size_t)rid * M.ns + (lane - M.ng)] : 0.0;
    if (lane < M.n) { S.conc[lane] = c; S.accw[lane] = 0.0; S.accs[lane] = 0.0; }
    const double Ctot = wave_sum(lane < M.ng ? c : 0.0);
    wave_sync();
    third_body(M, W.tb, S, Ctot, lane);
    wave_sync();
    production(M, W.tb, S, R_GAS * T, lane);
    wave_sync();
    const double w = lane < M.n ? S.accw[lane] : 0.0;
    const double s = lane < M.n ? S.accs[lane] : 0.0;
    if (lane < M.ng) W_[(size_t)rid * M.ng + lane] = w;
    if (SD && lane < M.n) SD[(size_t)rid * M.n + lane] = s;
}

__global__ __launch_bounds__(256) void k_rhs(DevMech M, int N, int rpb, const double* Tv, const double* Asvv,
                                             const double* U, double* DU) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx(M, smem_raw, rpb);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    Smem S = carve(reinterpret_cast<double*>(W.rbase) + CTL_BYTES / 8, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst(M, W.tb, S, T, lane);
    const bool act = lane < M.n;
    const double u = act ? U[(size_t)rid * M.n + lane] : 0.0;
    const double Mk = act ? M.molwt[lane] : 1.0;
    const double du = rhs(M, W.tb, S, T, Asv, Asv_th, u, lane, Mk, reinterpret_cast<double*>(W.rbase) + 8);
    if (act) DU[(size_t)rid * M.n + lane] = du;
}

template <int NMAX>
__global__ __launch_bounds__(256) void k_jac(DevMech M, int N, int rpb, const double* Tv, const double* Asvv,
                                             const double* U, double* J, double* Jws) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx(M, smem_raw, rpb);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    Smem S = carve(reinterpret_cast<double*>(W.rbase) + CTL_BYTES / 8, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst(M, W.tb, S, T, lane);
    const bool act = lane < M.n;
    const double u = act ? U[(size_t)rid * M.n + lane] : 0.0;
    const double Mk = act ? M.molwt[lane] : 1.0;
    double* Jsave = Jws + (size_t)rid * NMAX * WAVE;
    jacobian(M, W.tb, S, T, Asv, Asv_th, u, lane, Mk, Jsave);
    if (act) {
        double* row = J + ((size_t)rid * M.n + lane) * M.n;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) if (j < M.n) row[j] = Jsave[j * WAVE + lane];
    }
}

}  // namespace

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
struct br_mech {
    int device = 0;
    int ng = 0, ns = 0, nrg = 0, nrs = 0, n = 0, nmax = 64, rpb = 1, waves_per_cu = 0;
    DevMech dm{};
    size_t shmem1 = 0;
    std::vector<void*> allocs;
    size_t shmem = 0;
    // cached device workspace for host-buffer entry points
    void* ws = nullptr;
    size_t ws_bytes = 0;
    double* jws = nullptr;
    size_t jws_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool ev_recorded = false;
};

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
static int fail_code_input() { return fail(BR_ERR_INPUT, "bad argument"); }
#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) return fail(BR_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

template <class T>
static int upload(br_mech* m, const std::vector<T>& v, const T** out) {
    void* p = nullptr;
    size_t b = std::max<size_t>(v.size(), 1) * sizeof(T);
    HIPCHK(hipMalloc(&p, b));
    if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    m->allocs.push_back(p);
    *out = (const T*)p;
    return 0;
}

extern "C" {

int br_version(void) { return 200; }
const char* br_last_error(void) { return g_err.c_str(); }
int br_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int br_mech_info(const br_mech* m, int* ng, int* ns, int* nrg, int* nrs) {
    if (!m) return fail(BR_ERR_INPUT, "null mech");
    if (ng) *ng = m->ng;
    if (ns) *ns = m->ns;
    if (nrg) *nrg = m->nrg;
    if (nrs) *nrs = m->nrs;
    return 0;
}

int br_mech_create(const br_mech_desc* d, int device, br_mech** out) {
    if (!d || !out) return fail(BR_ERR_INPUT, "null argument");
    const int ng = d->ng, ns = d->ns, nrg = d->nrg, nrs = d->nrs, n = ng + ns;
    if (ng <= 0 || ns < 0 || nrg < 0 || nrs < 0) return fail(BR_ERR_INPUT, "bad sizes");
    if (n > 64) return fail(BR_ERR_UNSUPPORTED, "n > 64 components is not supported by this build");
    if (nrg + nrs > 65535) return fail(BR_ERR_UNSUPPORTED, "too many reactions");
    HIPCHK(hipSetDevice(device));
    br_mech* m = new br_mech();
    m->device = device; m->ng = ng; m->ns = ns; m->nrg = nrg; m->nrs = nrs; m->n = n;
    m->nmax = n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 56 ? 56 : 64));
    DevMech& M = m->dm;
    M.ng = ng; M.ns = ns; M.n = n; M.nrg = nrg; M.nrs = nrs; M.nr = nrg + nrs; M.conv = d->conv;
    M.p_std = d->p_std > 0 ? d->p_std : 1e5;
    M.G = d->site_density * 1e4;
    std::vector<double> molwt(n, 1.0), sigma(n, 1.0), nasa((size_t)ng * 15);
    for (int k = 0; k < ng; ++k) molwt[k] = d->molwt[k];
    for (int i = 0; i < ns; ++i) sigma[ng + i] = d->sigma ? d->sigma[i] : 1.0;
    for (size_t i = 0; i < (size_t)ng * 15; ++i) nasa[i] = d->nasa[i];
    auto pack4 = [](const int* v, int cnt) {
        uint32_t w = 0;
        for (int e = 0; e < 4; ++e) w |= (uint32_t)(e < cnt ? (v[e] & 255) : 255) << (8 * e);
        return w;
    };
    // ---- gas reactions, evaluated in a permuted order (falloff, then +M, then elementary) so
    //      that the lanes of one pass take the same branch; results are per species, so the
    //      order is invisible outside the kernel
    std::vector<int> perm;
    for (int pass = 2; pass >= 0; --pass)
        for (int r = 0; r < nrg; ++r) if (d->g_tb[r] == pass) perm.push_back(r);
    std::vector<uint32_t> rx_sp(nrg), rx_pr(nrg), rx_info(nrg), rx_sc(3 * (size_t)nrg);
    // net-stoichiometry scatter list of a reaction: up to 6 (species, nu != 0) pairs packed in
    // 3 words: w0 = species 0..3, w1 = species 4..5 | count << 16, w2 = 4-bit signed nu x 6
    auto scatter_pack = [](const int* f, int nf, const int* pr, int np, uint32_t* w) -> bool {
        int sp[12], nu[12], c = 0;
        auto add = [&](int k, int v) {
            for (int i = 0; i < c; ++i) if (sp[i] == k) { nu[i] += v; return; }
            sp[c] = k; nu[c] = v; ++c;
        };
        for (int e = 0; e < nf; ++e) add(f[e], -1);
        for (int e = 0; e < np; ++e) add(pr[e], 1);
        int m = 0;
        w[0] = w[1] = w[2] = 0;
        for (int i = 0; i < c; ++i) {
            if (nu[i] == 0) continue;
            if (m >= 6 || nu[i] < -8 || nu[i] > 7) return false;
            if (m < 4) w[0] |= (uint32_t)(sp[i] & 255) << (8 * m);
            else w[1] |= (uint32_t)(sp[i] & 255) << (8 * (m - 4));
            w[2] |= (uint32_t)(nu[i] & 15) << (4 * m);
            ++m;
        }
        w[1] |= (uint32_t)m << 16;
        return true;
    };
    std::vector<int> gdnu(nrg);
    std::vector<double> garr(3 * (size_t)std::max(nrg, 1), 0.0), gkcs(std::max(nrg, 1), 1.0);
    int ntb = 0, nfo = 0;
    std::vector<int> fo_of(nrg, -1), tb_of(nrg, -1);
    for (int i = 0; i < nrg; ++i) {
        const int r = perm[i];
        if (d->g_tb[r] == 2) fo_of[r] = nfo++;
        if (d->g_tb[r]) tb_of[r] = ntb++;
    }
    if (ntb > 1023 || nfo > 1023) { delete m; return fail(BR_ERR_UNSUPPORTED, "too many third-body reactions"); }
    std::vector<double> folow(3 * (size_t)std::max(nfo, 1), 0.0), fotroe(4 * (size_t)std::max(nfo, 1), 0.0);
    std::vector<int> fontroe(std::max(nfo, 1), 0);
    std::vector<int> tbptr(1, 0);
    std::vector<uint32_t> tbsp;
    std::vector<double> tbde, tbeff;
    for (int i = 0; i < nrg; ++i) {
        const int r = perm[i];
        const int nf = d->g_nf[r], nr = d->g_nr[r], tb = d->g_tb[r];
        if (nf > 4 || nr > 4 || nf < 1) { delete m; return fail(BR_ERR_UNSUPPORTED, "reaction with >4 entries"); }
        rx_sp[i] = pack4(d->g_f + r * 4, nf);
        rx_pr[i] = pack4(d->g_r + r * 4, nr);
        if (!scatter_pack(d->g_f + r * 4, nf, d->g_r + r * 4, nr, &rx_sc[3 * (size_t)i])) {
            delete m; return fail(BR_ERR_UNSUPPORTED, "reaction touches more than 6 species");
        }
        for (int c = 0; c < 3; ++c) garr[(size_t)c * nrg + i] = d->g_arr[r * 3 + c];
        gdnu[i] = nr - nf;
        if ((d->conv & BR_CONV_KC_UNIT_SLIP) && tb != 2) gkcs[i] = std::pow(1e6, (double)(nr - nf));
        int tbidx = 0, foidx = 0;
        if (tb) {
            tbidx = tb_of[r];
            for (int k = 0; k < ng; ++k) {
                const double e = d->g_eff[(size_t)r * ng + k];
                if (e != 1.0) { tbsp.push_back((uint32_t)k); tbde.push_back(e - 1.0); }
            }
            tbptr.push_back((int)tbsp.size());
            for (int k = 0; k < n; ++k) tbeff.push_back(k < ng ? d->g_eff[(size_t)r * ng + k] : 0.0);
        }
        if (tb == 2) {
            foidx = fo_of[r];
            for (int c = 0; c < 3; ++c) folow[(size_t)c * nfo + foidx] = d->g_low[r * 3 + c];
            fontroe[foidx] = d->g_troe_n[r];
            for (int c = 0; c < 4; ++c) fotroe[(size_t)c * nfo + foidx] = d->g_troe[r * 4 + c];
        }
        rx_info[i] = (uint32_t)(nf | (nr << 3) | ((d->g_rev[r] ? 1 : 0) << 6) | (tb << 7) | (tbidx << 9) | (foidx << 19));
    }
    M.ntb = ntb; M.nfo = nfo; M.ntbe = (int)tbsp.size();
    // ---- surface reactions
    std::vector<uint32_t> sx_sp(2 * (size_t)nrs), sx_pr(2 * (size_t)nrs), sx_info(nrs), scs(std::max(nrs, 1), 0);
    std::vector<uint32_t> sx_sc(3 * (size_t)nrs);
    std::vector<double> sarr(3 * (size_t)std::max(nrs, 1), 0.0), sce(4 * (size_t)std::max(nrs, 1), 0.0);
    for (int r = 0; r < nrs; ++r) {
        const int nf = d->s_nf[r], np = d->s_np[r], nc = d->s_ncov[r];
        if (nf > 6 || np > 6 || nc > 4) { delete m; return fail(BR_ERR_UNSUPPORTED, "surface reaction too large"); }
        int e6[6];
        for (int e = 0; e < 6; ++e) e6[e] = e < nf ? d->s_f[r * 6 + e] : 255;
        sx_sp[2 * r] = pack4(e6, 4);
        sx_sp[2 * r + 1] = pack4(e6 + 4, 2);
        int p6[6];
        for (int e = 0; e < 6; ++e) p6[e] = e < np ? d->s_p[r * 6 + e] : 255;
        sx_pr[2 * r] = pack4(p6, 4);
        sx_pr[2 * r + 1] = pack4(p6 + 4, 2);
        if (!scatter_pack(d->s_f + r * 6, nf, d->s_p + r * 6, np, &sx_sc[3 * (size_t)r])) {
            delete m; return fail(BR_ERR_UNSUPPORTED, "surface reaction touches more than 6 species");
        }
        for (int c = 0; c < 3; ++c) sarr[(size_t)c * nrs + r] = d->s_arr[r * 3 + c];
        int cs[4] = {0, 0, 0, 0};
        for (int c = 0; c < nc; ++c) { cs[c] = d->s_cov_sp[r * 4 + c]; sce[(size_t)c * nrs + r] = d->s_cov_eps[r * 4 + c]; }
        scs[r] = pack4(cs, 4);
        int g = -1;
        for (int e = 0; e < nf; ++e) if (d->s_f[r * 6 + e] < ng) g = d->s_f[r * 6 + e];
        if (d->s_stick[r] && g < 0) { delete m; return fail(BR_ERR_INPUT, "sticking reaction without gas reactant"); }
        sx_info[r] = (uint32_t)(nf | (np << 3) | ((d->s_stick[r] ? 1 : 0) << 6) | (nc << 7) | ((g < 0 ? 0 : g) << 10));
    }
    // ---- Jacobian column lists: reactions whose rate depends on component j
    std::vector<int> colptr(1, 0), colrx;
    for (int j = 0; j < n; ++j) {
        std::vector<int> rs;
        for (int i = 0; i < nrg; ++i) {
            const int r = perm[i];
            bool dep = false;
            for (int e = 0; e < d->g_nf[r]; ++e) dep |= d->g_f[r * 4 + e] == j;
            for (int e = 0; e < d->g_nr[r]; ++e) dep |= d->g_r[r * 4 + e] == j;
            if (d->g_tb[r] && j < ng && d->g_eff[(size_t)r * ng + j] != 0.0) dep = true;
            if (dep) rs.push_back(i);
        }
        for (int r = 0; r < nrs; ++r) {
            bool dep = false;
            for (int e = 0; e < d->s_nf[r]; ++e) dep |= d->s_f[r * 6 + e] == j;
            for (int c = 0; c < d->s_ncov[r]; ++c) dep |= d->s_cov_sp[r * 4 + c] == j;
            if (dep) rs.push_back(nrg + r);
        }
        for (int r : rs) colrx.push_back(r);
        colptr.push_back((int)colrx.size());
    }
    // ---- packed LDS table image
    M.tab_words = tab_words(nrg, nrs, ntb, M.ntbe);
    std::vector<uint32_t> tab(M.tab_words, 0);
    {
        size_t o = 0;
        auto put = [&](const std::vector<uint32_t>& v) { for (uint32_t x : v) tab[o++] = x; };
        put(rx_sp); put(rx_pr); put(rx_info); put(rx_sc); put(sx_sp); put(sx_pr); put(sx_info); put(sx_sc);
        std::vector<uint32_t> tp(tbptr.begin(), tbptr.end());
        put(tp); put(tbsp);
    }
    if (tbeff.empty()) tbeff.push_back(0.0);
    if (tbde.empty()) tbde.push_back(0.0);
    if (colrx.empty()) colrx.push_back(0);
    int rc = 0;
    rc |= upload(m, tab, &M.tab); rc |= upload(m, tbde, &M.tab_d);
    rc |= upload(m, molwt, &M.molwt); rc |= upload(m, sigma, &M.sigma); rc |= upload(m, nasa, &M.nasa);
    rc |= upload(m, garr, &M.g_arr); rc |= upload(m, gkcs, &M.g_kcs); rc |= upload(m, gdnu, &M.g_dnu);
    rc |= upload(m, folow, &M.fo_low); rc |= upload(m, fotroe, &M.fo_troe); rc |= upload(m, fontroe, &M.fo_ntroe);
    rc |= upload(m, tbeff, &M.tb_eff);
    rc |= upload(m, sarr, &M.s_arr); rc |= upload(m, scs, &M.s_cov_sp); rc |= upload(m, sce, &M.s_cov_eps);
    rc |= upload(m, colptr, &M.col_ptr); rc |= upload(m, colrx, &M.col_rx);
    if (rc) { br_mech_destroy(m); return rc; }
    // ---- reactors (waves) per workgroup: the value that maximises resident waves per CU,
    //      from the occupancy calculator (VGPRs, LDS: tables once per workgroup + one block
    //      per reactor); ties go to the smaller workgroup
    const void* kfn = m->nmax == 16 ? (const void*)k_integrate<16>
                    : m->nmax == 32 ? (const void*)k_integrate<32>
                    : m->nmax == 56 ? (const void*)k_integrate<56> : (const void*)k_integrate<64>;
    int best = 0, best_w = 0;
    for (int rpb = 1; rpb <= 4; ++rpb) {
        const size_t b = wg_lds_bytes(M, rpb);
        if (b > 160 * 1024) break;
        if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b) != hipSuccess) break;
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, 64 * rpb, b) != hipSuccess) break;
        if (nb * rpb > best_w) { best_w = nb * rpb; best = rpb; }
    }
    if (best_w == 0) { br_mech_destroy(m); return fail(BR_ERR_UNSUPPORTED, "mechanism too large for LDS"); }
    m->rpb = best;
    m->waves_per_cu = best_w;
    m->shmem = wg_lds_bytes(M, best);
    m->shmem1 = wg_lds_bytes(M, 1);
    HIPCHK(hipEventCreate(&m->ev0));
    HIPCHK(hipEventCreate(&m->ev1));
    *out = m;
    return 0;
}

int br_mech_destroy(br_mech* m) {
    if (!m) return 0;
    hipSetDevice(m->device);
    for (void* p : m->allocs) hipFree(p);
    if (m->ws) hipFree(m->ws);
    if (m->jws) hipFree(m->jws);
    if (m->ev0) hipEventDestroy(m->ev0);
    if (m->ev1) hipEventDestroy(m->ev1);
    delete m;
    return 0;
}

static int ensure_ws(br_mech* m, size_t bytes) {
    if (m->ws_bytes >= bytes) return 0;
    if (m->ws) hipFree(m->ws);
    m->ws = nullptr; m->ws_bytes = 0;
    HIPCHK(hipMalloc(&m->ws, bytes));
    m->ws_bytes = bytes;
    return 0;
}
static int ensure_jws(br_mech* m, int N) {
    const size_t bytes = (size_t)N * std::max(2 * m->nmax, 64) * WAVE * sizeof(double);
    if (m->jws_bytes >= bytes) return 0;
    if (m->jws) hipFree(m->jws);
    m->jws = nullptr; m->jws_bytes = 0;
    HIPCHK(hipMalloc((void**)&m->jws, bytes));
    m->jws_bytes = bytes;
    return 0;
}

int br_rates(br_mech* m, int N, const double* T, const double* p, const double* x, const double* theta, double* wdot,
             double* sdot) {
    if (!m || N < 0 || !T || !p || !x || !wdot) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    const int ng = m->ng, ns = m->ns, n = m->n;
    const size_t b_in = (size_t)N * (2 + ng + ns), b_out = (size_t)N * (ng + n);
    int rc = ensure_ws(m, (b_in + b_out) * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dp = dT + N;
    double* dx = dp + N;
    double* dth = dx + (size_t)N * ng;
    double* dw = dth + (size_t)N * ns;
    double* ds = dw + (size_t)N * ng;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dp, p, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dx, x, (size_t)N * ng * sizeof(double), hipMemcpyHostToDevice));
    if (ns && theta) HIPCHK(hipMemcpy(dth, theta, (size_t)N * ns * sizeof(double), hipMemcpyHostToDevice));
    else if (ns) HIPCHK(hipMemset(dth, 0, (size_t)N * ns * sizeof(double)));
    HIPCHK(hipFuncSetAttribute((const void*)k_rates, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
    hipLaunchKernelGGL(k_rates, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, dp, dx, ns ? dth : nullptr, dw, ds);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(wdot, dw, (size_t)N * ng * sizeof(double), hipMemcpyDeviceToHost));
    if (sdot) HIPCHK(hipMemcpy(sdot, ds, (size_t)N * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int br_rhs(br_mech* m, int N, const double* T, const double* Asv, const double* u, double* du) {
    if (!m || N < 0 || !T || !u || !du) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    const int n = m->n;
    int rc = ensure_ws(m, ((size_t)N * (2 + 2 * n)) * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* du_ = dA + N;
    double* ddu = du_ + (size_t)N * n;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipFuncSetAttribute((const void*)k_rhs, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
    hipLaunchKernelGGL(k_rhs, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, Asv ? dA : nullptr, du_, ddu);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(du, ddu, (size_t)N * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int br_jacobian(br_mech* m, int N, const double* T, const double* Asv, const double* u, double* J) {
    if (!m || N < 0 || !T || !u || !J) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    const int n = m->n;
    int rc = ensure_ws(m, ((size_t)N * (2 + n + (size_t)n * n)) * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* du_ = dA + N;
    double* dJ = du_ + (size_t)N * n;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    const double* pA = Asv ? dA : nullptr;
    rc = ensure_jws(m, N);
    if (rc) return rc;
    HIPCHK(hipFuncSetAttribute((const void*)k_jac<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
    hipLaunchKernelGGL(k_jac<64>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, pA, du_, dJ, m->jws);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(J, dJ, (size_t)N * n * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

static int integrate_dev(br_mech* m, int N, const double* dT, const double* dAsv, double* du, const double* dtf,
                         const br_opts* opts, br_stats* dstats, void* stream, double* trace) {
    if (!m || N < 0 || !dT || !du || !dtf) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    int rc = ensure_jws(m, N);
    if (rc) return rc;
    KOpts o;
    o.rtol = (opts && opts->rtol > 0) ? opts->rtol : 1e-6;
    o.atol = (opts && opts->atol > 0) ? opts->atol : 1e-10;
    o.max_steps = (opts && opts->max_steps > 0) ? opts->max_steps : 100000;
    o.hmax_inv = (opts && opts->hmax > 0) ? 1.0 / opts->hmax : 0.0;
    o.trace_cap = (opts && trace) ? opts->trace_cap : 0;
    o.ufac = (opts && opts->unstable_factor != 0.0) ? opts->unstable_factor : 10.0;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipEventRecord(m->ev0, s));
    const int rpb = m->rpb;
    const dim3 grid((N + rpb - 1) / rpb), block(64 * rpb);
    if (m->nmax == 16) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<16>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else if (m->nmax == 32) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<32>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else if (m->nmax == 56) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<56>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<56>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<64>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(m->ev1, s));
    m->ev_recorded = true;
    return 0;
}

int br_integrate_dev(br_mech* m, int N, const double* dT, const double* dAsv, double* du, const double* dtf,
                     const br_opts* opts, br_stats* dstats, void* stream) {
    return integrate_dev(m, N, dT, dAsv, du, dtf, opts, dstats, stream, nullptr);
}

int br_last_kernel_ms(br_mech* m, double* ms) {
    if (!m || !ms || !m->ev_recorded) return fail(BR_ERR_INPUT, "no kernel recorded");
    HIPCHK(hipEventSynchronize(m->ev1));
    float f = 0.f;
    HIPCHK(hipEventElapsedTime(&f, m->ev0, m->ev1));
    *ms = (double)f;
    return 0;
}

static int integrate_host(br_mech* m, int N, const double* T, const double* Asv, double* u, const double* tf,
                          const br_opts* opts, br_stats* stats, double* trace) {
    if (!m || N < 0 || !T || !u || !tf) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    const int n = m->n;
    const int cap = (trace && opts) ? opts->trace_cap : 0;
    if (trace && cap <= 0) return fail(BR_ERR_INPUT, "trace_cap must be > 0");
    const size_t ntr = trace ? (size_t)N * (cap + 1) * (n + 4) : 0;
    const size_t nd = (size_t)N * (3 + n + BR_NSTAT) + ntr;
    int rc = ensure_ws(m, nd * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* dtf = dA + N;
    double* du_ = dtf + N;
    double* dst = du_ + (size_t)N * n;
    double* dtr = dst + (size_t)N * BR_NSTAT;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dtf, tf, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    if (trace) HIPCHK(hipMemset(dtr, 0, ntr * sizeof(double)));
    rc = integrate_dev(m, N, dT, Asv ? dA : nullptr, du_, dtf, opts, (br_stats*)dst, nullptr, trace ? dtr : nullptr);
    if (rc) return rc;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(u, du_, (size_t)N * n * sizeof(double), hipMemcpyDeviceToHost));
    if (stats) HIPCHK(hipMemcpy(stats, dst, (size_t)N * BR_NSTAT * sizeof(double), hipMemcpyDeviceToHost));
    if (trace) HIPCHK(hipMemcpy(trace, dtr, ntr * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int br_integrate(br_mech* m, int N, const double* T, const double* Asv, double* u, const double* tf,
                 const br_opts* opts, br_stats* stats) {
    return integrate_host(m, N, T, Asv, u, tf, opts, stats, nullptr);
}

int br_integrate_traced(br_mech* m, int N, const double* T, const double* Asv, double* u, const double* tf,
                        const br_opts* opts, br_stats* stats, double* trace) {
    return integrate_host(m, N, T, Asv, u, tf, opts, stats, trace);
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// dense-solver check: factor (I - gamma*J) with the row-per-lane LU of the integrator and
// solve one right-hand side per matrix. J[N][n][n] row-major, b/x [N][n].
// ------------------------------------------------------------------------------------
namespace {
template <int NMAX>
__global__ __launch_bounds__(64) void k_lu_check(int N, int n, const double* J, const double* g, const double* b,
                                                 double* x, double* ws, int* fail) {
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    double* Jt = ws + (size_t)rid * 2 * NMAX * WAVE;
    double* LU = Jt + NMAX * WAVE;
    for (int j = 0; j < NMAX; ++j) Jt[j * WAVE + lane] = (lane < n && j < n) ? J[((size_t)rid * n + lane) * n + j] : 0.0;
    __shared__ int ps[64];
    const int f = lu_factor_mem<NMAX>(Jt, LU, g[rid], n, lane, &ps[lane]);
    const double r = lu_solve_mem<NMAX>(LU, n, lane, ps[lane], lane < n ? b[(size_t)rid * n + lane] : 0.0);
    if (lane < n) x[(size_t)rid * n + lane] = r;
    if (lane == 0) fail[rid] = f;
}
}  // namespace

extern "C" int br_debug_lu_solve(int N, int n, const double* J, const double* gamma, const double* b, double* x,
                                 int* fail_out) {
    if (N <= 0 || n <= 0 || n > 64) return fail_code_input();
    const int nmax = n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 56 ? 56 : 64));
    double *dJ, *dg, *db, *dx, *dws;
    int* df;
    HIPCHK(hipMalloc(&dJ, (size_t)N * n * n * 8));
    HIPCHK(hipMalloc(&dg, (size_t)N * 8));
    HIPCHK(hipMalloc(&db, (size_t)N * n * 8));
    HIPCHK(hipMalloc(&dx, (size_t)N * n * 8));
    HIPCHK(hipMalloc(&dws, (size_t)N * 2 * nmax * WAVE * 8));
    HIPCHK(hipMalloc(&df, (size_t)N * 4));
    HIPCHK(hipMemcpy(dJ, J, (size_t)N * n * n * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dg, gamma, (size_t)N * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(db, b, (size_t)N * n * 8, hipMemcpyHostToDevice));
    if (nmax == 16) hipLaunchKernelGGL(k_lu_check<16>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else if (nmax == 32) hipLaunchKernelGGL(k_lu_check<32>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else if (nmax == 56) hipLaunchKernelGGL(k_lu_check<56>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else hipLaunchKernelGGL(k_lu_check<64>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(x, dx, (size_t)N * n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(fail_out, df, (size_t)N * 4, hipMemcpyDeviceToHost));
    hipFree(dJ); hipFree(dg); hipFree(db); hipFree(dx); hipFree(dws); hipFree(df);
    return 0;
}
