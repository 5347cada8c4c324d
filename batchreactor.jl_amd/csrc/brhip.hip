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
    double rtol, atol, hmax_inv;
    int max_steps;
};

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

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
    return v;
}

// ------------------------------------------------------------------------------------
// the integrator: one reactor per 64-lane workgroup
// ------------------------------------------------------------------------------------
template <int NMAX>
__global__ __launch_bounds__(64) void k_integrate(DevMech M, int N, const double* __restrict__ Tv,
                                                  const double* __restrict__ Asvv, double* __restrict__ U,
                                                  const double* __restrict__ tfv, KOpts o,
                                                  double* __restrict__ stats, double* __restrict__ Jws) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    const int n = M.n;
    const bool act = lane < n;
    Smem S = carve(smem, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    const double tstop = tfv[rid];
    const double Mk = act ? M.molwt[lane] : 1.0;
    double* Jsave = Jws + (size_t)rid * NMAX * WAVE;

    init_tconst(M, S, T, lane);

    // Nordsieck history and work vectors (this lane's component)
    double z[QMAX + 1];
#pragma unroll
    for (int j = 0; j <= QMAX; ++j) z[j] = 0.0;
    double ewt = 1.0, acor = 0.0, y = 0.0, ftemp = 0.0, delta = 0.0, tempv = 0.0;
    double a[NMAX];
    int pstep = -1;
    // uniform controller state
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
#pragma unroll
    for (int i = 0; i < QMAX + 2; ++i) tau[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) tq[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
    double tn = 0.0, h = 0.0, hprime = 0.0, hscale = 0.0, eta = 1.0, etamax = ETAMX1;
    double rl1 = 0.0, gamma = 0.0, gammap = 0.0, gamrat = 1.0, crate = 1.0, delp = 0.0, acnrm = 0.0;
    double saved_tq5 = 0.0;
    int q = 1, qprime = 1, L = 2, qwait = 2;
    int nst = 0, nfe = 0, nsetups = 0, nje = 0, nni = 0, ncfn = 0, netf = 0, nstlp = 0, nstlj = 0;
    int jcur = 0;
    double p_last = 0.0, x_last = 0.0;
    const double hmin = 0.0;

    z[0] = act ? U[(size_t)rid * n + lane] : 0.0;

    auto F = [&](double yv) __attribute__((always_inline)) -> double { return rhs(M, S, T, Asv, Asv_th, yv, lane, Mk, p_last, x_last); };
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
#pragma unroll
            for (int j = 0; j < NMAX; ++j) a[j] = Jsave[j * WAVE + lane];
        } else {
            jcur = 1; nje++; nstlj = nst;
            jacobian<NMAX>(M, S, T, Asv, Asv_th, y, lane, Mk, a);
#pragma unroll
            for (int j = 0; j < NMAX; ++j) Jsave[j * WAVE + lane] = a[j];
        }
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            a[j] *= -gamma;
            if (j == lane) a[j] += 1.0;
        }
        return lu_factor<NMAX>(a, n, lane, pstep, S.pivl);
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
            delta = lu_solve<NMAX>(a, n, lane, pstep, S.pivl, delta);
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
        double* st = stats + (size_t)rid * 8;
        st[0] = (double)nst; st[1] = (double)nfe; st[2] = (double)nje; st[3] = (double)nsetups;
        st[4] = (double)nni; st[5] = (double)ncfn; st[6] = (double)netf; st[7] = (double)status;
    }
}

// ------------------------------------------------------------------------------------
// parity kernels: rates, rhs, jacobian (one reactor per wave)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_rates(DevMech M, int N, const double* Tv, const double* pv, const double* X,
                                              const double* TH, double* W, double* SD) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    Smem S = carve(smem, M);
    const double T = Tv[rid], p = pv[rid];
    init_tconst(M, S, T, lane);
    double c = 0.0;
    if (lane < M.ng) c = p * X[(size_t)rid * M.ng + lane] / (R_GAS * T);
    else if (lane < M.n) c = TH ? TH[(size_t)rid * M.ns + (lane - M.ng)] : 0.0;
    if (lane < M.n) S.conc[lane] = c;
    const double Ctot = wave_sum(lane < M.ng ? c : 0.0);
    __syncthreads();
    third_body(M, S, Ctot, lane);
    __syncthreads();
    rates_of_progress(M, S, R_GAS * T, lane);
    __syncthreads();
    double w, s;
    gather(M, S, lane, w, s);
    if (lane < M.ng) W[(size_t)rid * M.ng + lane] = w;
    if (SD && lane < M.n) SD[(size_t)rid * M.n + lane] = s;
}

__global__ __launch_bounds__(64) void k_rhs(DevMech M, int N, const double* Tv, const double* Asvv, const double* U,
                                            double* DU) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    Smem S = carve(smem, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst(M, S, T, lane);
    const bool act = lane < M.n;
    const double u = act ? U[(size_t)rid * M.n + lane] : 0.0;
    const double Mk = act ? M.molwt[lane] : 1.0;
    double p, x;
    const double du = rhs(M, S, T, Asv, Asv_th, u, lane, Mk, p, x);
    if (act) DU[(size_t)rid * M.n + lane] = du;
}

template <int NMAX>
__global__ __launch_bounds__(64) void k_jac(DevMech M, int N, const double* Tv, const double* Asvv, const double* U,
                                            double* J) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    Smem S = carve(smem, M);
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst(M, S, T, lane);
    const bool act = lane < M.n;
    const double u = act ? U[(size_t)rid * M.n + lane] : 0.0;
    const double Mk = act ? M.molwt[lane] : 1.0;
    double a[NMAX];
    jacobian<NMAX>(M, S, T, Asv, Asv_th, u, lane, Mk, a);
    if (act) {
        double* row = J + ((size_t)rid * M.n + lane) * M.n;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) if (j < M.n) row[j] = a[j];
    }
}

}  // namespace

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
struct br_mech {
    int device = 0;
    int ng = 0, ns = 0, nrg = 0, nrs = 0, n = 0, nmax = 64;
    DevMech dm{};
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

int br_version(void) { return 100; }
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
    HIPCHK(hipSetDevice(device));
    br_mech* m = new br_mech();
    m->device = device; m->ng = ng; m->ns = ns; m->nrg = nrg; m->nrs = nrs; m->n = n;
    m->nmax = n <= 16 ? 16 : (n <= 32 ? 32 : 64);
    DevMech& M = m->dm;
    M.ng = ng; M.ns = ns; M.n = n; M.nrg = nrg; M.nrs = nrs; M.conv = d->conv;
    M.p_std = d->p_std > 0 ? d->p_std : 1e5;
    M.G = d->site_density * 1e4;
    std::vector<double> molwt(n, 1.0), sigma(n, 1.0), nasa((size_t)ng * 15);
    for (int k = 0; k < ng; ++k) molwt[k] = d->molwt[k];
    for (int i = 0; i < ns; ++i) sigma[ng + i] = d->sigma ? d->sigma[i] : 1.0;
    for (size_t i = 0; i < (size_t)ng * 15; ++i) nasa[i] = d->nasa[i];
    // gas tables (SoA)
    std::vector<int> gf(4 * (size_t)nrg, 0), gr(4 * (size_t)nrg, 0), ginfo(nrg), gdnu(nrg);
    std::vector<double> garr(3 * (size_t)nrg), gkcs(nrg, 1.0);
    std::vector<double> folow, fotroe;
    std::vector<int> fontroe;
    std::vector<int> tbptr(1, 0), tbsp;
    std::vector<double> tbde, tbeff;
    int ntb = 0, nfo = 0;
    std::vector<int> fo_of(nrg, -1);
    for (int r = 0; r < nrg; ++r) if (d->g_tb[r] == 2) fo_of[r] = nfo++;
    folow.assign(3 * (size_t)std::max(nfo, 1), 0.0);
    fotroe.assign(4 * (size_t)std::max(nfo, 1), 0.0);
    fontroe.assign(std::max(nfo, 1), 0);
    for (int r = 0; r < nrg; ++r) {
        const int nf = d->g_nf[r], nr = d->g_nr[r], tb = d->g_tb[r];
        if (nf > 4 || nr > 4 || nf < 1) { delete m; return fail(BR_ERR_UNSUPPORTED, "reaction with >4 entries"); }
        for (int e = 0; e < 4; ++e) {
            gf[(size_t)e * nrg + r] = e < nf ? d->g_f[r * 4 + e] : 0;
            gr[(size_t)e * nrg + r] = e < nr ? d->g_r[r * 4 + e] : 0;
        }
        for (int c = 0; c < 3; ++c) garr[(size_t)c * nrg + r] = d->g_arr[r * 3 + c];
        gdnu[r] = nr - nf;
        if ((d->conv & BR_CONV_KC_UNIT_SLIP) && tb != 2) gkcs[r] = std::pow(1e6, (double)(nr - nf));
        int tbidx = 0, foidx = 0;
        if (tb) {
            tbidx = ntb++;
            for (int k = 0; k < ng; ++k) {
                const double e = d->g_eff[(size_t)r * ng + k];
                if (e != 1.0) { tbsp.push_back(k); tbde.push_back(e - 1.0); }
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
        ginfo[r] = nf | (nr << 3) | ((d->g_rev[r] ? 1 : 0) << 6) | (tb << 7) | (tbidx << 9) | (foidx << 19);
    }
    M.ntb = ntb; M.nfo = nfo;
    // surface tables
    std::vector<int> sf(6 * (size_t)std::max(nrs, 1), 0), sinfo(std::max(nrs, 1), 0), sgas(std::max(nrs, 1), 0);
    std::vector<int> scs(4 * (size_t)std::max(nrs, 1), 0);
    std::vector<double> sarr(3 * (size_t)std::max(nrs, 1), 0.0), sce(4 * (size_t)std::max(nrs, 1), 0.0);
    for (int r = 0; r < nrs; ++r) {
        const int nf = d->s_nf[r], np = d->s_np[r], nc = d->s_ncov[r];
        if (nf > 6 || np > 6 || nc > 4) { delete m; return fail(BR_ERR_UNSUPPORTED, "surface reaction too large"); }
        for (int e = 0; e < 6; ++e) sf[(size_t)e * nrs + r] = e < nf ? d->s_f[r * 6 + e] : 0;
        for (int c = 0; c < 3; ++c) sarr[(size_t)c * nrs + r] = d->s_arr[r * 3 + c];
        for (int c = 0; c < 4; ++c) {
            scs[(size_t)c * nrs + r] = c < nc ? d->s_cov_sp[r * 4 + c] : 0;
            sce[(size_t)c * nrs + r] = c < nc ? d->s_cov_eps[r * 4 + c] : 0.0;
        }
        int g = -1;
        for (int e = 0; e < nf; ++e) if (d->s_f[r * 6 + e] < ng) g = d->s_f[r * 6 + e];
        if (d->s_stick[r] && g < 0) { delete m; return fail(BR_ERR_INPUT, "sticking reaction without gas reactant"); }
        sgas[r] = g < 0 ? 0 : g;
        sinfo[r] = nf | (np << 3) | ((d->s_stick[r] ? 1 : 0) << 6) | (nc << 7);
    }
    // species production ELL (net stoichiometry, reaction order)
    std::vector<std::vector<std::pair<int, double>>> lists(n);
    for (int r = 0; r < nrg; ++r) {
        std::vector<std::pair<int, double>> nu;
        auto add = [&](int s, double v) __attribute__((always_inline)) {
            for (auto& p : nu) if (p.first == s) { p.second += v; return; }
            nu.push_back({s, v});
        };
        for (int e = 0; e < d->g_nf[r]; ++e) add(d->g_f[r * 4 + e], -1.0);
        for (int e = 0; e < d->g_nr[r]; ++e) add(d->g_r[r * 4 + e], 1.0);
        for (auto& p : nu) if (p.second != 0.0) lists[p.first].push_back({r, p.second});
    }
    for (int r = 0; r < nrs; ++r) {
        std::vector<std::pair<int, double>> nu;
        auto add = [&](int s, double v) __attribute__((always_inline)) {
            for (auto& p : nu) if (p.first == s) { p.second += v; return; }
            nu.push_back({s, v});
        };
        for (int e = 0; e < d->s_nf[r]; ++e) add(d->s_f[r * 6 + e], -1.0);
        for (int e = 0; e < d->s_np[r]; ++e) add(d->s_p[r * 6 + e], 1.0);
        for (auto& p : nu) if (p.second != 0.0) lists[p.first].push_back({nrg + r, p.second});
    }
    int ell = 0;
    for (auto& v : lists) ell = std::max<int>(ell, (int)v.size());
    std::vector<int> ellr((size_t)std::max(ell, 1) * n, -1);
    std::vector<double> ellnu((size_t)std::max(ell, 1) * n, 0.0);
    for (int k = 0; k < n; ++k)
        for (size_t i = 0; i < lists[k].size(); ++i) {
            ellr[i * n + k] = lists[k][i].first;
            ellnu[i * n + k] = lists[k][i].second;
        }
    M.ell_len = ell;
    if (tbeff.empty()) tbeff.push_back(0.0);
    int rc = 0;
    rc |= upload(m, molwt, &M.molwt); rc |= upload(m, sigma, &M.sigma); rc |= upload(m, nasa, &M.nasa);
    rc |= upload(m, gf, &M.g_f); rc |= upload(m, gr, &M.g_r); rc |= upload(m, ginfo, &M.g_info);
    rc |= upload(m, garr, &M.g_arr); rc |= upload(m, gkcs, &M.g_kcs); rc |= upload(m, gdnu, &M.g_dnu);
    rc |= upload(m, folow, &M.fo_low); rc |= upload(m, fotroe, &M.fo_troe); rc |= upload(m, fontroe, &M.fo_ntroe);
    rc |= upload(m, tbptr, &M.tb_ptr); rc |= upload(m, tbsp, &M.tb_sp); rc |= upload(m, tbde, &M.tb_de);
    rc |= upload(m, tbeff, &M.tb_eff);
    rc |= upload(m, sf, &M.s_f); rc |= upload(m, sinfo, &M.s_info); rc |= upload(m, sarr, &M.s_arr);
    rc |= upload(m, sgas, &M.s_gas); rc |= upload(m, scs, &M.s_cov_sp); rc |= upload(m, sce, &M.s_cov_eps);
    rc |= upload(m, ellr, &M.ell_r); rc |= upload(m, ellnu, &M.ell_nu);
    if (rc) { br_mech_destroy(m); return rc; }
    m->shmem = smem_bytes(ng, n, nrg, nrs, ntb, nfo);
    if (m->shmem > 64 * 1024) { br_mech_destroy(m); return fail(BR_ERR_UNSUPPORTED, "mechanism too large for LDS"); }
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
    const size_t bytes = (size_t)N * m->nmax * WAVE * sizeof(double);
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
    hipLaunchKernelGGL(k_rates, dim3(N), dim3(64), m->shmem, 0, m->dm, N, dT, dp, dx, ns ? dth : nullptr, dw, ds);
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
    hipLaunchKernelGGL(k_rhs, dim3(N), dim3(64), m->shmem, 0, m->dm, N, dT, Asv ? dA : nullptr, du_, ddu);
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
    if (m->nmax == 16) hipLaunchKernelGGL(k_jac<16>, dim3(N), dim3(64), m->shmem, 0, m->dm, N, dT, pA, du_, dJ);
    else if (m->nmax == 32) hipLaunchKernelGGL(k_jac<32>, dim3(N), dim3(64), m->shmem, 0, m->dm, N, dT, pA, du_, dJ);
    else hipLaunchKernelGGL(k_jac<64>, dim3(N), dim3(64), m->shmem, 0, m->dm, N, dT, pA, du_, dJ);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(J, dJ, (size_t)N * n * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int br_integrate_dev(br_mech* m, int N, const double* dT, const double* dAsv, double* du, const double* dtf,
                     const br_opts* opts, br_stats* dstats, void* stream) {
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
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipEventRecord(m->ev0, s));
    if (m->nmax == 16)
        hipLaunchKernelGGL(k_integrate<16>, dim3(N), dim3(64), m->shmem, s, m->dm, N, dT, dAsv, du, dtf, o, (double*)dstats, m->jws);
    else if (m->nmax == 32)
        hipLaunchKernelGGL(k_integrate<32>, dim3(N), dim3(64), m->shmem, s, m->dm, N, dT, dAsv, du, dtf, o, (double*)dstats, m->jws);
    else
        hipLaunchKernelGGL(k_integrate<64>, dim3(N), dim3(64), m->shmem, s, m->dm, N, dT, dAsv, du, dtf, o, (double*)dstats, m->jws);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(m->ev1, s));
    m->ev_recorded = true;
    return 0;
}

int br_last_kernel_ms(br_mech* m, double* ms) {
    if (!m || !ms || !m->ev_recorded) return fail(BR_ERR_INPUT, "no kernel recorded");
    HIPCHK(hipEventSynchronize(m->ev1));
    float f = 0.f;
    HIPCHK(hipEventElapsedTime(&f, m->ev0, m->ev1));
    *ms = (double)f;
    return 0;
}

int br_integrate(br_mech* m, int N, const double* T, const double* Asv, double* u, const double* tf,
                 const br_opts* opts, br_stats* stats) {
    if (!m || N < 0 || !T || !u || !tf) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    const int n = m->n;
    const size_t nd = (size_t)N * (3 + n + 8);
    int rc = ensure_ws(m, nd * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* dtf = dA + N;
    double* du_ = dtf + N;
    double* dst = du_ + (size_t)N * n;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dtf, tf, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    rc = br_integrate_dev(m, N, dT, Asv ? dA : nullptr, du_, dtf, opts, (br_stats*)dst, nullptr);
    if (rc) return rc;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(u, du_, (size_t)N * n * sizeof(double), hipMemcpyDeviceToHost));
    if (stats) HIPCHK(hipMemcpy(stats, dst, (size_t)N * 8 * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
