// host_cvode.cpp -- br_integrate_host (include/brhip.h): CVODE_BDF() on the CPU with a caller-supplied
// right-hand side, for the reference's user-defined-chemistry path.
//
// The reference integrates residual! with solve(prob, CVODE_BDF(), reltol=1e-6, abstol=1e-10,
// save_everystep=false, callback=FunctionCallingCallback(save_data)) whatever the chemistry
// (src/BatchReactor.jl:204-210); with userchem the RHS is the user's Julia function (:358-360,
// :371-372), which cannot run inside a HIP kernel. This file is the same CVODE 5.x restatement as the
// device engine (brhip.hip: Nordsieck BDF orders 1..5, cvHin, modified Newton with maxcor 3, msbp 20,
// msbj 51, dgmax 0.3 / 0.2, WRMS error test, order selection, tstop) with CVODE's difference-quotient
// Jacobian (cvLsDenseDQJac, the reference's own setting: no Jacobian is supplied) and SUNDIALS'
// denseGETRF / denseGETRS, written for one reactor on the host: the Python host (ctypes) and the Julia
// host (@cfunction) drive the user's function through the same solver and write the same rows.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/brhip.h"

namespace {

constexpr int QMAX = 5, LMAX = QMAX + 1;
constexpr double HLB_FACTOR = 100.0, HUB_FACTOR = 0.1, H_BIAS = 0.5;
constexpr int MAX_ITERS = 4;
constexpr double ETAMX1 = 10000.0, ETAMX2 = 10.0, ETAMX3 = 10.0, ETAMXF = 0.2, ETAMIN = 0.1, ETACF = 0.25;
constexpr double ADDON = 1e-6, BIAS1 = 6.0, BIAS2 = 6.0, BIAS3 = 10.0, ONEPSM = 1.000001;
constexpr int SMALL_NST = 10, MXNCF = 10, MXNEF = 7, MXNEF1 = 3, SMALL_NEF = 2, LONG_WAIT = 10;
constexpr int NLS_MAXCOR = 3, MSBP = 20, LS_MSBJ = 51;
constexpr double CRDOWN = 0.3, DGMAX = 0.3, RDIV = 2.0, CORTES = 0.1, THRESH = 1.5, FUZZ = 100.0, LS_DGMAX = 0.2;
constexpr double MIN_INC_MULT = 1000.0;
constexpr double UROUND = DBL_EPSILON;
enum { FIRST_CALL, PREV_CONV_FAIL, PREV_ERR_FAIL };
enum { NO_FAILURES, FAIL_BAD_J, FAIL_OTHER };

struct HostCvode {
    int n;
    br_rhs_fn f;
    void* user;
    double rtol, atol;
    std::vector<double> zn[LMAX + 1];
    std::vector<double> ewt, y, acor, tempv, ftemp, delta, savedJ, A, fdq;
    std::vector<int> piv;
    double tn = 0, h = 0, hprime = 0, hscale = 0, eta = 1, etamax = ETAMX1, hmin = 0, hu = 0, tstop = 0;
    double tau[LMAX + 1] = {}, tq[6] = {}, l[LMAX] = {};
    double rl1 = 0, gamma = 0, gammap = 0, gamrat = 1, crate = 1, delp = 0, acnrm = 0, saved_tq5 = 0;
    double etaq = 0, etaqm1 = 0, etaqp1 = 0;
    int q = 1, qprime = 1, L = 2, qwait = 2, indx_acor = QMAX;
    long nst = 0, nfe = 0, nsetups = 0, nje = 0, nni = 0, ncfn = 0, netf = 0, nstlp = 0, nstlj = 0, nfe_dq = 0;
    int jcur = 0;
    int rhs_fail = 0;   // the user's function returned non-zero

    HostCvode(int n_, br_rhs_fn f_, void* u_, double rt, double at) : n(n_), f(f_), user(u_), rtol(rt), atol(at) {
        for (auto& z : zn) z.assign(n, 0.0);
        for (auto* v : {&ewt, &y, &acor, &tempv, &ftemp, &delta, &fdq}) v->assign(n, 0.0);
        savedJ.assign((size_t)n * n, 0.0);
        A.assign((size_t)n * n, 0.0);
        piv.assign(n, 0);
    }
    double wrms(const double* x) const {
        double s = 0;
        for (int i = 0; i < n; ++i) { const double t = x[i] * ewt[i]; s += t * t; }
        return std::sqrt(s / n);
    }
    void rhs(const double* u, double* du) {
        if (f(user, tn, u, du) != 0) rhs_fail = 1;
    }
    void set_ewt(const double* u) {
        for (int i = 0; i < n; ++i) ewt[i] = 1.0 / (rtol * std::fabs(u[i]) + atol);
    }
    // SUNDIALS denseGETRF / denseGETRS, column-major a[j n + i]
    static int getrf(double* a, int n, int* p) {
        for (int k = 0; k < n; ++k) {
            double* ck = a + (size_t)k * n;
            int lp = k;
            for (int i = k + 1; i < n; ++i) if (std::fabs(ck[i]) > std::fabs(ck[lp])) lp = i;
            p[k] = lp;
            if (ck[lp] == 0.0) return k + 1;
            if (lp != k)
                for (int j = 0; j < n; ++j) std::swap(a[(size_t)j * n + lp], a[(size_t)j * n + k]);
            const double mult = 1.0 / ck[k];
            for (int i = k + 1; i < n; ++i) ck[i] *= mult;
            for (int j = k + 1; j < n; ++j) {
                double* cj = a + (size_t)j * n;
                const double akj = cj[k];
                if (akj != 0.0) for (int i = k + 1; i < n; ++i) cj[i] -= akj * ck[i];
            }
        }
        return 0;
    }
    static void getrs(const double* a, int n, const int* p, double* b) {
        for (int k = 0; k < n; ++k) if (p[k] != k) std::swap(b[k], b[p[k]]);
        for (int k = 0; k < n - 1; ++k) {
            const double* ck = a + (size_t)k * n;
            const double bk = b[k];
            for (int i = k + 1; i < n; ++i) b[i] -= ck[i] * bk;
        }
        for (int k = n - 1; k > 0; --k) {
            const double* ck = a + (size_t)k * n;
            b[k] /= ck[k];
            const double bk = b[k];
            for (int i = 0; i < k; ++i) b[i] -= ck[i] * bk;
        }
        b[0] /= a[0];
    }
    // cvLsDenseDQJac: column j = (f(y + inc_j e_j) - f(y)) / inc_j
    void dq_jac(const double* yv, const double* fy, double* Jc) {
        const double srur = std::sqrt(UROUND);
        const double fnorm = wrms(fy);
        const double mininc = fnorm != 0.0 ? MIN_INC_MULT * std::fabs(h) * UROUND * n * fnorm : 1.0;
        std::vector<double> yy(yv, yv + n);
        for (int j = 0; j < n; ++j) {
            const double ys = yy[j];
            const double inc = std::max(srur * std::fabs(ys), mininc / ewt[j]);
            yy[j] += inc;
            rhs(yy.data(), fdq.data());
            ++nfe_dq;
            yy[j] = ys;
            const double ii = 1.0 / inc;
            for (int i = 0; i < n; ++i) Jc[(size_t)j * n + i] = ii * fdq[i] - ii * fy[i];
        }
    }
    // cvLsSetup
    int ls_setup(int convfail, const double* ypred, const double* fpred) {
        const double dgamma = std::fabs(gamma / gammap - 1.0);
        const bool jbad = nst == 0 || nst > nstlj + LS_MSBJ || (convfail == FAIL_BAD_J && dgamma < LS_DGMAX) ||
                          convfail == FAIL_OTHER;
        if (!jbad) {
            jcur = 0;
            A = savedJ;
        } else {
            jcur = 1;
            ++nje;
            nstlj = nst;
            dq_jac(ypred, fpred, A.data());
            savedJ = A;
        }
        for (double& a : A) a *= -gamma;
        for (int i = 0; i < n; ++i) A[(size_t)i * n + i] += 1.0;
        return getrf(A.data(), n, piv.data());
    }
    void rescale() {
        double fac = eta;
        for (int j = 1; j <= q; ++j) {
            for (double& z : zn[j]) z *= fac;
            fac *= eta;
        }
        h = hscale * eta;
        hscale = h;
    }
    void predict() {
        tn += h;
        if ((tn - tstop) * h > 0) tn = tstop;
        for (int k = 1; k <= q; ++k)
            for (int j = q; j >= k; --j)
                for (int i = 0; i < n; ++i) zn[j - 1][i] += zn[j][i];
    }
    void restore(double saved_t) {
        tn = saved_t;
        for (int k = 1; k <= q; ++k)
            for (int j = q; j >= k; --j)
                for (int i = 0; i < n; ++i) zn[j - 1][i] -= zn[j][i];
    }
    // cvSetBDF + cvSetTqBDF
    void set_coeffs() {
        double xi_inv = 1.0, xistar_inv = 1.0;
        l[0] = l[1] = 1.0;
        for (int i = 2; i <= q; ++i) l[i] = 0.0;
        double alpha0 = -1.0, alpha0_hat = -1.0, hsum = h;
        if (q > 1) {
            for (int j = 2; j < q; ++j) {
                hsum += tau[j - 1];
                xi_inv = h / hsum;
                alpha0 -= 1.0 / j;
                for (int i = j; i >= 1; --i) l[i] += l[i - 1] * xi_inv;
            }
            alpha0 -= 1.0 / q;
            xistar_inv = -l[1] - alpha0;
            hsum += tau[q - 1];
            xi_inv = h / hsum;
            alpha0_hat = -l[1] - xi_inv;
            for (int i = q; i >= 1; --i) l[i] += l[i - 1] * xistar_inv;
        }
        const double A1 = 1.0 - alpha0_hat + alpha0, A2 = 1.0 + q * A1;
        tq[2] = std::fabs(A1 / (alpha0 * A2));
        tq[5] = std::fabs(A2 * xistar_inv / (l[q] * xi_inv));
        if (qwait == 1) {
            if (q > 1) {
                const double C = xistar_inv / l[q], A3 = alpha0 + 1.0 / q, A4 = alpha0_hat + xi_inv;
                tq[1] = std::fabs(C * ((1.0 - A4 + A3) / A3));
            } else {
                tq[1] = 1.0;
            }
            hsum += tau[q];
            xi_inv = h / hsum;
            const double A5 = alpha0 - 1.0 / (q + 1), A6 = alpha0_hat - xi_inv;
            tq[3] = std::fabs(((1.0 - A6 + A5) / A2) / (xi_inv * (q + 2) * A5));
        }
        tq[4] = CORTES / tq[2];
        rl1 = 1.0 / l[1];
        gamma = h * rl1;
        if (nst == 0) gammap = gamma;
        gamrat = nst > 0 ? gamma / gammap : 1.0;
    }
    void increase_order() {   // cvIncreaseBDF
        std::fill(l, l + LMAX, 0.0);
        l[2] = 1.0;
        double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = hscale;
        if (q > 1) {
            for (int j = 1; j < q; ++j) {
                hsum += tau[j + 1];
                const double xi = hsum / hscale;
                prod *= xi;
                alpha0 -= 1.0 / (j + 1);
                alpha1 += 1.0 / xi;
                for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xiold + l[i - 1];
                xiold = xi;
            }
        }
        const double A1 = (-alpha0 - alpha1) / prod;
        for (int i = 0; i < n; ++i) zn[q + 1][i] = A1 * zn[indx_acor][i];
        for (int j = 2; j <= q; ++j)
            for (int i = 0; i < n; ++i) zn[j][i] += l[j] * zn[q + 1][i];
    }
    void decrease_order() {   // cvDecreaseBDF
        std::fill(l, l + LMAX, 0.0);
        l[2] = 1.0;
        double hsum = 0.0;
        for (int j = 1; j <= q - 2; ++j) {
            hsum += tau[j];
            const double xi = hsum / hscale;
            for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xi + l[i - 1];
        }
        for (int j = 2; j < q; ++j)
            for (int i = 0; i < n; ++i) zn[j][i] -= l[j] * zn[q][i];
    }
    void adjust_order(int dq) {
        if (q == 2 && dq != 1) return;
        if (dq == 1) increase_order();
        else decrease_order();
    }
    void residual(const std::vector<double>& ycor) {
        for (int i = 0; i < n; ++i) y[i] = zn[0][i] + ycor[i];
        rhs(y.data(), ftemp.data());
        ++nfe;
        for (int i = 0; i < n; ++i) delta[i] = (rl1 * zn[1][i] + ycor[i]) - gamma * ftemp[i];
    }
    // SUNNonlinSol_Newton + cvNls: 0 converged, > 0 recoverable failure
    int newton(int nflag) {
        const int convfail = (nflag == FIRST_CALL || nflag == PREV_ERR_FAIL) ? NO_FAILURES : FAIL_OTHER;
        bool call_setup = nflag == PREV_CONV_FAIL || nflag == PREV_ERR_FAIL || nst == 0 || nst >= nstlp + MSBP ||
                          std::fabs(gamrat - 1.0) > DGMAX;
        std::vector<double>& ycor = acor;
        std::fill(ycor.begin(), ycor.end(), 0.0);
        const double tol = tq[4];
        bool jbad = false;
        for (;;) {
            residual(ycor);
            bool jc = false;
            if (call_setup) {
                const int lr = ls_setup(jbad ? FAIL_BAD_J : convfail, y.data(), ftemp.data());
                ++nsetups;
                jc = jcur != 0;
                gamrat = 1.0;
                gammap = gamma;
                crate = 1.0;
                nstlp = nst;
                if (lr) return 2;   // singular Newton matrix: recoverable
            }
            int ret = 0;
            for (int m = 0;;) {
                ++nni;
                for (double& d : delta) d = -d;
                getrs(A.data(), n, piv.data(), delta.data());
                if (gamrat != 1.0) {
                    const double s = 2.0 / (1.0 + gamrat);
                    for (double& d : delta) d *= s;
                }
                for (int i = 0; i < n; ++i) ycor[i] += delta[i];
                const double del = wrms(delta.data());
                if (m > 0) crate = std::max(CRDOWN * crate, del / delp);
                if (del * std::min(1.0, crate) / tol <= 1.0) {
                    acnrm = m == 0 ? del : wrms(ycor.data());
                    for (int i = 0; i < n; ++i) y[i] = zn[0][i] + ycor[i];
                    jcur = 0;
                    return 0;
                }
                if (m >= 1 && del > RDIV * delp) { ret = 1; break; }
                delp = del;
                if (++m >= NLS_MAXCOR) { ret = 1; break; }
                residual(ycor);
            }
            if (ret > 0 && !jc) {   // retry with a fresh Jacobian
                call_setup = true;
                jbad = true;
                std::fill(ycor.begin(), ycor.end(), 0.0);
                continue;
            }
            for (int i = 0; i < n; ++i) y[i] = zn[0][i] + ycor[i];
            return ret;
        }
    }
    void complete_step() {
        ++nst;
        hu = h;
        for (int i = q; i >= 2; --i) tau[i] = tau[i - 1];
        if (q == 1 && nst > 1) tau[2] = tau[1];
        tau[1] = h;
        for (int j = 0; j <= q; ++j)
            for (int i = 0; i < n; ++i) zn[j][i] += l[j] * acor[i];
        if (--qwait == 1 && q != QMAX) {
            zn[QMAX] = acor;
            saved_tq5 = tq[5];
            indx_acor = QMAX;
        }
    }
    void set_eta(double hmax_inv) {
        if (eta < THRESH) {
            eta = 1.0;
            hprime = h;
        } else {
            eta = std::min(eta, etamax);
            eta /= std::max(1.0, std::fabs(h) * hmax_inv * eta);
            hprime = h * eta;
        }
    }
    void prepare_next(double dsm, double hmax_inv) {   // cvPrepareNextStep + cvChooseEta
        if (etamax == 1.0) {
            qwait = std::max(qwait, 2);
            qprime = q;
            hprime = h;
            eta = 1.0;
            return;
        }
        etaq = 1.0 / (std::pow(BIAS2 * dsm, 1.0 / L) + ADDON);
        if (qwait != 0) {
            eta = etaq;
            qprime = q;
            set_eta(hmax_inv);
            return;
        }
        qwait = 2;
        etaqm1 = 0.0;
        if (q > 1) etaqm1 = 1.0 / (std::pow(BIAS1 * (wrms(zn[q].data()) * tq[1]), 1.0 / q) + ADDON);
        etaqp1 = 0.0;
        if (q != QMAX && saved_tq5 != 0.0) {
            const double cquot = (tq[5] / saved_tq5) * std::pow(h / tau[2], (double)L);
            for (int i = 0; i < n; ++i) tempv[i] = acor[i] - cquot * zn[QMAX][i];
            etaqp1 = 1.0 / (std::pow(BIAS3 * (wrms(tempv.data()) * tq[3]), 1.0 / (L + 1)) + ADDON);
        }
        const double etam = std::max(etaqm1, std::max(etaq, etaqp1));
        if (etam < THRESH) { eta = 1.0; qprime = q; }
        else if (etam == etaq) { eta = etaq; qprime = q; }
        else if (etam == etaqm1) { eta = etaqm1; qprime = q - 1; }
        else { eta = etaqp1; qprime = q + 1; zn[QMAX] = acor; }
        set_eta(hmax_inv);
    }
    // cvStep: 0 accepted, < 0 failure (CVODE flags)
    int step(double hmax_inv) {
        const double saved_t = tn;
        int ncf = 0, nef = 0, nflag = FIRST_CALL;
        double dsm = 0;
        if (nst > 0 && hprime != h) {
            if (qprime != q) {
                adjust_order(qprime - q);
                q = qprime;
                L = q + 1;
                qwait = L;
            }
            rescale();
        }
        for (;;) {
            predict();
            set_coeffs();
            const int r = newton(nflag);
            if (rhs_fail) return -8;   // CV_RHSFUNC_FAIL
            if (r != 0) {   // cvHandleNFlag
                ++ncfn;
                restore(saved_t);
                ++ncf;
                etamax = 1.0;
                if (std::fabs(h) <= hmin * ONEPSM || ncf == MXNCF) return BR_ERR_CONV;
                eta = std::max(ETACF, hmin / std::fabs(h));
                nflag = PREV_CONV_FAIL;
                rescale();
                continue;
            }
            dsm = acnrm * tq[2];   // cvDoErrorTest
            if (dsm <= 1.0) break;
            ++nef;
            ++netf;
            nflag = PREV_ERR_FAIL;
            restore(saved_t);
            if (std::fabs(h) <= hmin * ONEPSM || nef == MXNEF) return BR_ERR_ERRTEST;
            etamax = 1.0;
            if (nef <= MXNEF1) {
                eta = 1.0 / (std::pow(BIAS2 * dsm, 1.0 / L) + ADDON);
                eta = std::max(ETAMIN, std::max(eta, hmin / std::fabs(h)));
                if (nef >= SMALL_NEF) eta = std::min(eta, ETAMXF);
                rescale();
                continue;
            }
            if (q > 1) {
                eta = std::max(ETAMIN, hmin / std::fabs(h));
                adjust_order(-1);
                L = q;
                --q;
                qwait = L;
                rescale();
                continue;
            }
            eta = std::max(ETAMIN, hmin / std::fabs(h));
            h *= eta;
            hscale = h;
            qwait = LONG_WAIT;
            rhs(zn[0].data(), tempv.data());
            ++nfe;
            for (int i = 0; i < n; ++i) zn[1][i] = h * tempv[i];
        }
        complete_step();
        prepare_next(dsm, hmax_inv);
        etamax = nst <= SMALL_NST ? ETAMX2 : ETAMX3;
        for (double& a : acor) a *= tq[2];
        return 0;
    }
    void initial_step(double tout) {   // cvHin
        const double tdist = std::fabs(tout - tn), tround = UROUND * std::max(std::fabs(tn), std::fabs(tout));
        const double hlb = HLB_FACTOR * tround;
        double hub_inv = 0;
        for (int i = 0; i < n; ++i)
            hub_inv = std::max(hub_inv, std::fabs(zn[1][i]) / (HUB_FACTOR * std::fabs(zn[0][i]) + 1.0 / ewt[i]));
        double hub = HUB_FACTOR * tdist;
        if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
        double hg = std::sqrt(hlb * hub);
        if (hub < hlb) { h = hg; return; }
        bool ok = false;
        double hnew = hg;
        for (int count = 1; count <= MAX_ITERS; ++count) {
            for (int i = 0; i < n; ++i) y[i] = hg * zn[1][i] + zn[0][i];
            rhs(y.data(), tempv.data());
            ++nfe;
            for (int i = 0; i < n; ++i) tempv[i] = (tempv[i] - zn[1][i]) * (1.0 / hg);
            const double yddnrm = wrms(tempv.data());
            if (ok || count == MAX_ITERS) { hnew = hg; break; }
            hnew = yddnrm * hub * hub > 2.0 ? std::sqrt(2.0 / yddnrm) : std::sqrt(hg * hub);
            const double hrat = hnew / hg;
            if (hrat > 0.5 && hrat < 2.0) ok = true;
            if (count > 1 && hrat > 2.0) { hnew = hg; ok = true; }
            hg = hnew;
        }
        h = std::min(std::max(H_BIAS * hnew, hlb), hub);
    }
    void dky(double t, double* out) const {   // CVodeGetDky, k = 0
        const double s = (t - tn) / h;
        for (int i = 0; i < n; ++i) out[i] = zn[q][i];
        for (int j = q - 1; j >= 0; --j)
            for (int i = 0; i < n; ++i) out[i] = zn[j][i] + s * out[i];
    }
};

}  // namespace

extern "C" int br_integrate_host(int n, br_rhs_fn f, void* user, double* u, double tf, double rtol, double atol,
                                 int max_steps, br_step_fn cb, void* cb_user, double* stats) {
    if (n <= 0 || !f || !u || !(tf > 0.0) || !(rtol > 0.0) || !(atol > 0.0)) return BR_ERR_INPUT;
    HostCvode cv(n, f, user, rtol, atol);
    const long mxstep = max_steps > 0 ? max_steps : 100000;
    const double hmax_inv = 0.0;
    cv.tstop = tf;
    std::copy(u, u + n, cv.zn[0].begin());
    if (cb) cb(cb_user, 0.0, u);   // save_data at t0
    cv.set_ewt(cv.zn[0].data());
    cv.rhs(cv.zn[0].data(), cv.zn[1].data());
    ++cv.nfe;
    int status = 0;
    if (cv.rhs_fail) status = -8;
    if (!status) {
        cv.initial_step(tf);
        if ((cv.tn + cv.h - cv.tstop) * cv.h > 0.0) cv.h = (cv.tstop - cv.tn) * (1.0 - 4.0 * UROUND);
        cv.hscale = cv.h;
        cv.hprime = cv.h;
        for (double& z : cv.zn[1]) z *= cv.h;
    }
    long nstloc = 0;
    while (!status) {
        if (cv.nst > 0) cv.set_ewt(cv.zn[0].data());
        if (nstloc >= mxstep) { status = BR_ERR_MAXSTEPS; break; }
        const int kf = cv.step(hmax_inv);
        if (kf) { status = kf; break; }
        ++nstloc;
        bool finite = true;
        for (double z : cv.zn[0]) finite = finite && std::isfinite(z);
        if (!finite) { status = BR_ERR_UNSTABLE; break; }   // SciML unstable_check
        const double troundoff = FUZZ * UROUND * (std::fabs(cv.tn) + std::fabs(cv.h));
        if (std::fabs(cv.tn - cv.tstop) <= troundoff) {   // tstop reached: interpolate there
            cv.dky(cv.tstop, u);
            if (cb) cb(cb_user, cv.tstop, u);
            break;
        }
        if ((cv.tn + cv.hprime - cv.tstop) * cv.h > 0.0) {
            cv.hprime = (cv.tstop - cv.tn) * (1.0 - 4.0 * UROUND);
            cv.eta = cv.hprime / cv.h;
        }
        if (cb) cb(cb_user, cv.tn, cv.zn[0].data());
    }
    if (status) std::copy(cv.zn[0].begin(), cv.zn[0].end(), u);
    if (stats) {
        std::fill(stats, stats + BR_NSTAT, 0.0);
        stats[0] = (double)cv.nst; stats[1] = (double)cv.nfe; stats[2] = (double)cv.nje; stats[3] = (double)cv.nsetups;
        stats[4] = (double)cv.nni; stats[5] = (double)cv.ncfn; stats[6] = (double)cv.netf; stats[7] = (double)status;
        stats[13] = status ? cv.tn : tf;
        stats[16] = stats[17] = stats[18] = NAN;
        stats[19] = (double)cv.nfe_dq;
    }
    return status;
}
