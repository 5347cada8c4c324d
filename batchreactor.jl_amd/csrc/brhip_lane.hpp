// brhip_lane.hpp -- ONE REACTOR PER LANE integrator for small gas-phase mechanisms
// (n <= 12 components, no surface species; e.g. H2/O2, n = 9, the C2 ensemble).
// Included by brhip.hip inside its anonymous namespace: it uses that file's CVODE constants,
// KOpts, inv_int, root_int and pow_int.
//
// Why a second engine: with n = 9 a wave-per-reactor layout leaves 55 of 64 lanes idle in the
// LU and solve and 46 idle in the RHS (18 reactions). Here every lane owns a reactor, so each
// VALU instruction advances 64 reactors.
//
// Algorithm: the same CVODE 5.x restatement as k_integrate and oracle/oracle.c (cv_step, cv_nls,
// cvHin, tstop), per lane, with CVODE's own dense difference-quotient Jacobian (cvLsDenseDQJac,
// the one the reference's CVODE_BDF() uses, src/BatchReactor.jl:138-141,:210) instead of the
// analytic one. It runs as a phase machine: each loop iteration evaluates exactly ONE right-hand
// side per lane, at the point that lane's controller asks for (a Newton iterate, a cvHin probe or
// a DQ Jacobian column), so the RHS -- the bulk of the work -- never runs with lanes masked off.
// Lanes that need it then factor I - gamma J (registers, partial pivoting as SUNDIALS
// denseGETRF) and solve. A lane whose reactor is done takes the next one from a global work
// counter (persistent grid), so the spread of step counts costs no idle lanes until the queue
// drains.
//
// Per-lane data: Nordsieck array z0..z5, ewt, acor, the next evaluation point y, the LU factors
// and the controller scalars in VGPRs; concentrations, production sums, third-body sums, the
// T-only rate constants and the DQ base f(y) in LDS rows [row][64 lanes] (lane k -> bank pair k:
// conflict-free); the saved Jacobian in a global slot-major workspace Jg[e][slot] (coalesced
// across lanes). Mechanism records are read with scalar loads (all lanes evaluate the same
// reaction at the same time).
#pragma once
#include <utility>

typedef const __attribute__((address_space(4))) uint32_t CU32;
typedef const __attribute__((address_space(4))) double CF64;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// The lane's global rows (saved J, T-only rate constants, DQ base, LU factors), block-interleaved:
// row e of lane l in workgroup b at byte ((b * E + e) * 64 + l) * 8. Accessed with buffer
// instructions: descriptor and row offset in SGPRs, the lane offset (l * 8) the only VGPR, so no
// per-row 64-bit addresses are formed or kept live.
struct GRows {
    __amdgpu_buffer_rsrc_t r;
    int vo;      // lane * 8
    int base;    // b * E * 512
    __device__ __forceinline__ double ld(int e) const {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, base + e * 512, 0));
    }
    __device__ __forceinline__ void st(int e, double v) const {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, vo, base + e * 512, 0);
    }
    __device__ __forceinline__ double ld_lane(int e_lane, int e) const {   // per-lane row e_lane + e
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo + e_lane * 512, base + e * 512, 0));
    }
    __device__ __forceinline__ void st_lane(int e_lane, int e, double v) const {   // per-lane row e_lane + e
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, vo + e_lane * 512, base + e * 512, 0);
    }
};

// LDS rows of one wave (each row = 64 doubles, one per lane) and global slot-major rows
// (row r of slot s at G[r * S + s], S = slots in the grid)
struct LaneLay {
    int zh, conc, acc, mc, rows;                        // LDS
    int g_rxd, g_fod, g_fp, g_lu, g_rpv, g_rows;        // global; the saved Jacobian is rows [0, NM*NM)
};
__host__ __device__ inline LaneLay lane_lay(int nm, int n, int nset, int nrg, int nfo) {
    LaneLay L;
    L.zh = 0;                   // Nordsieck rows z2..z5 first: row (j - 2) * nm + i, a compile-time
                                // offset from the lane's base (ds_read_b64 immediate)
    L.conc = (QMAX - 1) * nm;   // conc[0..n-1], conc[n] = 1.0 (pad species of the packed records)
    L.acc = L.conc + n + 1;     // production sums (and g/RT scratch at reactor start)
    L.mc = L.acc + n;           // third-body concentration per efficiency set
    L.rows = L.mc + nset;       // 4 waves per CU fit for H2/O2 (one wave per SIMD, VGPR-bound)
    L.g_rxd = nm * nm;          // kf, kr per gas reaction
    L.g_fod = L.g_rxd + 2 * nrg;   // k0, log10 Fcent, c, n per falloff reaction
    L.g_fp = L.g_fod + 4 * nfo;    // f(y) at the DQ Jacobian base point
    L.g_lu = L.g_fp + n;          // LU factors of I - gamma J, column-major NM x NM
    L.g_rpv = L.g_lu + nm * nm;   // reciprocal pivots
    L.g_rows = L.g_rpv + nm;
    return L;
}
__host__ __device__ inline size_t lane_lds_bytes(int nm, int n, int nset, int nrg, int nfo) {
    return (size_t)lane_lay(nm, n, nset, nrg, nfo).rows * 64 * sizeof(double);
}

// Nordsieck array of one lane: z0, z1 in registers (every Newton iteration reads them), z2..z5 in
// LDS rows (touched once per step). get/set with a compile-time j fold to one access.
template <int NM>
struct ZH {
    double z0[NM], z1[NM];
    double* Lz;     // this lane's LDS row base for z2: element (j, i) at Lz[((j - 2) * NM + i) * 64]
    int n;
    __device__ __forceinline__ double get(int j, int i) const {
        return j == 0 ? z0[i] : (j == 1 ? z1[i] : Lz[((j - 2) * NM + i) * 64]);   // pad rows hold 0
    }
    __device__ __forceinline__ void set(int j, int i, double v) {
        if (j == 0) z0[i] = v;
        else if (j == 1) z1[i] = v;
        else Lz[((j - 2) * NM + i) * 64] = v;
    }
    // row j (per-lane j) into out
    __device__ __forceinline__ void row(int j, double (&out)[NM]) const {
        const int jj = j < 2 ? 2 : j;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
            const double lv = Lz[((jj - 2) * NM + i) * 64];
            out[i] = j == 0 ? z0[i] : (j == 1 ? z1[i] : lv);
        }
    }
};

#if BR_ASM_MARKS   // analysis builds: phase markers in the ISA listing
#define LCLK(v) asm volatile("; BR_PHASE_BEGIN " #v)
#define LACC(acc, v) asm volatile("; BR_PHASE_END " #acc)
#elif BR_PHASE_CLOCKS
#define LCLK(v) const unsigned long long v = clock64()
#define LACC(acc, v) acc += clock64() - v
#else
#define LCLK(v)
#define LACC(acc, v)
#endif

enum { PH_JAC = 4 };
enum { A_NONE = 7 };
constexpr int ST_DEFER = 1;   // lane status: hand the reactor to the wavefront pass
enum { PEND_NONE = 0, PEND_STEP = 1, PEND_ATTEMPT = 2, PEND_ADJ = 3, PEND_EF1 = 4 };

// per-lane CVODE scalars (cv_mem)
struct LCV {
    double tn, h, hprime, hscale, eta, etamax, rl1, gamma, gammap, gamrat, crate, delp, acnrm;
    double saved_tq5, saved_t, tol, hg, hub, hlb, tstop, ulimit, minInc;
    double tau[QMAX + 2], tq[6], l[QMAX + 2];
    int q, qprime, L, qwait, nst, nfe, nsetups, nje, nni, ncfn, netf, nstlp, nstlj;
    int ncf, nef, nstloc, status, m_it, convfail, count1, phase, callSetup, jbad, jcur_nls, hnewOK, jcol;
    int pend, pflag;   // deferred step/attempt start (one call site in the kernel): PEND_*, nflag
    double ign_x, ign_t, ign_rate, t_ign, ign_dt;   // ignition marker (max dX_ign/dt over accepted steps)
    int iout, rid;                          // dense-output cursor, reactor index
};

// mole fraction of gas species k (gas-only mechanisms: n = ng) in the lane's state v
template <int NM>
__device__ __forceinline__ double l_mole_frac(const double (&v)[NM], int n, int k) {
    const CF64* mw = (const CF64*)MF(img);                      // molwt[] at image offset 0
    double g = 0.0, xk = 0.0;
#pragma unroll
    for (int i = 0; i < NM; ++i)
        if (i < n) { const double cc = v[i] / mw[i]; g += cc; xk = (i == k) ? cc : xk; }
    return xk / g;
}

// x^(1/L) for the order-dependent step ratios (pow(x, 1.0/L) in CVODE): fp32 estimate of the
// exponent with the binary exponent split off (any fp64 x > 0), then two fp64 Newton steps
__device__ __forceinline__ double lroot(double x, int L) {
    int e;
    const double mnt = frexp(x, &e);
    const float t = ((float)e + __builtin_amdgcn_logf((float)mnt)) / (float)L;
    const float ti = floorf(t);
    double y = ldexp((double)__builtin_amdgcn_exp2f(t - ti), (int)ti);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        double pw = 1.0;                                   // y^(L-1)
#pragma unroll
        for (int k = 1; k < QMAX + 1; ++k) pw = (k < L) ? pw * y : pw;
        y -= (pw * y - x) / (L * pw);
    }
    return (L == 1 || x == 0.0) ? x : y;
}

// per-lane index tests through an opaque copy of the index: written as plain select chains over a
// register array, they are turned back into a dynamically indexed array in scratch memory
__device__ __forceinline__ bool is_idx(int i, int k) {
    asm volatile("" : "+v"(i));
    return i == k;
}
template <int K>
__device__ __forceinline__ double sel(const double (&v)[K], int i) {   // v[i], i per lane
    double r = v[0];
#pragma unroll
    for (int k = 1; k < K; ++k) r = is_idx(i, k) ? v[k] : r;
    return r;
}
template <int NM>
__device__ __forceinline__ double lwrms(const double (&v)[NM], const double (&w)[NM], int n) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NM; ++k) { const double t = v[k] * w[k]; s += t * t; }   // pad entries are 0
    return sqrt(s / n);
}

// ---- Nordsieck history operations (oracle/oracle.c cv_rescale / cv_predict / cv_restore /
//      increase_bdf / decrease_bdf), unrolled over QMAX with per-lane order predicates
template <int NM>
__device__ __forceinline__ void l_rescale(LCV& c, ZH<NM>& z) {
    double fj[QMAX + 1];                             // eta^j for rows j <= q, 1 above (x * 1 = x)
    double factor = c.eta;
#pragma unroll
    for (int j = 1; j <= QMAX; ++j) {
        fj[j] = (j <= c.q) ? factor : 1.0;
        factor *= c.eta;
    }
#pragma unroll
    for (int j = 1; j <= QMAX; ++j)
#pragma unroll
        for (int i = 0; i < NM; ++i) z.set(j, i, z.get(j, i) * fj[j]);
    c.h = c.hscale * c.eta;
    c.hscale = c.h;
}
// Nordsieck prediction z <- P z (P the Pascal matrix of order q) and its inverse, as one
// matrix-vector product per component with per-lane masked binomial coefficients: z_j += sum_{i>j,
// i<=q} (+-)C(i,j) z_i (CVODE's repeated row additions, same values up to rounding)
template <int NM, bool SUB>
__device__ __forceinline__ void l_pascal(const LCV& c, ZH<NM>& z) {
    constexpr double BIN[QMAX + 1][QMAX + 1] = {{1, 1, 1, 1, 1, 1}, {0, 1, 2, 3, 4, 5}, {0, 0, 1, 3, 6, 10},
                                                {0, 0, 0, 1, 4, 10}, {0, 0, 0, 0, 1, 5}, {0, 0, 0, 0, 0, 1}};
    double cf[QMAX][QMAX + 1];                       // cf[j][i], i > j
#pragma unroll
    for (int i = 1; i <= QMAX; ++i) {
        const double mi = (i <= c.q) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < i; ++j) cf[j][i] = ((SUB && ((i - j) & 1)) ? -BIN[j][i] : BIN[j][i]) * mi;
    }
#pragma unroll
    for (int k = 0; k < NM; ++k) {
        double r[QMAX + 1];
#pragma unroll
        for (int j = 0; j <= QMAX; ++j) r[j] = z.get(j, k);
#pragma unroll
        for (int j = 0; j < QMAX; ++j) {
            double acc = r[j];
#pragma unroll
            for (int i = j + 1; i <= QMAX; ++i) acc = fma(cf[j][i], r[i], acc);
            if (j < 2) z.set(j, k, acc);
            else if (j < c.q) z.set(j, k, acc);
        }
    }
}
template <int NM>
__device__ __forceinline__ void l_predict(LCV& c, ZH<NM>& z) {
    c.tn += c.h;
    if ((c.tn - c.tstop) * c.h > 0) c.tn = c.tstop;
    l_pascal<NM, false>(c, z);
}
template <int NM>
__device__ __forceinline__ void l_restore(LCV& c, ZH<NM>& z) {
    c.tn = c.saved_t;
    l_pascal<NM, true>(c, z);
}
// cvAdjustOrder (oracle/oracle.c increase_bdf / decrease_bdf): the coefficient recurrences per
// lane, then ONE pass over the components for both directions:
//   increase: z[q+1] = A1 z5, z[j] += l[j] z[q+1] (2 <= j <= q);  decrease: z[j] -= l[j] z[q] (2 <= j < q)
template <int NM>
__device__ __forceinline__ void l_adjust_order(LCV& c, ZH<NM>& z, int dq) {
    const int q = c.q;
    const bool inc = dq == 1;
    const bool act = inc || q > 2;                   // cvAdjustOrder: nothing for q == 2 going down
    double* l = c.l;
#pragma unroll
    for (int i = 0; i <= QMAX + 1; ++i) l[i] = 0.0;
    l[2] = 1.0;
    double A1 = 0.0;
    if (inc) {                                        // increase_bdf coefficients
        double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = c.hscale;
#pragma unroll
        for (int j = 1; j < QMAX - 1; ++j) {
            if (j < q) {
                hsum += c.tau[j + 1];
                const double xi = hsum / c.hscale;
                prod *= xi;
                alpha0 -= inv_int(j + 1);
                alpha1 += 1.0 / xi;
#pragma unroll
                for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xiold + l[i - 1];
                xiold = xi;
            }
        }
        A1 = (-alpha0 - alpha1) / prod;
    } else {                                          // decrease_bdf coefficients
        double hsum = 0.0;
#pragma unroll
        for (int j = 1; j <= QMAX - 2; ++j) {
            if (j <= q - 2) {
                hsum += c.tau[j];
                const double xi = hsum / c.hscale;
#pragma unroll
                for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xi + l[i - 1];
            }
        }
    }
    double cf[QMAX + 1];
#pragma unroll
    for (int j = 2; j <= QMAX; ++j)
        cf[j] = !act ? 0.0 : (inc ? ((j <= q) ? l[j] : 0.0) : ((j < q) ? -l[j] : 0.0));
    const int L = inc ? q + 1 : -1;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        double r[QMAX + 1];
#pragma unroll
        for (int j = 2; j <= QMAX; ++j) r[j] = z.get(j, i);
        double zq = r[2];
#pragma unroll
        for (int j = 3; j <= QMAX; ++j) zq = is_idx(q, j) ? r[j] : zq;
        const double src = inc ? A1 * r[QMAX] : zq;
#pragma unroll
        for (int j = 2; j <= QMAX; ++j) {
            const double v = (j == L) ? src : fma(cf[j], src, r[j]);
            if (act) z.set(j, i, v);
        }
    }
}

// cvSet + cvSetTqBDF (oracle/oracle.c cv_set / set_tq_bdf)
__device__ __forceinline__ void l_set(LCV& c) {
    const int q = c.q;
    double* l = c.l;
    double xi_inv = 1.0, xistar_inv = 1.0;
    l[0] = l[1] = 1.0;
#pragma unroll
    for (int i = 2; i <= QMAX + 1; ++i) l[i] = 0.0;
    double alpha0 = -1.0, alpha0_hat = -1.0, hsum = c.h;
    if (q > 1) {
#pragma unroll
        for (int j = 2; j < QMAX; ++j) {
            if (j < q) {
                hsum += c.tau[j - 1];
                xi_inv = c.h / hsum;
                alpha0 -= inv_int(j);
#pragma unroll
                for (int i = j; i >= 1; --i) l[i] += l[i - 1] * xi_inv;
            }
        }
        alpha0 -= inv_int(q);
        xistar_inv = -l[1] - alpha0;
        hsum += sel(c.tau, q - 1);
        xi_inv = c.h / hsum;
        alpha0_hat = -l[1] - xi_inv;
#pragma unroll
        for (int i = QMAX; i >= 1; --i) if (i <= q) l[i] += l[i - 1] * xistar_inv;
    }
    const double lq = sel(c.l, q);
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = 1.0 + q * A1;
    c.tq[2] = fabs(A1 / (alpha0 * A2));
    c.tq[5] = fabs(A2 * xistar_inv / (lq * xi_inv));
    if (c.qwait == 1) {
        if (q > 1) {
            const double C = xistar_inv / lq;
            const double A3 = alpha0 + inv_int(q);
            const double A4 = alpha0_hat + xi_inv;
            const double Cpinv = (1.0 - A4 + A3) / A3;
            c.tq[1] = fabs(C * Cpinv);
        } else {
            c.tq[1] = 1.0;
        }
        hsum += sel(c.tau, q);
        xi_inv = c.h / hsum;
        const double A5 = alpha0 - inv_int(q + 1);
        const double A6 = alpha0_hat - xi_inv;
        const double Cppinv = (1.0 - A6 + A5) / A2;
        c.tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
    }
    c.tq[4] = CORTES / c.tq[2];
    c.rl1 = 1.0 / l[1];
    c.gamma = c.h * c.rl1;
    if (c.nst == 0) c.gammap = c.gamma;
    c.gamrat = (c.nst > 0) ? c.gamma / c.gammap : 1.0;
}

template <int NM>
__device__ __forceinline__ void l_begin_attempt(LCV& c, ZH<NM>& z, double (&acor)[NM], double (&y)[NM],
                                                int nflag) {
    l_predict<NM>(c, z);
    l_set(c);
    c.convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? NO_FAILURES : FAIL_OTHER;
    c.callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (c.nst == 0) || (c.nst >= c.nstlp + MSBP) ||
                  (fabs(c.gamrat - 1.0) > DGMAX);
#pragma unroll
    for (int i = 0; i < NM; ++i) { acor[i] = 0.0; y[i] = z.z0[i]; }
    c.tol = c.tq[4];
    c.jbad = 0;
    c.jcur_nls = 0;
    c.m_it = 0;
}
// the deferred start of a step (PEND_STEP: cvStep entry with order change / rescale) or of a
// retry (PEND_ATTEMPT: rescale; PEND_ADJ: order - 1 and rescale; PEND_EF1: none), then the attempt
template <int NM>
__device__ __forceinline__ void l_run_pending(LCV& c, ZH<NM>& z, double (&acor)[NM], double (&ewt)[NM],
                                              double (&y)[NM], const KOpts& o, int n) {
    int dq, nflag;
    bool resc;
    if (c.pend == PEND_STEP) {
#pragma unroll
        for (int i = 0; i < NM; ++i) ewt[i] = (i < n) ? 1.0 / (o.rtol * fabs(z.z0[i]) + o.atol) : 1.0;
        c.saved_t = c.tn;
        c.ncf = 0;
        c.nef = 0;
        resc = (c.nst > 0) && (c.hprime != c.h);
        dq = resc ? c.qprime - c.q : 0;
        nflag = FIRST_CALL;
    } else {
        dq = (c.pend == PEND_ADJ) ? -1 : 0;
        resc = c.pend != PEND_EF1;
        nflag = c.pflag;
    }
    if (dq != 0) {
        l_adjust_order<NM>(c, z, dq);
        c.q += dq; c.L = c.q + 1; c.qwait = c.L;
    }
    if (resc) l_rescale<NM>(c, z);
    l_begin_attempt<NM>(c, z, acor, y, nflag);
    c.pend = PEND_NONE;
}

// the DQ Jacobian column jcol is evaluated at y = z0 + inc e_jcol (cvLsDenseDQJac)
constexpr double SRUR = 1.4901161193847656e-08;   // sqrt(UROUND) = 2^-26
constexpr double MIN_INC_MULT = 1000.0;
template <int NM>
__device__ __forceinline__ double l_dq_point(const LCV& c, const double (&z0)[NM], const double (&ewt)[NM],
                                             double (&y)[NM]) {
    const double yj = sel(z0, c.jcol), wj = sel(ewt, c.jcol);
    const double inc = fmax(SRUR * fabs(yj), c.minInc / wj);
#pragma unroll
    for (int i = 0; i < NM; ++i) y[i] = (i == c.jcol) ? z0[i] + inc : z0[i];
    return inc;
}

// Controller, part 1 (after f = F(y) of this lane): A_RHS (next y set), A_SOLVE / A_SETUP
// (b = -delta for the solve; A_SETUP: factor I - gamma J from the saved J first), A_DONE.
template <int NM>
__device__ __forceinline__ int l_post_rhs(LCV& c, ZH<NM>& z, double (&acor)[NM], double (&ewt)[NM],
                                          double (&y)[NM], const double (&f)[NM], double (&b)[NM], double* Lp,
                                          const LaneLay& LL, const GRows& G, const KOpts& o, int n) {
    const int phase = c.phase;
    if (phase == PH_JAC) {                      // one DQ column: J[:, jcol] = (f - fy) / inc
        const double yj = sel(z.z0, c.jcol), wj = sel(ewt, c.jcol);
        const double inc = fmax(SRUR * fabs(yj), c.minInc / wj);
        const double ii = 1.0 / inc;
#pragma unroll
        for (int i = 0; i < NM; ++i)
            if (i < n) G.st_lane(c.jcol * NM, i, ii * f[i] - ii * G.ld(LL.g_fp + i));
        c.jcol += 1;
        if (c.jcol < n) {
            l_dq_point<NM>(c, z.z0, ewt, y);
            return A_RHS;
        }
        c.phase = PH_NEWTON;
#pragma unroll
        for (int i = 0; i < NM; ++i) {          // the residual at the setup point (y = z0, acor = 0)
            const double fy = i < n ? G.ld(LL.g_fp + i) : 0.0;
            b[i] = -((c.rl1 * z.z1[i] + acor[i]) - c.gamma * fy);
        }
        return A_SETUP;
    }
    c.nfe += 1;
    if (phase == PH_NEWTON) {
#pragma unroll
        for (int i = 0; i < NM; ++i) b[i] = -((c.rl1 * z.z1[i] + acor[i]) - c.gamma * f[i]);   // cvNlsResidual
        if (c.m_it == 0 && c.callSetup) {      // cvLsSetup decision
            const double dgamma = fabs(c.gamma / c.gammap - 1.0);
            const int cf = c.jbad ? FAIL_BAD_J : c.convfail;
            const int newj = (c.nst == 0) || (c.nst > c.nstlj + LS_MSBJ) || ((cf == FAIL_BAD_J) && (dgamma < LS_DGMAX)) ||
                             (cf == FAIL_OTHER);
            if (newj) { c.nje += 1; c.nstlj = c.nst; }
            c.nsetups += 1;
            c.jcur_nls = newj;
            c.gamrat = 1.0; c.gammap = c.gamma; c.crate = 1.0; c.nstlp = c.nst;
            if (newj && !o.dq_jac) {            // analytic Jacobian at y (the RHS point just evaluated)
                lane_jac<NM>(LL, Lp, G, n);
                return A_SETUP;
            }
            if (newj) {                         // DQ Jacobian at (y, f): n more RHS iterations
                const double fnorm = lwrms<NM>(f, ewt, n);
                c.minInc = (fnorm != 0.0) ? (MIN_INC_MULT * fabs(c.h) * UROUND * n * fnorm) : 1.0;
#pragma unroll
                for (int i = 0; i < NM; ++i) if (i < n) G.st(LL.g_fp + i, f[i]);
                c.jcol = 0;
                c.phase = PH_JAC;
                l_dq_point<NM>(c, z.z0, ewt, y);
                return A_RHS;
            }
            return A_SETUP;
        }
        return A_SOLVE;
    }
    if (phase == PH_EF1) {                      // restart at order 1 after repeated error-test failures
#pragma unroll
        for (int i = 0; i < NM; ++i) z.z1[i] = c.h * f[i];
        c.pend = PEND_EF1; c.pflag = PREV_ERR_FAIL;
        c.phase = PH_NEWTON;
        return A_RHS;
    }
    double h;
    if (phase == PH_F0) {                       // cvHin, first part (cvUpperBoundH0)
        const double tdist = fabs(c.tstop - c.tn);
        const double tround = UROUND * fmax(fabs(c.tn), fabs(c.tstop));
        const double hlb = HLB_FACTOR * tround;
        double hub_inv = 0.0;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
            z.z1[i] = f[i];
            const double r = fabs(f[i]) / (HUB_FACTOR * fabs(z.z0[i]) + 1.0 / ewt[i]);
            if (i < n && r > hub_inv) hub_inv = r;
        }
        double hub = HUB_FACTOR * tdist;
        if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
        const double hg = sqrt(hlb * hub);
        c.hlb = hlb; c.hub = hub; c.hg = hg;
        if (hub < hlb) {
            h = hg;
        } else {
            c.count1 = 1; c.hnewOK = 0;
#pragma unroll
            for (int i = 0; i < NM; ++i) y[i] = hg * f[i] + z.z0[i];
            c.phase = PH_HIN;
            return A_RHS;
        }
    } else {                                    // PH_HIN: cvYddNorm + the cvHin iteration
        double hg = c.hg;
        double t[NM];
#pragma unroll
        for (int i = 0; i < NM; ++i) t[i] = (f[i] - z.z1[i]) * (1.0 / hg);
        const double yddnrm = lwrms<NM>(t, ewt, n);
        double hnew;
        if (c.hnewOK || c.count1 == MAX_ITERS) {
            hnew = hg;
        } else {
            hnew = (yddnrm * c.hub * c.hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * c.hub);
            const double hrat = hnew / hg;
            int ok = 0;
            if ((hrat > 0.5) && (hrat < 2.0)) ok = 1;
            if ((c.count1 > 1) && (hrat > 2.0)) { hnew = hg; ok = 1; }
            c.hnewOK = ok;
            c.hg = hnew;
            c.count1 += 1;
#pragma unroll
            for (int i = 0; i < NM; ++i) y[i] = hnew * z.z1[i] + z.z0[i];
            return A_RHS;
        }
        double h0 = H_BIAS * hnew;
        if (h0 < c.hlb) h0 = c.hlb;
        if (h0 > c.hub) h0 = c.hub;
        h = h0;
    }
    // first step size known
    if (o.hmax_inv > 0) { const double rh = fabs(h) * o.hmax_inv; if (rh > 1.0) h /= rh; }
    if ((c.tn + h - c.tstop) * h > 0.0) h = (c.tstop - c.tn) * (1.0 - 4.0 * UROUND);
    c.h = h; c.hscale = h; c.hprime = h;
#pragma unroll
    for (int i = 0; i < NM; ++i) z.z1[i] *= h;
    if (o.max_steps <= 0) { c.status = BR_ERR_MAXSTEPS; return A_DONE; }
    c.pend = PEND_STEP;
    c.phase = PH_NEWTON;
    return A_RHS;
}

// Controller, part 2 (after the solve, delta = Newton correction, or an LU failure): convergence
// test, error test, cvCompleteStep, cvPrepareNextStep, tstop. A_RHS (next y set) or A_DONE
// (y = the state at tstop when status == 0).
template <int NM>
__device__ __forceinline__ int l_post_solve(LCV& c, ZH<NM>& z, double (&acor)[NM], double (&ewt)[NM],
                                            double (&y)[NM], double (&delta)[NM], int lu_fail, const KOpts& o, int n) {
    int nls;
    if (lu_fail) {
        nls = 2;
    } else {
        c.nni += 1;
        if (c.gamrat != 1.0) {
            const double s = 2.0 / (1.0 + c.gamrat);
#pragma unroll
            for (int i = 0; i < NM; ++i) delta[i] *= s;
        }
#pragma unroll
        for (int i = 0; i < NM; ++i) acor[i] += delta[i];
        const double del = lwrms<NM>(delta, ewt, n);   // cvNlsConvTest
        const int m = c.m_it;
        if (m > 0) c.crate = fmax(CRDOWN * c.crate, del / c.delp);
        const double dcon = del * fmin(1.0, c.crate) / c.tol;
        if (dcon <= 1.0) {
            c.acnrm = (m == 0) ? del : lwrms<NM>(acor, ewt, n);
            nls = 0;
        } else {
            bool fail = (m >= 1) && (del > RDIV * c.delp);
            if (!fail) {
                c.delp = del;
                c.m_it = m + 1;
                if (m + 1 >= NLS_MAXCOR) fail = true;
            }
            if (!fail) {
#pragma unroll
                for (int i = 0; i < NM; ++i) y[i] = z.z0[i] + acor[i];
                return A_RHS;
            }
            if (!c.jcur_nls) {                   // retry with a fresh Jacobian
                c.callSetup = 1; c.jbad = 1; c.m_it = 0;
#pragma unroll
                for (int i = 0; i < NM; ++i) { acor[i] = 0.0; y[i] = z.z0[i]; }
                return A_RHS;
            }
            nls = 1;
        }
    }
    if (nls != 0) {                              // cvHandleNFlag
        c.ncfn += 1;
        l_restore<NM>(c, z);
        c.ncf += 1;
        c.etamax = 1.0;
        if (c.ncf == MXNCF) { c.status = BR_ERR_CONV; return A_DONE; }
        c.eta = ETACF;
        c.pend = PEND_ATTEMPT; c.pflag = PREV_CONV_FAIL;
        return A_RHS;
    }
    // cvDoErrorTest
    const double dsm = c.acnrm * c.tq[2];
    const int q = c.q;
    if (dsm > 1.0) {
        c.nef += 1; c.netf += 1;
        l_restore<NM>(c, z);
        if (c.nef == MXNEF) { c.status = BR_ERR_ERRTEST; return A_DONE; }
        c.etamax = 1.0;
        if (c.nef <= MXNEF1) {
            double eta = 1.0 / (lroot(BIAS2 * dsm, c.L) + ADDON);
            eta = fmax(ETAMIN, eta);
            if (c.nef >= SMALL_NEF) eta = fmin(eta, ETAMXF);
            c.eta = eta;
            c.pend = PEND_ATTEMPT; c.pflag = PREV_ERR_FAIL;
            return A_RHS;
        }
        if (q > 1) {
            c.eta = ETAMIN;
            c.pend = PEND_ADJ; c.pflag = PREV_ERR_FAIL;
            return A_RHS;
        }
        c.eta = ETAMIN;
        c.h *= ETAMIN; c.hscale = c.h; c.qwait = LONG_WAIT;
#pragma unroll
        for (int i = 0; i < NM; ++i) y[i] = z.z0[i];
        c.phase = PH_EF1;
        return A_RHS;
    }
    // cvCompleteStep
    c.nst += 1;
    const int nst = c.nst;
    const double h = c.h;
#pragma unroll
    for (int i = QMAX; i >= 2; --i) if (i <= q) c.tau[i] = c.tau[i - 1];
    if ((q == 1) && (nst > 1)) c.tau[2] = c.tau[1];
    c.tau[1] = h;
#pragma unroll
    for (int j = 0; j <= QMAX; ++j)
        if (j <= q) {
            const double lj = c.l[j];
#pragma unroll
            for (int i = 0; i < NM; ++i) z.set(j, i, z.get(j, i) + lj * acor[i]);
        }
    int qwait = c.qwait - 1;
    if ((qwait == 1) && (q != QMAX)) {
#pragma unroll
        for (int i = 0; i < NM; ++i) z.set(QMAX, i, acor[i]);
        c.saved_tq5 = c.tq[5];
    }
    // cvPrepareNextStep
    double eta = 1.0, hprime = h;
    int qprime = q;
    if (c.etamax == 1.0) {
        qwait = qwait > 2 ? qwait : 2;
    } else {
        const int L = c.L;
        const double etaq = 1.0 / (lroot(BIAS2 * dsm, L) + ADDON);
        if (qwait != 0) {
            eta = etaq;
        } else {
            qwait = 2;
            double etaqm1 = 0.0, etaqp1 = 0.0;
            if (q > 1) {
                double zq[NM];
                z.row(q, zq);
                const double ddn = lwrms<NM>(zq, ewt, n) * c.tq[1];
                etaqm1 = 1.0 / (lroot(BIAS1 * ddn, q) + ADDON);
            }
            if (q != QMAX && c.saved_tq5 != 0.0) {
                const double cquot = (c.tq[5] / c.saved_tq5) * pow_int(h / c.tau[2], L);
                double t[NM];
#pragma unroll
                for (int i = 0; i < NM; ++i) t[i] = acor[i] - cquot * z.get(QMAX, i);
                const double dup = lwrms<NM>(t, ewt, n) * c.tq[3];
                etaqp1 = 1.0 / (lroot(BIAS3 * dup, L + 1) + ADDON);
            }
            const double etam = fmax(etaqm1, fmax(etaq, etaqp1));
            if (etam < THRESH) { eta = 1.0; }
            else if (etam == etaq) { eta = etaq; }
            else if (etam == etaqm1) { eta = etaqm1; qprime = q - 1; }
            else {
                eta = etaqp1; qprime = q + 1;
#pragma unroll
                for (int i = 0; i < NM; ++i) z.set(QMAX, i, acor[i]);
            }
        }
        if (eta < THRESH) { eta = 1.0; hprime = h; }            // cvSetEta
        else {
            eta = fmin(eta, c.etamax);
            eta /= fmax(1.0, fabs(h) * o.hmax_inv * eta);
            hprime = h * eta;
        }
    }
    c.qwait = qwait;
    c.etamax = (nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
#pragma unroll
    for (int i = 0; i < NM; ++i) acor[i] *= c.tq[2];
    c.nstloc += 1;
    c.eta = eta; c.hprime = hprime; c.qprime = qprime;
    {   // SciML unstable_check: NaN state (ulimit = inf), or opt-in runaway (br_opts.unstable_factor);
        // first, as in the oracle: an unstable step writes no dense output
        double zm = 0.0;
#pragma unroll
        for (int i = 0; i < NM; ++i) { const double a = fabs(z.z0[i]); zm = fmax(zm, a == a ? a : INFINITY); }
        if (!(zm < INFINITY) || zm > c.ulimit) { c.status = BR_ERR_UNSTABLE; return A_DONE; }
    }
    if (o.ign >= 0) {                            // ignition marker (midpoint of the steepest step)
        const double x = l_mole_frac<NM>(z.z0, n, o.ign);
        const double r = (x - c.ign_x) / (c.tn - c.ign_t);
        if (r > c.ign_rate) { c.ign_rate = r; c.t_ign = 0.5 * (c.ign_t + c.tn); c.ign_dt = c.tn - c.ign_t; }
        c.ign_x = x; c.ign_t = c.tn;
    }
    const double tlim = fabs(c.tn - c.tstop) <= FUZZ * UROUND * (fabs(c.tn) + fabs(h)) ? c.tstop : c.tn;
    while (c.iout < o.nout && o.tout[c.iout] <= tlim) {   // dense output (CVodeGetDky, CV_NORMAL)
        const double sk = (o.tout[c.iout] - c.tn) / h;
        double zq[NM], yo[NM];
        z.row(q, zq);
#pragma unroll
        for (int i = 0; i < NM; ++i) yo[i] = zq[i];
#pragma unroll
        for (int j = QMAX - 1; j >= 0; --j)
            if (j <= q - 1) {
#pragma unroll
                for (int i = 0; i < NM; ++i) yo[i] = z.get(j, i) + sk * yo[i];
            }
        double* row = o.yout + ((size_t)c.rid * o.nout + c.iout) * n;
#pragma unroll
        for (int i = 0; i < NM; ++i) if (i < n) row[i] = yo[i];
        c.iout += 1;
    }
    const double tn = c.tn;
    const double troundoff = FUZZ * UROUND * (fabs(tn) + fabs(h));
    if (fabs(tn - c.tstop) <= troundoff) {       // CVodeGetDky(tstop, 0)
        const double sk = (c.tstop - tn) / h;
        double zq[NM];
        z.row(q, zq);
#pragma unroll
        for (int i = 0; i < NM; ++i) y[i] = zq[i];
#pragma unroll
        for (int j = QMAX - 1; j >= 0; --j)
            if (j <= q - 1) {
#pragma unroll
                for (int i = 0; i < NM; ++i) y[i] = z.get(j, i) + sk * y[i];
            }
        return A_DONE;
    }
    if ((tn + hprime - c.tstop) * h > 0.0) {
        c.hprime = (c.tstop - tn) * (1.0 - 4.0 * UROUND);
        c.eta = c.hprime / h;
    }
    if (c.nstloc >= o.max_steps) { c.status = BR_ERR_MAXSTEPS; return A_DONE; }
    if (c.nstloc == o.defer_steps) { c.status = ST_DEFER; return A_DONE; }   // kernel decides
    c.pend = PEND_STEP;
    return A_RHS;
}

// ---- dense LU of the lane's matrix in registers (SUNDIALS denseGETRF: first maximal |a_ik|
//      of column k, full-row swap, multipliers by the reciprocal pivot, rank-1 update).
//      Pad rows / columns (i >= n) hold the identity, so the loops run over NM unconditionally.
template <int NM, int k>
__device__ __forceinline__ void l_getrf_step(double (&a)[NM][NM], unsigned long long& pv, double (&rpv)[NM], int& fail) {
    int p = k;
    double best = fabs(a[k][k]);
#pragma unroll
    for (int i = k + 1; i < NM; ++i) {
        const double v = fabs(a[i][k]);
        if (v > best) { best = v; p = i; }
    }
    pv |= (unsigned long long)p << (4 * k);
    if (best == 0.0 && fail == 0) fail = k + 1;
    if (p != k) {                                   // lanes that pivot off the diagonal
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            const double rk = a[k][j];
            double rp = rk;
#pragma unroll
            for (int i = k + 1; i < NM; ++i) rp = is_idx(p, i) ? a[i][j] : rp;
#pragma unroll
            for (int i = k + 1; i < NM; ++i) a[i][j] = is_idx(p, i) ? rk : a[i][j];
            a[k][j] = rp;
        }
    }
    const double mult = 1.0 / a[k][k];
    rpv[k] = mult;
#pragma unroll
    for (int i = k + 1; i < NM; ++i) a[i][k] *= mult;
#pragma unroll
    for (int j = k + 1; j < NM; ++j) {
        const double akj = a[k][j];
#pragma unroll
        for (int i = k + 1; i < NM; ++i) a[i][j] -= akj * a[i][k];
    }
}
template <int NM, int... K>
__device__ __forceinline__ int l_getrf_seq(double (&a)[NM][NM], unsigned long long& pv, double (&rpv)[NM],
                                           std::integer_sequence<int, K...>) {
    int fail = 0;
    pv = 0;
    (l_getrf_step<NM, K>(a, pv, rpv, fail), ...);   // compile-time unrolled over the pivot steps
    return fail;
}
template <int NM>
__device__ __forceinline__ int l_getrf(double (&a)[NM][NM], unsigned long long& pv, double (&rpv)[NM]) {
    return l_getrf_seq<NM>(a, pv, rpv, std::make_integer_sequence<int, NM>{});
}
// denseGETRS on the factors kept in the lane's global rows (column-major LU at G[(lu + k*NM + i)*S],
// reciprocal pivots at G[(rpv + k)*S]; pivot rows packed 4 bits each in pv)
template <int NM>
__device__ __forceinline__ void l_getrs(const GRows& G, const LaneLay& LL, unsigned long long pv,
                                        double (&b)[NM]) {
#pragma unroll
    for (int k = 0; k < NM; ++k) {
        const int p = (int)((pv >> (4 * k)) & 15);
        if (p != k) {
            const double bk = b[k];
            double bp = bk;
#pragma unroll
            for (int i = k + 1; i < NM; ++i) bp = is_idx(p, i) ? b[i] : bp;
#pragma unroll
            for (int i = k + 1; i < NM; ++i) b[i] = is_idx(p, i) ? bk : b[i];
            b[k] = bp;
        }
    }
    // all factors in one burst of loads (one exposed latency), then the sweeps
    double lu[NM][NM], rp[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) {
        rp[k] = G.ld(LL.g_rpv + k);
#pragma unroll
        for (int i = 0; i < NM; ++i) lu[k][i] = (i != k) ? G.ld(LL.g_lu + k * NM + i) : 0.0;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < NM - 1; ++k)
#pragma unroll
        for (int i = k + 1; i < NM; ++i) b[i] -= lu[k][i] * b[k];
#pragma unroll
    for (int k = NM - 1; k > 0; --k) {
        b[k] *= rp[k];
#pragma unroll
        for (int i = 0; i < k; ++i) b[i] -= lu[k][i] * b[k];
    }
    b[0] *= rp[0];
}

// ---- rates: T-only constants per lane (at reactor start) and the gas-phase RHS
//      (residual!, src/BatchReactor.jl:312-376, gas-only: du_k = wdot_k M_k, :355,:363-370)
__device__ __forceinline__ int lane_sp(uint32_t w, int e, int n) {   // record species -> LDS conc row
    const int k = (int)((w >> (8 * e)) & 255);
    return k == Lay<1>::ONE ? n : k;
}
__device__ __forceinline__ void lane_tconst(const LaneLay& LL, double* Lp, const GRows& G, double T, int n) {
    const double lT = log(T);
    const int ng = MF(ng), nrg = MF(nrg);
    for (int k = 0; k < ng; ++k) {                   // g/RT (NASA-7) into the acc rows
        const CF64* cf = (const CF64*)MF(nasa) + 15 * k;
        const double tmid = cf[0];
        const CF64* a = (T < tmid) ? cf + 8 : cf + 1;
        const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        const double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        Lp[(LL.acc + k) * 64] = h - s;
    }
    const double RT = R_GAS * T;
    const CU32* rx = (const CU32*)((const char*)MF(img) + Lay<1>::IMG_RX);
    for (int r = 0; r < nrg; ++r) {
        const auto rq = rx_rec(rx, r);
        const uint32_t w0 = rq[0], w1 = rq[1], info = rq[2];
        const CF64* gp = (const CF64*)MF(g_par) + 4 * r;
        const double kf = gp[0] * exp(gp[1] * lT - gp[2] / T);
        double kr = 0.0;
        if (gi_rev(info)) {
            double dg = 0.0;
            const int nf = gi_nf(info), nr = gi_nr(info);
            for (int e = 0; e < 4; ++e) if (e < nr) dg += Lp[(LL.acc + lane_sp(w1, e, n)) * 64];
            for (int e = 0; e < 4; ++e) if (e < nf) dg -= Lp[(LL.acc + lane_sp(w0, e, n)) * 64];
            double Kc = exp(-dg) * pow(MF(p_std) / RT, (double)((const __attribute__((address_space(4))) int*)MF(g_dnu))[r]);
            Kc *= gp[3];
            kr = kf / Kc;
        }
        G.st(LL.g_rxd + 2 * r, kf);
        G.st(LL.g_rxd + 2 * r + 1, kr);
        if (gi_tb(info) == 2) {
            const int fi = gi_foidx(info);
            const CF64* fp = (const CF64*)MF(fo_par) + 8 * fi;
            G.st(LL.g_fod + 4 * fi, fp[0] * exp(fp[1] * lT - fp[2] / T) / kf);   // k0 / k_inf
            double fcv = 1.0;
            if (gi_troe(info)) {
                fcv = (1 - fp[3]) * exp(-T / fp[4]) + fp[3] * exp(-T / fp[5]);
                if (gi_troe(info) == 4) fcv += exp(-fp[6] / T);
            }
            const double lfc = log10(fcv);
            G.st(LL.g_fod + 4 * fi + 1, lfc);
            G.st(LL.g_fod + 4 * fi + 2, ((MF(conv) & BR_CONV_TROE_C4) ? -4.0 : -0.4) - 0.67 * lfc);
            G.st(LL.g_fod + 4 * fi + 3, 0.75 - 1.27 * lfc);
        }
    }
}

template <int NM>
__device__ __forceinline__ void lane_rhs(const LaneLay& LL, double* Lp, const GRows& G, const double (&y)[NM], int n,
                                         double (&f)[NM]) {
    const CF64* mw = (const CF64*)MF(img);                      // molwt[] at image offset 0
    // c_k = u_k / M_k (= p x_k / RT, :326-338); production sums cleared
    double ct = 0.0;
#pragma unroll
    for (int k = 0; k < NM; ++k) {
        if (k < n) {
            const double c = y[k] / mw[k];
            Lp[(LL.conc + k) * 64] = c;
            Lp[(LL.acc + k) * 64] = 0.0;
            ct += c;
        }
    }
    // third-body concentrations per efficiency set: Ctot + sum (eff - 1) c
    const int nset = MF(nset);
    if (nset) {
        const CU32* tbs = (const CU32*)((const char*)MF(img) + MF(tbs_off));
        const char* tbe = (const char*)MF(img) + MF(tbe_off);
        for (int t = 0; t < nset; ++t) {
            const uint32_t w = tbs[t];
            const int b = w & 0xFFFFF, e = b + (int)(w >> 20);
            double s = ct;
            for (int i = b; i < e; ++i) {
                const int k = *(const CU32*)(tbe + 16 * i) & 0xFFFF;
                s = fma(*(const CF64*)(tbe + 16 * i + 8), Lp[(LL.conc + k) * 64], s);
            }
            Lp[(LL.mc + t) * 64] = s;
        }
    }
    // rates of progress and the net-stoichiometry scatter into the production sums
    const bool xm = (MF(conv) & 2) != 0;
    const int nrg = MF(nrg), nu4 = MF(nu4);
    const CU32* rx = (const CU32*)((const char*)MF(img) + Lay<1>::IMG_RX);
    // kf, kr come from the lane's global rows: prefetched PF reactions ahead (a register ring)
    constexpr int PF = 3;
    double kq[PF][2];
#pragma unroll
    for (int d = 0; d < PF; ++d) {
        const int rr = d < nrg ? d : 0;
        kq[d][0] = G.ld(LL.g_rxd + 2 * rr);
        kq[d][1] = G.ld(LL.g_rxd + 2 * rr + 1);
    }
    for (int r = 0; r < nrg; ++r) {
        const auto rec = rx_rec(rx, r);
        const uint32_t w0 = rec[0], w1 = rec[1], info = rec[2], sw[4] = {rec[4], rec[5], rec[6], rec[7]};
        const double kf = kq[0][0], kr = kq[0][1];
#pragma unroll
        for (int d = 0; d < PF - 1; ++d) { kq[d][0] = kq[d + 1][0]; kq[d][1] = kq[d + 1][1]; }
        {
            const int rr = r + PF < nrg ? r + PF : 0;
            kq[PF - 1][0] = G.ld(LL.g_rxd + 2 * rr);
            kq[PF - 1][1] = G.ld(LL.g_rxd + 2 * rr + 1);
        }
        double Pf = (Lp[(LL.conc + lane_sp(w0, 0, n)) * 64] * Lp[(LL.conc + lane_sp(w0, 1, n)) * 64]) *
                    Lp[(LL.conc + lane_sp(w0, 2, n)) * 64];
        double Pb = (Lp[(LL.conc + lane_sp(w1, 0, n)) * 64] * Lp[(LL.conc + lane_sp(w1, 1, n)) * 64]) *
                    Lp[(LL.conc + lane_sp(w1, 2, n)) * 64];
        if (nu4) { Pf *= Lp[(LL.conc + lane_sp(w0, 3, n)) * 64]; Pb *= Lp[(LL.conc + lane_sp(w1, 3, n)) * 64]; }
        double D = kf * Pf - kr * Pb;
        const int tbk = gi_tb(info);
        if (tbk) {
            const double Mc = Lp[(LL.mc + gi_tbidx(info)) * 64];
            if (tbk == 1) {
                D *= Mc;
            } else {                                            // Lindemann / Troe falloff
                const int fi = gi_foidx(info);
                const double Pr = G.ld(LL.g_fod + 4 * fi) * Mc;     // k0/k_inf [M]
                double F = 1.0;
                if (gi_troe(info)) {
                    const double fo[4] = {0.0, G.ld(LL.g_fod + 4 * fi + 1), G.ld(LL.g_fod + 4 * fi + 2),
                                          G.ld(LL.g_fod + 4 * fi + 3)};
                    double x, den;
                    F = troe_F(Pr, fo, x, den);
                }
                D *= Pr / (1 + Pr) * F;
                if (xm) D *= Mc * 1e-6;                         // [M] in mol/cm3
            }
        }
        const int cnt = (int)(sw[3] >> 24);
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            if (e < cnt) {
                const int k = (int)(sl_off(sw[e >> 1], e & 1) >> 3);
                const int nu = sl_nu(sw[3], e);
                lds_add(&Lp[(LL.acc + k) * 64], (double)nu * D);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NM; ++k) f[k] = (k < n) ? Lp[(LL.acc + k) * 64] * mw[k] : 0.0;
}

// analytic Jacobian d(du)/du of the lane's reactor (gas only, du_k = M_k sum_r nu_kr q_r,
// c_j = u_j / M_j), at the state of the RHS just evaluated (its concentrations and third-body sums
// are still in the lane's LDS rows), column-major into the lane's saved-J rows: element (i, j) at
// row j * NM + i. Same derivative terms as the wavefront engine and the oracle (jac_tc):
// mass-action partial products, third-body / falloff d[M] columns.
template <int NM>
__device__ __forceinline__ void lane_jac(const LaneLay& LL, const double* Lp, const GRows& G, int n) {
    const CF64* mw = (const CF64*)MF(img);
    const bool xm = (MF(conv) & 2) != 0;
    const int nrg = MF(nrg);
    const CU32* rx = (const CU32*)((const char*)MF(img) + Lay<1>::IMG_RX);
    const CU32* tbs = (const CU32*)((const char*)MF(img) + MF(tbs_off));
    const char* tbe = (const char*)MF(img) + MF(tbe_off);
#pragma unroll
    for (int j = 0; j < NM; ++j)
#pragma unroll
        for (int i = 0; i < NM; ++i) G.st(j * NM + i, 0.0);
    for (int r = 0; r < nrg; ++r) {
        const auto rec = rx_rec(rx, r);
        const uint32_t w0 = rec[0], w1 = rec[1], info = rec[2], sw[4] = {rec[4], rec[5], rec[6], rec[7]};
        const double kf = G.ld(LL.g_rxd + 2 * r), kr = G.ld(LL.g_rxd + 2 * r + 1);
        double cf[4], cb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            cf[e] = Lp[(LL.conc + lane_sp(w0, e, n)) * 64];
            cb[e] = Lp[(LL.conc + lane_sp(w1, e, n)) * 64];
        }
        const double D = kf * (cf[0] * cf[1] * cf[2] * cf[3]) - kr * (cb[0] * cb[1] * cb[2] * cb[3]);
        double pre = 1.0, coefM = 0.0;
        const int tbk = gi_tb(info);
        if (tbk) {
            const double Mc = Lp[(LL.mc + gi_tbidx(info)) * 64];
            if (tbk == 1) { pre = Mc; coefM = 1.0; }
            else {
                const int fi = gi_foidx(info);
                double fo[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) fo[c] = G.ld(LL.g_fod + 4 * fi + c);
                double fac, dfac;
                falloff<true>(fo, gi_troe(info) != 0, Mc, fac, dfac);
                const double xs = xm ? Mc * 1e-6 : 1.0;                   // [M] in mol/cm3 (reference)
                pre = fac * xs;
                coefM = dfac * xs + (xm ? fac * 1e-6 : 0.0);
            }
        }
        double dq[NM];                                                 // d q_r / d c_j
#pragma unroll
        for (int j = 0; j < NM; ++j) dq[j] = tbk ? D * coefM : 0.0;
        if (tbk) {                                                     // non-unit efficiencies
            const uint32_t w = tbs[gi_tbidx(info)];
            const int b = w & 0xFFFFF, e = b + (int)(w >> 20);
            for (int t = b; t < e; ++t) {
                const int k = *(const CU32*)(tbe + 16 * t) & 0xFFFF;
                const double em1 = *(const CF64*)(tbe + 16 * t + 8);
#pragma unroll
                for (int j = 0; j < NM; ++j) dq[j] += (j == k) ? D * coefM * em1 : 0.0;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int kfs = (int)((w0 >> (8 * e)) & 255), kbs = (int)((w1 >> (8 * e)) & 255);
            double pf = kf * pre, pb = -kr * pre;
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) if (e2 != e) { pf *= cf[e2]; pb *= cb[e2]; }
#pragma unroll
            for (int j = 0; j < NM; ++j) {
                dq[j] += (j == kfs) ? pf : 0.0;                         // pad slots (SP_ONE) match no j
                dq[j] += (j == kbs) ? pb : 0.0;
            }
        }
        const int cnt = (int)(sw[3] >> 24);
        for (int e = 0; e < cnt; ++e) {                                // rows of the touched species
            const uint32_t we = (e >> 1) == 0 ? sw[0] : ((e >> 1) == 1 ? sw[1] : sw[2]);   // (uniform selects)
            const int k = (int)(sl_off(we, e & 1) >> 3);
            const int nu = sl_nu(sw[3], e);
            const double sk = (double)nu * mw[k];
#pragma unroll
            for (int j = 0; j < NM; ++j)
                if (j < n) G.st(j * NM + k, G.ld(j * NM + k) + sk * dq[j] / mw[j]);
        }
    }
}

// ------------------------------------------------------------------------------------
// the lane integrator kernel (persistent grid; 64-thread workgroups, one wave each)
// ------------------------------------------------------------------------------------
template <int NM>
__global__ __launch_bounds__(64) void k_lane(DevMech M, int N, const double* __restrict__ Tv, double* __restrict__ U,
                                             const double* __restrict__ tfv, KOpts o, double* __restrict__ stats,
                                             double* __restrict__ Jg, int* __restrict__ queue, double* __restrict__ defer_t0,
                                             int defer_cap) {
    // queue[0]: next reactor; queue[1]: deferred count; queue[2 ..]: deferred reactor ids;
    // defer_t0[i]: the time of deferred entry i's last accepted state
    const int lane = threadIdx.x;
    const int n = MF(n);
    const LaneLay LL = lane_lay(NM, n, MF(nset), MF(nrg), MF(nfo));
    double* Lp = reinterpret_cast<double*>(br_lds) + lane;
    Lp[(LL.conc + n) * 64] = 1.0;
    GRows G;
    G.r = __builtin_amdgcn_make_buffer_rsrc(Jg, 0, 0x7fffffff, 0x00020000);
    G.vo = lane * 8;
    G.base = blockIdx.x * LL.g_rows * 512;

    LCV c;
    ZH<NM> z;
    z.Lz = Lp + LL.zh * 64;
    z.n = n;
    double acor[NM], ewt[NM], y[NM];
    unsigned long long pv = 0;   // pivot rows of the lane's current LU factors (4 bits each)
#pragma unroll
    for (int i = 0; i < NM; ++i) y[i] = 0.0;
    int rid = 0;
    bool has = false, drained = false;
    unsigned long long cyc0 = 0;
#if BR_PHASE_CLOCKS
    unsigned long long k_rhs = 0, k_ref = 0, k_lu = 0, k_sol = 0, k_ctl = 0, k_all = 0;
#endif
    for (;;) {
        LCLK(t0);
        if (!has && !drained) {                              // take the next reactor
            rid = atomicAdd(queue, 1);
            if (rid < N) {
                has = true;
                cyc0 = wall_clock64();
#if BR_PHASE_CLOCKS
                k_rhs = k_ref = k_lu = k_sol = k_ctl = 0; k_all = clock64();
#endif
                lane_tconst(LL, Lp, G, Tv[rid], n);
                double su = 0.0;
#pragma unroll
                for (int i = 0; i < NM; ++i) {
                    const double u0 = i < n ? U[(size_t)rid * n + i] : 0.0;
#pragma unroll
                    for (int j = 1; j <= QMAX; ++j) z.set(j, i, 0.0);
                    z.z0[i] = u0;
                    y[i] = u0;
                    acor[i] = 0.0;
                    ewt[i] = i < n ? 1.0 / (o.rtol * fabs(u0) + o.atol) : 1.0;
                    su += fabs(u0);
                }
        #pragma unroll
                for (int i = 0; i < QMAX + 2; ++i) { c.tau[i] = 0.0; c.l[i] = 0.0; }
#pragma unroll
                for (int i = 0; i < 6; ++i) c.tq[i] = 0.0;
                c.tn = 0.0; c.h = 0.0; c.hprime = 0.0; c.hscale = 0.0; c.eta = 1.0; c.etamax = ETAMX1;
                c.rl1 = 0.0; c.gamma = 0.0; c.gammap = 0.0; c.gamrat = 1.0; c.crate = 1.0; c.delp = 0.0;
                c.acnrm = 0.0; c.saved_tq5 = 0.0; c.saved_t = 0.0; c.tol = 0.0; c.hg = 0.0; c.hub = 0.0;
                c.hlb = 0.0; c.tstop = tfv[rid]; c.ulimit = o.ufac > 0.0 ? o.ufac * su : INFINITY; c.minInc = 0.0;
                c.q = 1; c.qprime = 1; c.L = 2; c.qwait = 2;
                c.nst = 0; c.nfe = 0; c.nsetups = 0; c.nje = 0; c.nni = 0; c.ncfn = 0; c.netf = 0;
                c.nstlp = 0; c.nstlj = 0; c.ncf = 0; c.nef = 0; c.nstloc = 0; c.status = 0; c.m_it = 0;
                c.convfail = 0; c.count1 = 0; c.phase = PH_F0; c.callSetup = 0; c.jbad = 0; c.jcur_nls = 0;
                c.hnewOK = 0; c.jcol = 0; c.pend = PEND_NONE; c.pflag = 0;
                c.rid = rid; c.iout = 0; c.ign_t = 0.0; c.ign_rate = -INFINITY; c.t_ign = NAN; c.ign_dt = NAN;
                c.ign_x = o.ign >= 0 ? l_mole_frac<NM>(y, n, o.ign) : 0.0;
                while (c.iout < o.nout && !(o.tout[c.iout] > 0.0)) {   // outputs at t <= 0: u0
                    double* row = o.yout + ((size_t)rid * o.nout + c.iout) * n;
#pragma unroll
                    for (int i = 0; i < NM; ++i) if (i < n) row[i] = y[i];
                    c.iout += 1;
                }
            } else {
                drained = true;
            }
        }
        if (!__any(has)) break;                              // uniform: the whole wave leaves together
        LACC(k_ref, t0);
        LCLK(t1);
        double f[NM];
        lane_rhs<NM>(LL, Lp, G, y, n, f);
        LACC(k_rhs, t1);
        LCLK(t2);
        double b[NM];
#pragma unroll
        for (int i = 0; i < NM; ++i) b[i] = 0.0;
        int act = A_NONE;
        if (has) act = l_post_rhs<NM>(c, z, acor, ewt, y, f, b, Lp, LL, G, o, n);
        LACC(k_ctl, t2);
        LCLK(t3);
        int lu_fail = 0;
        if (__any(act == A_SETUP)) {
            if (act == A_SETUP) {                            // A = I - gamma J from the saved J
                const double mg = -c.gamma;
                double a[NM][NM], rpv[NM];
#pragma unroll
                for (int j = 0; j < NM; ++j)
#pragma unroll
                    for (int i = 0; i < NM; ++i) a[i][j] = (i < n && j < n) ? G.ld(j * NM + i) : 0.0;
                __builtin_amdgcn_sched_barrier(0);   // one burst of loads, then the factorisation
#pragma unroll
                for (int j = 0; j < NM; ++j)
#pragma unroll
                    for (int i = 0; i < NM; ++i) a[i][j] = a[i][j] * mg + (i == j ? 1.0 : 0.0);
                lu_fail = l_getrf<NM>(a, pv, rpv);
#pragma unroll
                for (int j = 0; j < NM; ++j) {
                    G.st(LL.g_rpv + j, rpv[j]);
#pragma unroll
                    for (int i = 0; i < NM; ++i) G.st(LL.g_lu + j * NM + i, a[i][j]);
                }
            }
        }
        LACC(k_lu, t3);
        LCLK(t4);
        const bool solve = (act == A_SOLVE) || (act == A_SETUP && !lu_fail);
        if (__any(solve)) {
            if (solve) l_getrs<NM>(G, LL, pv, b);
        }
        LACC(k_sol, t4);
        LCLK(t5);
        if (act == A_SOLVE || act == A_SETUP) act = l_post_solve<NM>(c, z, acor, ewt, y, b, lu_fail, o, n);
        if (act == A_RHS && c.pend != PEND_NONE) l_run_pending<NM>(c, z, acor, ewt, y, o, n);
        LACC(k_ctl, t5);
        if (act == A_DONE && c.status == ST_DEFER) {
            const int di = atomicAdd(queue + 1, 1);
            if (di < defer_cap) {                            // hand over the last accepted state
                queue[2 + di] = rid;
                defer_t0[di] = c.tn;
#pragma unroll
                for (int i = 0; i < NM; ++i) if (i < n) U[(size_t)rid * n + i] = z.z0[i];
                if (stats) {                                 // counters so far (the wave pass adds its own)
                    double* st = stats + (size_t)rid * BR_NSTAT;
                    st[0] = (double)c.nst; st[1] = (double)c.nfe; st[2] = (double)c.nje; st[3] = (double)c.nsetups;
                    st[4] = (double)c.nni; st[5] = (double)c.ncfn; st[6] = (double)c.netf;
                    st[16] = c.t_ign; st[17] = c.ign_rate; st[18] = c.ign_dt;
                    st[19] = o.dq_jac ? (double)c.nje * n : 0.0;   // nfe_dq
                }
                has = false;
            } else {                                         // no room: keep integrating here
                c.status = 0;
                c.pend = PEND_STEP;
                l_run_pending<NM>(c, z, acor, ewt, y, o, n);
            }
            act = A_RHS;
        }
        if (act == A_DONE) {
            const int status = c.status;
#pragma unroll
            for (int i = 0; i < NM; ++i)
                if (i < n) U[(size_t)rid * n + i] = status ? z.z0[i] : y[i];
            if (stats) {
                double* st = stats + (size_t)rid * BR_NSTAT;
                st[0] = (double)c.nst; st[1] = (double)c.nfe; st[2] = (double)c.nje; st[3] = (double)c.nsetups;
                st[4] = (double)c.nni; st[5] = (double)c.ncfn; st[6] = (double)c.netf; st[7] = (double)status;
                st[8] = (double)(wall_clock64() - cyc0);
#if BR_PHASE_CLOCKS
                st[9] = (double)k_rhs; st[10] = (double)k_ref; st[11] = (double)k_lu; st[12] = (double)k_sol;
                st[14] = (double)k_ctl; st[15] = (double)(clock64() - k_all);
#else
                st[9] = st[10] = st[11] = st[12] = st[14] = st[15] = 0.0;
#endif
                st[13] = c.tn;
                st[16] = o.ign >= 0 ? c.t_ign : NAN; st[17] = o.ign >= 0 ? c.ign_rate : NAN;
                st[18] = o.ign >= 0 ? c.ign_dt : NAN; st[19] = o.dq_jac ? (double)c.nje * n : 0.0;   // nfe_dq
            }
            has = false;
        }
    }
}
