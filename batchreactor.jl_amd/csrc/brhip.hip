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
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/brhip.h"
#ifndef BR_ASM_MARKS
#define BR_ASM_MARKS 0
#endif
#ifndef BR_PHASE_CLOCKS
#define BR_PHASE_CLOCKS 0   // per-phase shader-clock counters in br_stats (diagnostic build: libbrhip_diag.so)
#endif
#include "brhip_device.hpp"
// Diagnostic-only instruction-count experiments (scripts/micro/exp_hooks.hpp: a phase run twice,
// extra VALU or memory work per Newton iteration) attach at these points of k_integrate; the
// product build leaves them empty.
#ifdef BR_EXPERIMENT_HOOKS
#include BR_EXPERIMENT_HOOKS
#endif
#ifndef BR_X_AFTER_RHS
#define BR_X_AFTER_RHS()
#define BR_X_AFTER_JAC()
#define BR_X_AFTER_SOLVE()
#define BR_X_AFTER_ITER()
#endif
#ifndef BR_XC_AFTER_CVSET   // ... and inside the controller (cvSet, the step-size ratio root)
#define BR_XC_AFTER_CVSET()
#define BR_XC_AFTER_ETAQ()
#endif
#ifndef BR_XG_AFTER_RHS   // the same for k_group (brhip_group.hpp)
#define BR_XG_AFTER_RHS()
#define BR_XG_AFTER_JAC()
#define BR_XG_AFTER_LU()
#define BR_XG_AFTER_SOLVE()
#endif

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
    int ign;                  // gas species index of the ignition marker (-1: not tracked)
    int nout;                 // dense output: tout[nout] (device), yout[N][nout][n] (device)
    const double* tout;
    double* yout;
    int dq_jac;               // CVODE's DQ Jacobian (br_opts.dq_jacobian) instead of the analytic one (both engines)
    int defer_steps;          // k_lane: hand a reactor still running after this many steps to the
                              // wavefront engine (restart from u0); >= max_steps disables
    const int* rid_list;      // k_integrate: integrate reactors rid_list[0 .. min(*rid_count, N)) only
    const int* rid_count;
    const double* rid_t0;     // with rid_list: start time of list entry i (a deferred lane reactor
                              // continues from its last accepted state U[rid] at rid_t0[i]: CVODE
                              // restart there) and its counters so far are in stats[rid]
    int* work;                // k_integrate: persistent waves take reactor indices from this
                              // counter (nullptr: one reactor per wave, index = wave slot)
};

// ------------------------------------------------------------------------------------
// per-reactor LDS block: [Ctl: CVODE's cv_mem scalars][Vec: per-lane vectors][Smem: rate work]
//
// The kernel keeps only the hot path inline (RHS, Jacobian, LU, solve). All step control lives
// in two __noinline__ functions that read and write this block through address-space-3
// pointers, so their register allocation is isolated from the hot path's (no spills there, and
// the VGPR file stays free for the row-per-lane Newton matrix). Every lane writes the same
// uniform value; reads go through readfirstlane, so branches on them are scalar.
// ------------------------------------------------------------------------------------
struct Ctl {
    double p_last;
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double tn, h, rl1, gamma, gamrat, gammap, crate, delp;
    double hprime, hscale, eta, etamax, acnrm, saved_tq5, saved_t, tol;
    double hg, hub, hlb, hnew, ulimit, tstop;
    int q, qprime, L, qwait;
    int nst, nfe, nsetups, nje, nni, ncfn, netf, nstlp, nstlj;
    int ncf, nef, nstloc, status, m_it, convfail, count1, phase;
    int callSetup, jbad, jcur_nls, hnewOK, newj;
    // ignition marker (max dX_ign/dt over accepted steps) and dense-output cursor
    double ign_x, ign_t, ign_rate, t_ign, ign_dt;
    double dq_mininc;         // CVODE's DQ Jacobian: minInc of the Jacobian being built
    int nfe_dq;               // RHS evaluations of the DQ Jacobian (CVODE's nfeDQ)
    int iout;
    // per-launch constants (here rather than in registers: they are read once per step)
    double a_rtol, a_atol, a_hmax_inv, a_ufac;
    double* a_trace;
    const double* a_tout;
    double* a_yout;
    int a_max_steps, a_trace_cap, a_rid, a_n, a_ign, a_nout;
};
constexpr int CTL_BYTES = (sizeof(Ctl) + 15) / 16 * 16;
enum { V_Z0 = 0, V_ACOR = QMAX + 1, V_EWT, V_TEMP, V_Y, NVEC };   // z0..z5, acor, ewt, tempv, y
// V[vec * 64 + lane] for the first component slot. Two components per lane (n = 65..72): slot 1 of
// vector j (components 64..71, lanes 0..7) at V1OFF + 8 j + lane; lanes 8..63 of slot 1 (components
// 72..127, never real) at V1OFF + 8 j + 72 + lane, a dump region whose entries alias only each other.
// Every access is then base + per-lane constant + 8 j (an immediate): no per-vector select that
// the compiler would hoist out of the integrator loop and keep live (40 VGPRs spilled at 3 waves/
// SIMD with the previous 72-wide rows and one shared dump row). 6.6 KB per gas+surface reactor.
constexpr int V1OFF = NVEC * 64;
// BR_VS32 = 1: k_integrate<32> (16 < n <= 32) keeps its vectors 32 wide (VS = 32): lanes 32..63 hold
// no component, read the entry of lane - 32 (a finite value every use of theirs masks: norms, maxima
// and outputs test component < n) and never store (VProxy below). 2.5 KB less LDS per reactor.
#ifndef BR_VS32
#define BR_VS32 1
#endif
__host__ __device__ constexpr int vec_stride(int nmax) { return (BR_VS32 && nmax == 32) ? 32 : 64; }
__host__ __device__ constexpr int nmax_of(int n) { return n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 56 ? 56 : (n <= 64 ? 64 : 72))); }
__host__ __device__ inline int vec_bytes(int cpl, int vs = 64) {
    return cpl == 2 ? (V1OFF + 8 * (NVEC - 1) + 72 + 64) * 8 : NVEC * vs * 8;
}
typedef __attribute__((address_space(3))) double LDbl;
// an entry of a VS < 64 vector: loads by every lane, stores by lanes < VS only
struct VProxy {
    LDbl* a;
    bool w;
    __device__ __forceinline__ operator double() const { return *a; }
    __device__ __forceinline__ VProxy& operator=(double x) { if (w) *a = x; return *this; }
    __device__ __forceinline__ VProxy& operator=(const VProxy& o) { return *this = (double)o; }
    __device__ __forceinline__ VProxy& operator+=(double x) { return *this = (double)*this + x; }
    __device__ __forceinline__ VProxy& operator-=(double x) { return *this = (double)*this - x; }
    __device__ __forceinline__ VProxy& operator*=(double x) { return *this = (double)*this * x; }
};
// Nordsieck / work vectors in the reactor's LDS block: V.at(vec, s) = component lane + 64 s of
// vector vec. (Register-resident vectors stored to LDS around each Newton setup measured GRI
// -1.1 %, surf -11 % in round 2: the extra VGPRs cost occupancy.)
template <int CPL, int GW = 64, int VS = GW>
struct VA {
    typedef __attribute__((address_space(3))) double LD;
    LD* p;
    int lane;
    __device__ __forceinline__ decltype(auto) at(int j, int s) const {
        if constexpr (VS < GW) {
            static_assert(CPL == 1, "narrow vectors: one component per lane");
            // lanes >= VS read a real entry (lane - VS for a power-of-2 width, else the last one)
            const int li = (VS & (VS - 1)) == 0 ? (lane & (VS - 1)) : (lane < VS ? lane : VS - 1);
            return VProxy{&p[j * VS + li], lane < VS};
        } else {
            if (CPL == 1 || s == 0) return static_cast<LD&>(p[j * GW + lane]);
            return static_cast<LD&>(p[V1OFF + 8 * j + (lane < 8 ? lane : 72 + lane)]);
        }
    }
};
template <int CPL, int GW = 64> using VT = VA<CPL, GW>;
// component slot s's value of vector j for a uniform j in [0, QMAX + 1] (register arrays cannot be
// indexed dynamically: a select chain, scalar branches on the uniform j)
template <int CPL, class V_>
__device__ __forceinline__ double vget(V_& V, int j, int s) {
    double r = 0.0;
#pragma unroll
    for (int jj = 0; jj <= QMAX + 1; ++jj) if (jj == j) r = V.at(jj, s);
    return r;
}
template <int CPL, class V_>
__device__ __forceinline__ void vset(V_& V, int j, int s, double x) {
#pragma unroll
    for (int jj = 0; jj <= QMAX + 1; ++jj) if (jj == j) V.at(jj, s) = x;
}
typedef __attribute__((address_space(3))) Ctl LCtl;

__host__ __device__ inline size_t reactor_bytes(const DevMech& M) {
    return CTL_BYTES + vec_bytes(M.cpl, vec_stride(nmax_of(M.n))) + (size_t)M.rblock_bytes;
}
__host__ __device__ inline size_t wg_lds_bytes(const DevMech& M, int rpb) { return M.img_bytes + rpb * reactor_bytes(M); }
// per-reactor global workspace (doubles): saved J, LU factors, Jacobian scratch (2 per gas rxn);
// matrix columns hold 64 * CPL rows (CPL = 2 for nmax > 64)
__host__ __device__ inline int col_rows(int nmax) { return nmax > 64 ? CR2 : 64; }   // CR2 = 80 (lu_factor2)
// factors + D^-1: CPL = 1 NMAX columns of NMAX rows + 64 (lu_factor), CPL = 2 NMAX + 1 columns of CR2 rows
__host__ __device__ inline size_t lu_ws_doubles(int nmax) {
    return nmax > 64 ? (size_t)(nmax + 1) * CR2 : (size_t)nmax * nmax + WAVE;
}
// [J | LU factors, aliased by the Jacobian scratch (2 per gas reaction) | RXD: {kf, kr} per gas
// reaction]. The scratch is live only while a new J is built, and every new J is followed by a
// factorization that overwrites the old factors, so the two share one region (-5.2 KB per GRI
// slot; with NMAX-row factor columns 4096 slots of 60 KB = 245 MB against the 256 MB Infinity Cache).
__host__ __device__ inline size_t lu_area_doubles(int nmax, int nrg) {
    const size_t a = lu_ws_doubles(nmax), b = (((size_t)2 * nrg + 63) / 64) * 64;
    return a > b ? a : b;
}
__host__ __device__ inline size_t rxd_ws_off(int nmax, int nrg) {
    return (size_t)nmax * col_rows(nmax) + lu_area_doubles(nmax, nrg);
}
__host__ __device__ inline size_t ws_doubles(int nmax, int nrg) {
    return rxd_ws_off(nmax, nrg) + (((size_t)2 * nrg + 63) / 64) * 64;
}

struct WaveCtx {
    int wave, lane, rid;
    Tab tb;
    char* rbase;   // this wave's reactor block
    RView R;
};
// ws: the global workspace, NMAX-instance slots (slot = wave index rid)
template <int CPL, int NMAX>
__device__ __forceinline__ WaveCtx wave_ctx(const DevMech& M, char* smem, int rpb, double* ws) {
    WaveCtx w;
    w.wave = uni((int)(threadIdx.x >> 6));   // uniform per wave: scalar addressing of its reactor
    w.lane = threadIdx.x & 63;
    w.rid = blockIdx.x * rpb + w.wave;
    stage_tables(M, smem);
    w.tb = tab_view<CPL>(smem, M);
    w.rbase = smem + M.img_bytes + (size_t)w.wave * reactor_bytes(M);
    // (the vector width follows n, as reactor_bytes: the rates / Jacobian kernels run as NMAX 64)
    w.R = rview<CPL>(w.rbase + CTL_BYTES + vec_bytes(CPL, vec_stride(nmax_of(M.n))), M,
                     launder(ws + (size_t)w.rid * ws_doubles(NMAX, M.nrg) + rxd_ws_off(NMAX, M.nrg)));
    return w;
}

// loads from the LDS controller: ints through v_readfirstlane (SGPRs: scalar branches and loop
// bounds); doubles stay in VGPRs (every lane reads the same value; fp64 arithmetic runs on the VALU
// either way, and the two readfirstlanes per value were VALU instructions of their own: GRI +0.7 %,
// surface-only +2.7 %, round 3)
__device__ __forceinline__ double ud(const LDbl& x) { return (double)x; }
__device__ __forceinline__ int ui(const __attribute__((address_space(3))) int& x) { return uni((int)x); }
// Reactor groups: the wavefront engine runs one reactor per wave (group width GW = 64); the group
// engines (brhip_group.hpp) two or four per wave, one per 32-lane half or 16-lane DPP row (GW = 32 /
// 16), with `lane` the lane within the group. The controller's values are uniform per group: scalar
// for GW = 64 (readfirstlane: SGPRs, scalar branches), per-lane VGPRs with exec-masked branches for
// GW < 64; reductions and broadcasts over the group (DPP row butterflies, permlane16 swaps between
// the rows of a half, ds_bpermute inside the group).
template <int GW>
__device__ __forceinline__ int gui(const __attribute__((address_space(3))) int& x) {
    if constexpr (GW == 64) return uni((int)x);
    else return (int)x;
}
template <int GW>
__device__ __forceinline__ int guni(int v) {
    if constexpr (GW == 64) return uni(v);
    else return v;
}
template <int GW>
__device__ __forceinline__ double guni(double v) {
    if constexpr (GW == 64) return uni(v);
    else return v;
}
template <int GW>
__device__ __forceinline__ double gsum(double v) {
    if constexpr (GW == 64) return wave_sum(v);
    else if constexpr (GW == 32) return half_sum(v);
    else return row_sum(v);
}
template <int GW>
__device__ __forceinline__ double gmax(double v) {
    if constexpr (GW == 64) return wave_max(v);
    else if constexpr (GW == 32) return half_max(v);
    else return row_max(v);
}
// value of v in lane k of the group (k uniform per group)
template <int GW>
__device__ __forceinline__ double gbcast(double v, int k) {
    if constexpr (GW == 64) return bcast(v, k);
    else return lane_pull(v, (int)(threadIdx.x & (64 - GW)) + k);
}

// analysis builds (BR_ASM_QMARKS): region markers in the 16-lane controller's ISA listing
#ifdef BR_ASM_QMARKS
#define BR_QMARK(name) do { if constexpr (GW == 16) asm volatile("; QMARK " #name); } while (0)
#else
#define BR_QMARK(name) do { } while (0)
#endif
#ifndef BR_CTL_INLINE
#define BR_CTL_INLINE __forceinline__
#endif
enum { PH_F0 = 0, PH_HIN = 1, PH_NEWTON = 2, PH_EF1 = 3 };
// action codes returned by the controller to the hot loop
enum { A_RHS = 0, A_SOLVE = 1, A_SETUP = 2, A_DONE = 3 };

// wrms norm of the lane's component values (components lane + 64 s) with weights ewt
template <int CPL, int GW = 64>
__device__ __forceinline__ double wrms_l(const double (&v)[CPL], const double (&ewt)[CPL], int lane, int n) {
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < CPL; ++s) {
        const double t = (lane + 64 * s < n) ? v[s] * ewt[s] : 0.0;
        acc += t * t;
    }
    return guni<GW>(sqrt(gsum<GW>(acc) / n));
}
// per-component slot loops over the lane's components c = lane + 64 s
#define FOR_S for (int s = 0; s < CPL; ++s)
#define CS (lane + 64 * s)

struct CtlArgs {   // per-launch constants the controller needs, read (uniform) from the LDS controller
    double rtol, atol, hmax_inv, ufac;
    // (global-address-space pointers: generic ones compile to flat accesses, which count on both the
    // memory and the LDS counter and make the waitcnt pass fall back to full waits after them)
    BR_GLOBAL double* trace;
    const BR_GLOBAL double* tout;
    BR_GLOBAL double* yout;
    int max_steps, trace_cap, rid, n, ign, nout;
};
// uniform 64-bit pointer from the LDS controller
template <class P>
__device__ __forceinline__ P ld_ptr(const __attribute__((address_space(3))) P& f) {
    const volatile __attribute__((address_space(3))) unsigned long long& tp =
        *reinterpret_cast<const volatile __attribute__((address_space(3))) unsigned long long*>(&f);
    const unsigned long long tv = tp;
    const unsigned lo = (unsigned)uni((int)(tv & 0xffffffffull)), hi = (unsigned)uni((int)(tv >> 32));
    return reinterpret_cast<P>(((unsigned long long)hi << 32) | lo);
}
template <int GW = 64>
__device__ __forceinline__ CtlArgs load_args(LCtl* C) {
    CtlArgs a;
    a.rtol = ud(C->a_rtol); a.atol = ud(C->a_atol); a.hmax_inv = ud(C->a_hmax_inv); a.ufac = ud(C->a_ufac);
    a.trace = launder(ld_ptr(C->a_trace));
    a.tout = launder(ld_ptr(C->a_tout));
    a.yout = launder(ld_ptr(C->a_yout));
    a.max_steps = gui<GW>(C->a_max_steps); a.trace_cap = gui<GW>(C->a_trace_cap); a.rid = gui<GW>(C->a_rid); a.n = gui<GW>(C->a_n);
    a.ign = gui<GW>(C->a_ign); a.nout = gui<GW>(C->a_nout);
    return a;
}

// mole fraction of gas species k in state v (components lane + 64 s): (v_k/M_k) / sum_j v_j/M_j
template <int CPL, int GW = 64>
__device__ __forceinline__ double mole_frac_of(const double (&v)[CPL], int lane, int k) {
    const double* mw = reinterpret_cast<const double*>(br_lds);   // staged molwt[] (image offset 0)
    const int ng = MF(ng);
    double g = 0.0, c0 = 0.0, c1 = 0.0;
#pragma unroll
    FOR_S if (CS < ng) { const double c = v[s] / mw[CS]; g += c; if (s == 0) c0 = c; else c1 = c; }
    const double ck = (k < 64) ? gbcast<GW>(c0, k) : gbcast<GW>(c1, k - 64);   // k uniform: one readlane pair
    return ck / gsum<GW>(g);
}
// ignition marker after an accepted step to (tn, v): midpoint of the step with the largest dX/dt
template <int CPL, int GW = 64>
__device__ __forceinline__ void track_ignition(LCtl* C, const CtlArgs& a, int lane, double tn, const double (&v)[CPL]) {
    const double x = guni<GW>(mole_frac_of<CPL, GW>(v, lane, a.ign));
    const double t0 = ud(C->ign_t), xp = ud(C->ign_x), rate = ud(C->ign_rate);
    const double dt = tn - t0;   // > 0 (accepted step): compare without the division, divide on a new max
    if (x - xp > rate * dt) {
        const double r = (x - xp) / dt;
        if (r > rate) { C->ign_rate = r; C->t_ign = 0.5 * (t0 + tn); C->ign_dt = dt; }
    }
    C->ign_x = x; C->ign_t = tn;
}
// dense output (CVode CV_NORMAL): every tout in (t_{n-1}, t_n] from the Nordsieck array of the step
// just completed, y(t) = sum_j z_j ((t - tn)/h)^j (CVodeGetDky, k = 0)
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void dense_output(LCtl* C, VA<CPL, GW, VS>& V, const CtlArgs& a, int lane, double tn, double h, int q,
                                             double tlim) {
    int io = gui<GW>(C->iout);
    while (io < a.nout) {
        const double t = guni<GW>(a.tout[io]);
        if (!(t <= tlim)) break;
        const double sk = (t - tn) / h;
        auto row = a.yout + ((size_t)a.rid * a.nout + io) * a.n;
#pragma unroll
        FOR_S {
            double yv = vget<CPL>(V, q, s);
#pragma unroll
            for (int j = QMAX - 1; j >= 0; --j) if (j < q) yv = V.at(j, s) + sk * yv;
            if (CS < a.n) row[CS] = yv;
        }
        ++io;
    }
    C->iout = io;
}

// 1.0 / j for the small integers of the BDF coefficient formulas (exactly the rounded quotient)
// (j is in 1 .. QMAX + 1 at every call site; no run-time division for the impossible rest: with
// per-lane j it was evaluated on every call, ~11 VALU each)
__device__ __forceinline__ double inv_int(int j) {
    return j == 1 ? 1.0 : j == 2 ? 0.5 : j == 3 ? 1.0 / 3.0 : j == 4 ? 0.25 : j == 5 ? 0.2 : 1.0 / 6.0;
}

// the controller scalars one attempt (predict + cvSet) reads, loaded in one batch before the
// prediction's Nordsieck stores (V shares LDS with the controller: a load after a V store waits)
struct AttemptIn {
    int q, qwait, nst, nstlp;
    double h, tn, tstop, gammap;
    double tau[QMAX + 2];
};
template <int GW = 64>
__device__ __forceinline__ AttemptIn load_attempt(LCtl* C) {
    AttemptIn in;
    in.q = gui<GW>(C->q); in.qwait = gui<GW>(C->qwait); in.nst = gui<GW>(C->nst); in.nstlp = gui<GW>(C->nstlp);
    in.h = ud(C->h); in.tn = ud(C->tn); in.tstop = ud(C->tstop); in.gammap = ud(C->gammap);
#pragma unroll
    for (int i = 0; i < QMAX + 2; ++i) in.tau[i] = ud(C->tau[i]);
    return in;
}
// cvSet (BDF coefficients l[], tq[], gamma) for the current q, h, tau
template <int GW = 64>
__device__ __forceinline__ void cv_set(LCtl* C, const AttemptIn& in, double& tq4_out, double& gamrat_out) {
    const int q = in.q, qwait = in.qwait, nst = in.nst;
    const double h = in.h;
    double lv[QMAX + 1] = {1.0, 1.0, 0.0, 0.0, 0.0, 0.0};
    double tau[QMAX + 2];
#pragma unroll
    for (int i = 0; i < QMAX + 2; ++i) tau[i] = in.tau[i];
    // h / hsum_m for every m up front (hsum_m = h + tau[1] + ... + tau[m-1], summed in CVODE's
    // order): the divisions are independent, so they overlap instead of forming a chain
    double xinv[QMAX + 2];
    {
        double hs = h;
#pragma unroll
        for (int m = 2; m <= QMAX + 1; ++m) {
            hs += tau[m - 1];
            xinv[m] = h / hs;
        }
    }
    // element m of a small local array for a uniform m: a select chain over opaque copies (written
    // as a plain chain, the compiler turns it back into a dynamically indexed array in scratch
    // memory: a global-memory round trip on every cv_set)
    auto pick = [&](const double* arr, int lo, int hi, int m) {
        double v = arr[lo];
#pragma unroll
        for (int i = lo + 1; i <= QMAX + 1; ++i) {
            if (i <= hi) {
                double x = arr[i];
                asm volatile("" : "+v"(x));
                v = (m == i) ? x : v;
            }
        }
        return v;
    };
    auto xinv_at = [&](int m) { return pick(xinv, 2, QMAX + 1, m); };   // uniform m in [2, QMAX + 1]
    double xi_inv = 1.0, xistar_inv = 1.0, alpha0 = -1.0, alpha0_hat = -1.0;
    if (q > 1) {
#pragma unroll
        for (int j = 2; j < QMAX; ++j) {
            if (j < q) {
                alpha0 -= inv_int(j);
#pragma unroll
                for (int i = QMAX; i >= 1; --i) if (i <= j) lv[i] += lv[i - 1] * xinv[j];
            }
        }
        alpha0 -= inv_int(q);
        xistar_inv = -lv[1] - alpha0;
        xi_inv = xinv_at(q);
        alpha0_hat = -lv[1] - xi_inv;
#pragma unroll
        for (int i = QMAX; i >= 1; --i) if (i <= q) lv[i] += lv[i - 1] * xistar_inv;
    }
#pragma unroll
    for (int i = 0; i <= QMAX; ++i) C->l[i] = lv[i];
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = 1.0 + q * A1;
    const double lq = pick(lv, 1, QMAX, q);
    const double tq2 = fabs(A1 / (alpha0 * A2));
    C->tq[2] = tq2;
    C->tq[5] = fabs(A2 * xistar_inv / (lq * xi_inv));
    if (qwait == 1) {
        if (q > 1) {
            const double Cc = xistar_inv / lq;
            const double A3 = alpha0 + inv_int(q);
            const double A4 = alpha0_hat + xi_inv;
            const double Cpinv = (1.0 - A4 + A3) / A3;
            C->tq[1] = fabs(Cc * Cpinv);
        } else C->tq[1] = 1.0;
        xi_inv = xinv_at(q + 1);   // h / (h + tau[1] + ... + tau[q])
        const double A5 = alpha0 - inv_int(q + 1);
        const double A6 = alpha0_hat - xi_inv;
        const double Cppinv = (1.0 - A6 + A5) / A2;
        C->tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
    }
    tq4_out = CORTES / tq2;
    C->tq[4] = tq4_out;
    const double rl1 = 1.0 / lv[1];
    C->rl1 = rl1;
    const double gamma = h * rl1;
    C->gamma = gamma;
    if (nst == 0) C->gammap = gamma;
    gamrat_out = (nst > 0) ? gamma / in.gammap : 1.0;
    C->gamrat = gamrat_out;
}

// cvSet in every engine (cv_set_lp): cv_set's operations, with the independent divisions spread over
// the lanes of each 16-lane DPP row -- lane t computes one quotient and a row broadcast
// (row_newbcast) hands it to the row (a 16-lane group is one row; in 32- and 64-lane groups every
// row computes the same quotients), 3 division sequences instead of 14 -- and the order masks of the
// l recurrences folded into zero coefficients (exact: every l_i is >= 0 and finite, so
// l_i + l_{i-1} * 0 = l_i). cv_set was 19 % of C2's VALU instructions and 7.1 % of GRI's
// (profiles/r06_quad_valu_split.json). On the same inputs it returns cv_set's bits
// (scripts/micro/cvset_check.hip, 8192 random states), and the wavefront engine's trajectories are
// bit-identical to the cv_set build (GRI, surface-only, gas + surface); inside k_group the compiler
// fuses multiplies and adds of the surrounding code differently, so C2 trajectories move by
// rounding (< 0.5 band against the cv_set build, parity windows unchanged).
template <int K>
__device__ __forceinline__ double row_lane(double v) { return dppd<0x150 + K>(v); }
__device__ __forceinline__ double sel6(int t, double v0, double v1, double v2, double v3, double v4, double v5) {
    // lane t's operand (opaque copies: a select chain, not a private array in scratch memory)
    double v = v0;
    const double c[5] = {v1, v2, v3, v4, v5};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        double x = c[i];
        asm volatile("" : "+v"(x));
        v = (t == i + 1) ? x : v;
    }
    return v;
}
__device__ __forceinline__ void cv_set_lp(LCtl* C, const AttemptIn& in, double& tq4_out, double& gamrat_out) {
    const int t = (int)(threadIdx.x & 15);
    const int q = in.q, qwait = in.qwait, nst = in.nst;
    const double h = in.h;
    // h / hsum_m, hsum_m = h + tau[1] + ... + tau[m-1] in CVODE's order, m = 2 .. QMAX + 1: lane m - 2
    double hsum[QMAX + 2];
    {
        double hs = h;
#pragma unroll
        for (int m = 2; m <= QMAX + 1; ++m) {
            hs += in.tau[m - 1];
            hsum[m] = hs;
        }
    }
    const double xq = h / sel6(t, hsum[2], hsum[3], hsum[4], hsum[5], hsum[6], hsum[6]);
    double xinv[QMAX + 2];
    xinv[0] = xinv[1] = 0.0;
    xinv[2] = row_lane<0>(xq); xinv[3] = row_lane<1>(xq); xinv[4] = row_lane<2>(xq);
    xinv[5] = row_lane<3>(xq); xinv[6] = row_lane<4>(xq);
    auto pick = [&](const double* arr, int lo, int hi, int m) {
        double v = arr[lo];
#pragma unroll
        for (int i = lo + 1; i <= QMAX + 1; ++i) {
            if (i <= hi) {
                double x = arr[i];
                asm volatile("" : "+v"(x));
                v = (m == i) ? x : v;
            }
        }
        return v;
    };
    double lv[QMAX + 1] = {1.0, 1.0, 0.0, 0.0, 0.0, 0.0};
    double xi_inv = 1.0, xistar_inv = 1.0, alpha0 = -1.0, alpha0_hat = -1.0;
    if (q > 1) {
#pragma unroll
        for (int j = 2; j < QMAX; ++j) {
            const bool on = j < q;
            const double c = on ? xinv[j] : 0.0;
            alpha0 -= on ? inv_int(j) : 0.0;
#pragma unroll
            for (int i = QMAX; i >= 1; --i) if (i <= j) lv[i] += lv[i - 1] * c;
        }
        alpha0 -= inv_int(q);
        xistar_inv = -lv[1] - alpha0;
        xi_inv = pick(xinv, 2, QMAX + 1, q);
        alpha0_hat = -lv[1] - xi_inv;
        // no order mask: l_i = 0 for i >= q here, and the descending sweep reads each l_{i-1} before
        // updating it, so every l_i with i > q stays 0 (0 + 0 * xistar_inv)
#pragma unroll
        for (int i = QMAX; i >= 1; --i) lv[i] += lv[i - 1] * xistar_inv;
    }
#pragma unroll
    for (int i = 0; i <= QMAX; ++i) C->l[i] = lv[i];
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = 1.0 + q * A1;
    const double lq = pick(lv, 1, QMAX, q);
    // round 1, lane t: 0 tq2, 1 tq5, 2 1/l_1, 3 Cc, 4 Cpinv, 5 Cppinv (3..5 used when qwait == 1)
    const double A3 = alpha0 + inv_int(q);
    const double A4 = alpha0_hat + xi_inv;
    const double xi1 = pick(xinv, 2, QMAX + 1, q + 1);   // h / (h + tau[1] + ... + tau[q])
    const double A5 = alpha0 - inv_int(q + 1);
    const double A6 = alpha0_hat - xi1;
    const double num = sel6(t, A1, A2 * xistar_inv, 1.0, xistar_inv, 1.0 - A4 + A3, 1.0 - A6 + A5);
    const double den = sel6(t, alpha0 * A2, lq * xi_inv, lv[1], lq, A3, A2);
    const double r1 = num / den;
    const double tq2 = fabs(row_lane<0>(r1));
    const double rl1 = row_lane<2>(r1);
    const double Cc = row_lane<3>(r1), Cpinv = row_lane<4>(r1), Cppinv = row_lane<5>(r1);
    C->tq[2] = tq2;
    C->tq[5] = fabs(row_lane<1>(r1));
    C->rl1 = rl1;
    const double gamma = h * rl1;
    C->gamma = gamma;
    if (nst == 0) C->gammap = gamma;
    // round 2, lane t: 0 tq4, 1 tq3's quotient, 2 gamrat
    const double r2 = sel6(t, CORTES, Cppinv, gamma, 1.0, 1.0, 1.0) /
                      sel6(t, tq2, xi1 * (q + 2) * A5, in.gammap, 1.0, 1.0, 1.0);
    tq4_out = row_lane<0>(r2);
    C->tq[4] = tq4_out;
    if (qwait == 1) {
        C->tq[1] = (q > 1) ? fabs(Cc * Cpinv) : 1.0;
        C->tq[3] = fabs(row_lane<1>(r2));
    }
    gamrat_out = (nst > 0) ? row_lane<2>(r2) : 1.0;
    C->gamrat = gamrat_out;
}

// Nordsieck rescale of z[1..q] by eta^j; h = hscale*eta
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void cv_rescale(LCtl* C, VA<CPL, GW, VS>& V, int lane) {
    const int q = gui<GW>(C->q);
    const double eta = ud(C->eta), hscale = ud(C->hscale);
    double f = eta;
#pragma unroll
    for (int j = 1; j <= QMAX; ++j) {
        if (j <= q) {
#pragma unroll
            FOR_S V.at(j, s) *= f;
            f *= eta;
        }
    }
    const double h = hscale * eta;
    C->h = h; C->hscale = h;
}
// prediction (tn += h, Pascal triangle on z) and its inverse
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void cv_predict(LCtl* C, VA<CPL, GW, VS>& V, int lane, const AttemptIn& in) {
    const int q = in.q;
    double tn = in.tn + in.h;
    const double tstop = in.tstop;
    if ((tn - tstop) * in.h > 0) tn = tstop;
    C->tn = tn;
#pragma unroll
    FOR_S {
        double z[QMAX + 1];
#pragma unroll
        for (int j = 0; j <= QMAX; ++j) z[j] = V.at(j, s);
#pragma unroll
        for (int k = 1; k <= QMAX; ++k)
#pragma unroll
            for (int j = QMAX; j >= k; --j)
                if (j <= q && k <= q) z[j - 1] += z[j];
#pragma unroll
        for (int j = 0; j < QMAX; ++j) V.at(j, s) = z[j];
    }
}
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void cv_restore(LCtl* C, VA<CPL, GW, VS>& V, int lane) {
    const int q = gui<GW>(C->q);
    C->tn = ud(C->saved_t);
#pragma unroll
    FOR_S {
        double z[QMAX + 1];
#pragma unroll
        for (int j = 0; j <= QMAX; ++j) z[j] = V.at(j, s);
#pragma unroll
        for (int k = 1; k <= QMAX; ++k)
#pragma unroll
            for (int j = QMAX; j >= k; --j)
                if (j <= q && k <= q) z[j - 1] -= z[j];
#pragma unroll
        for (int j = 0; j < QMAX; ++j) V.at(j, s) = z[j];
    }
}
// cvAdjustOrder for BDF (zn[L] from zn[qmax] = indx_acor on increase)
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void cv_adjust_order(LCtl* C, VA<CPL, GW, VS>& V, int lane, int dq) {
    const int q = gui<GW>(C->q);
    if (q == 2 && dq != 1) return;
    double lv[QMAX + 1] = {0.0, 0.0, 1.0, 0.0, 0.0, 0.0};
    const double hscale = ud(C->hscale);
    if (dq == 1) {
        double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = hscale;
        for (int j = 1; j < q; ++j) {
            hsum += ud(C->tau[j + 1]);
            const double xi = hsum / hscale;
            prod *= xi;
            alpha0 -= inv_int(j + 1);
            alpha1 += 1.0 / xi;
#pragma unroll
            for (int i = QMAX; i >= 2; --i) if (i <= j + 2) lv[i] = lv[i] * xiold + lv[i - 1];
            xiold = xi;
        }
        const double A1 = (-alpha0 - alpha1) / prod;
#pragma unroll
        FOR_S {
            const double zL = A1 * V.at(QMAX, s);
#pragma unroll
            for (int j = 2; j <= QMAX; ++j) if (j <= q) V.at(j, s) += lv[j] * zL;
            vset<CPL>(V, q + 1, s, zL);
        }
    } else {
        double hsum = 0.0;
        for (int j = 1; j <= q - 2; ++j) {
            hsum += ud(C->tau[j]);
            const double xi = hsum / hscale;
#pragma unroll
            for (int i = QMAX; i >= 2; --i) if (i <= j + 2) lv[i] = lv[i] * xi + lv[i - 1];
        }
#pragma unroll
        FOR_S {
            const double zq = vget<CPL>(V, q, s);
#pragma unroll
            for (int j = 2; j < QMAX; ++j) if (j < q) V.at(j, s) -= lv[j] * zq;
        }
    }
}
// trace row of an accepted step (save_data, src/BatchReactor.jl:383-402): t, h, q, the pressure
// of the last RHS evaluation, the accepted state u_n, the state y of the last RHS evaluation
template <int CPL, int GW = 64>
__device__ __forceinline__ void trace_row(LCtl* C, const CtlArgs& a, int lane, int step, double t,
                                          const double (&v)[CPL], const double (&y)[CPL]) {
    if (a.trace && step <= a.trace_cap) {
        auto row = a.trace + ((size_t)a.rid * (a.trace_cap + 1) + step) * (2 * a.n + 4);
        if (lane == 0) { row[0] = t; row[1] = ud(C->h); row[2] = (double)gui<GW>(C->q); row[3] = ud(C->p_last); }
#pragma unroll
        FOR_S if (CS < a.n) { row[4 + CS] = v[s]; row[4 + a.n + CS] = y[s]; }
    }
}
// one attempt of cvStep: predict, coefficients, and the Newton iteration's setup decision
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void begin_attempt(LCtl* C, VA<CPL, GW, VS>& V, int lane, int nflag) {
    const AttemptIn in = load_attempt<GW>(C);
    cv_predict<CPL, GW>(C, V, lane, in);
    double tq4, gamrat;
    cv_set_lp(C, in, tq4, gamrat);   // (cv_set: the plain form it is checked against)
    BR_XC_AFTER_CVSET();
    const int nst = in.nst;
    C->convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? NO_FAILURES : FAIL_OTHER;
    C->callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (nst == 0) ||
                   (nst >= in.nstlp + MSBP) || (fabs(gamrat - 1.0) > DGMAX);
#pragma unroll
    FOR_S V.at(V_ACOR, s) = 0.0;
    C->tol = tq4;
    C->jbad = 0;
    C->jcur_nls = 0;
    C->m_it = 0;
#pragma unroll
    FOR_S V.at(V_Y, s) = V.at(0, s);   // y = z0
}
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void begin_step(LCtl* C, VA<CPL, GW, VS>& V, int lane, const CtlArgs& a) {
    BR_SUB_T(bt0);
    BR_QMARK(begin_step);
    const double tn = ud(C->tn), hprime = ud(C->hprime), h = ud(C->h);   // read before the V stores
    const int nst = gui<GW>(C->nst), qp = gui<GW>(C->qprime), q = gui<GW>(C->q);
#pragma unroll
    FOR_S {
        const double z0 = V.at(0, s);
        V.at(V_EWT, s) = (CS < a.n) ? 1.0 / (a.rtol * fabs(z0) + a.atol) : 1.0;
    }
    C->saved_t = tn;
    C->ncf = 0; C->nef = 0;
    if ((nst > 0) && (hprime != h)) {
        if (qp != q) {
            cv_adjust_order<CPL, GW>(C, V, lane, qp - q);
            C->q = qp; C->L = qp + 1; C->qwait = qp + 1;
        }
        cv_rescale<CPL, GW>(C, V, lane);
    }
    BR_QMARK(begin_step_attempt);
    begin_attempt<CPL, GW>(C, V, lane, FIRST_CALL);
    BR_QMARK(begin_step_end);
    BR_SUB_ADD(7, bt0);
}

// Controller, part 1: after the RHS value f = F(y) of this lane is known.
// Returns A_RHS (next y in V[V_Y]), A_SOLVE (delta for the solve returned in *rhs_out),
// A_SETUP (Jacobian decision in C->newj, then LU and solve), A_DONE.
template <int CPL, int GW = 64, int VS = GW>
__device__ BR_CTL_INLINE int ctl_post_rhs(LCtl* C, VA<CPL, GW, VS>& V, int lane, const double (&f)[CPL], double (&rhs_out)[CPL]) {
    const CtlArgs a = load_args<GW>(C);
    const int n = a.n;
    C->nfe = gui<GW>(C->nfe) + 1;
    const int phase = gui<GW>(C->phase);
    double z0[CPL];
#pragma unroll
    FOR_S z0[s] = V.at(0, s);
    if (phase == PH_NEWTON) {
        const double rl1 = ud(C->rl1), gamma = ud(C->gamma);
#pragma unroll
        FOR_S {
            const double acor = V.at(V_ACOR, s);
            const double delta = (rl1 * V.at(1, s) + acor) - gamma * f[s];   // cvNlsResidual
            rhs_out[s] = -delta;
        }
        if (gui<GW>(C->m_it) == 0 && gui<GW>(C->callSetup)) {          // cvLsSetup decision
            const int nst = gui<GW>(C->nst);
            const double dgamma = fabs(ud(C->gamma) / ud(C->gammap) - 1.0);
            const int cf = gui<GW>(C->jbad) ? FAIL_BAD_J : gui<GW>(C->convfail);
            const int newj = (nst == 0) || (nst > gui<GW>(C->nstlj) + LS_MSBJ) || ((cf == FAIL_BAD_J) && (dgamma < LS_DGMAX)) ||
                             (cf == FAIL_OTHER);
            C->newj = newj;
            if (newj) { C->nje = gui<GW>(C->nje) + 1; C->nstlj = nst; }
            C->nsetups = gui<GW>(C->nsetups) + 1;
            C->jcur_nls = newj;
            C->gamrat = 1.0; C->gammap = ud(C->gamma); C->crate = 1.0; C->nstlp = nst;
            return A_SETUP;
        }
        return A_SOLVE;
    }
    double h = 0.0;
    if (phase == PH_EF1) {   // restart at order 1 after repeated error-test failures
        const double hh = ud(C->h);
#pragma unroll
        FOR_S V.at(1, s) = hh * f[s];
        begin_attempt<CPL, GW>(C, V, lane, PREV_ERR_FAIL);
        C->phase = PH_NEWTON;
        return A_RHS;
    }
    double z1in[CPL], ewt[CPL];
#pragma unroll
    FOR_S {
        z1in[s] = (phase == PH_F0) ? f[s] : V.at(1, s);
        ewt[s] = V.at(V_EWT, s);
    }
    if (phase == PH_F0) {
        const double tn = ud(C->tn), tstop = ud(C->tstop);
        const double tdist = fabs(tstop - tn);
        const double tround = UROUND * fmax(fabs(tn), fabs(tstop));
        const double hlb = HLB_FACTOR * tround;
        double ratio = 0.0;
#pragma unroll
        FOR_S {
            V.at(1, s) = f[s];
            if (CS < n) ratio = fmax(ratio, fabs(f[s]) / (HUB_FACTOR * fabs(z0[s]) + 1.0 / ewt[s]));
        }
        const double hub_inv = guni<GW>(gmax<GW>(ratio));
        double hub = HUB_FACTOR * tdist;
        if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
        const double hg = sqrt(hlb * hub);
        C->hlb = hlb; C->hub = hub; C->hg = hg;
        if (hub < hlb) {
            h = hg;
        } else {
            C->count1 = 1; C->hnewOK = 0; C->hnew = hg;
#pragma unroll
            FOR_S V.at(V_Y, s) = hg * f[s] + z0[s];
            C->phase = PH_HIN;
            return A_RHS;
        }
    } else {                 // PH_HIN (cvYddNorm + the cvHin iteration)
        double hg = ud(C->hg);
        const double hub = ud(C->hub), hlb = ud(C->hlb);
        double tempv[CPL];
#pragma unroll
        FOR_S tempv[s] = (f[s] - z1in[s]) * (1.0 / hg);
        const double yddnrm = wrms_l<CPL, GW>(tempv, ewt, lane, n);
        const int count1 = gui<GW>(C->count1);
        double hnew;
        if (gui<GW>(C->hnewOK) || count1 == MAX_ITERS) {
            hnew = hg;
        } else {
            hnew = (yddnrm * hub * hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * hub);
            const double hrat = hnew / hg;
            int ok = 0;
            if ((hrat > 0.5) && (hrat < 2.0)) ok = 1;
            if ((count1 > 1) && (hrat > 2.0)) { hnew = hg; ok = 1; }
            C->hnewOK = ok;
            hg = hnew;
            C->hg = hg;
            C->count1 = count1 + 1;
#pragma unroll
            FOR_S V.at(V_Y, s) = hg * z1in[s] + z0[s];
            return A_RHS;
        }
        double h0 = H_BIAS * hnew;
        if (h0 < hlb) h0 = hlb;
        if (h0 > hub) h0 = hub;
        h = h0;
    }
    // ---- first step size known
    if (a.hmax_inv > 0) { const double rh = fabs(h) * a.hmax_inv; if (rh > 1.0) h /= rh; }
    const double tn = ud(C->tn), tstop = ud(C->tstop);
    if ((tn + h - tstop) * h > 0.0) h = (tstop - tn) * (1.0 - 4.0 * UROUND);
    C->h = h; C->hscale = h; C->hprime = h;
    trace_row<CPL, GW>(C, a, lane, 0, 0.0, z0, z0);
#pragma unroll
    FOR_S V.at(1, s) *= h;
    if (a.max_steps <= 0) { C->status = BR_ERR_MAXSTEPS; return A_DONE; }
    begin_step<CPL, GW>(C, V, lane, a);
    C->phase = PH_NEWTON;
    return A_RHS;
}

// x^(1/L) for the step-size ratios (L = order + 1 <= 6): hardware fp32 log2/exp2 estimate and
// two fp64 Newton steps (within a few ulp of pow(x, 1.0/L), which CVODE uses; ~40 instructions
// instead of ~280 for the generic pow); outside [1e-30, 1e30] the generic pow
__device__ __forceinline__ double root_int(double x, int L) {
    if (L == 1) return x;
    if (L == 2) return sqrt(x);
    if (!(x >= 1e-30 && x <= 1e30)) return pow(x, 1.0 / L);
    double y = (double)__builtin_amdgcn_exp2f(__builtin_amdgcn_logf((float)x) / (float)L);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        double p = y;                                  // y^(L-1)
        for (int k = 2; k < L; ++k) p *= y;
        y -= (p * y - x) / (L * p);
    }
    return y;
}
// x^L for the small integer L of cvPrepareNextStep (repeated products; pow in CVODE)
__device__ __forceinline__ double pow_int(double x, int L) {
    double p = x;
    for (int k = 1; k < L; ++k) p *= x;
    return p;
}

// Controller, part 2: after the linear solve (delta = this lane's Newton correction) or after
// an LU failure (lu_fail != 0). Runs the convergence test, the error test, cvCompleteStep,
// cvPrepareNextStep and the tstop logic; returns A_RHS (next y in V[V_Y]) or A_DONE.
template <int CPL, int GW = 64, int VS = GW>
__device__ BR_CTL_INLINE int ctl_post_solve(LCtl* C, VA<CPL, GW, VS>& V, int lane, double (&delta)[CPL], int lu_fail) {
    BR_SUB_T(ps0);
    BR_QMARK(ps_start);
    const CtlArgs a = load_args<GW>(C);
    const int n = a.n;
    double ewt[CPL], acor[CPL];
#pragma unroll
    FOR_S ewt[s] = V.at(V_EWT, s);
    int nls;                                                   // 0 converged, else failure
    double acnrm = 0.0;
    const double tq2_e = ud(C->tq[2]);
    if (lu_fail) {
        nls = 2;
    } else {
        C->nni = gui<GW>(C->nni) + 1;
        const double gamrat = ud(C->gamrat);
        const int m = gui<GW>(C->m_it);                            // read before the V stores
        double crate = ud(C->crate);
        const double delp = ud(C->delp), tol = ud(C->tol);
#pragma unroll
        FOR_S {
            if (gamrat != 1.0) delta[s] *= 2.0 / (1.0 + gamrat);
            acor[s] = V.at(V_ACOR, s) + delta[s];
            V.at(V_ACOR, s) = acor[s];
        }
        const double del = wrms_l<CPL, GW>(delta, ewt, lane, n);     // cvNlsConvTest
        if (m > 0) { crate = fmax(CRDOWN * crate, del / delp); C->crate = crate; }
        const double dcon = del * fmin(1.0, crate) / tol;
        if (dcon <= 1.0) {
            acnrm = (m == 0) ? del : wrms_l<CPL, GW>(acor, ewt, lane, n);
            C->acnrm = acnrm;
            nls = 0;
        } else {
            bool fail = (m >= 1) && (del > RDIV * delp);
            if (!fail) {
                C->delp = del;
                C->m_it = m + 1;
                if (m + 1 >= NLS_MAXCOR) fail = true;
            }
            if (!fail) {
#pragma unroll
                FOR_S V.at(V_Y, s) = V.at(0, s) + acor[s];
                return A_RHS;
            }
            if (!gui<GW>(C->jcur_nls)) {                          // retry with a fresh Jacobian
                C->callSetup = 1; C->jbad = 1; C->m_it = 0;
#pragma unroll
                FOR_S {
                    V.at(V_ACOR, s) = 0.0;
                    V.at(V_Y, s) = V.at(0, s);
                }
                return A_RHS;
            }
            nls = 1;
        }
    }
    BR_QMARK(ps_nflag);
    if (nls != 0) {                                          // cvHandleNFlag
        C->ncfn = gui<GW>(C->ncfn) + 1;
        cv_restore<CPL, GW>(C, V, lane);
        const int ncf = gui<GW>(C->ncf) + 1;
        C->ncf = ncf;
        C->etamax = 1.0;
        if (ncf == MXNCF) { C->status = BR_ERR_CONV; return A_DONE; }
        C->eta = ETACF;
        cv_rescale<CPL, GW>(C, V, lane);
        begin_attempt<CPL, GW>(C, V, lane, PREV_CONV_FAIL);
        return A_RHS;
    }
    // ---- cvDoErrorTest
    BR_QMARK(ps_errtest);
    const double dsm = acnrm * tq2_e;
    const int q = gui<GW>(C->q);
    if (dsm > 1.0) {
        const int nef = gui<GW>(C->nef) + 1;
        C->nef = nef; C->netf = gui<GW>(C->netf) + 1;
        cv_restore<CPL, GW>(C, V, lane);
        if (nef == MXNEF) { C->status = BR_ERR_ERRTEST; return A_DONE; }
        C->etamax = 1.0;
        if (nef <= MXNEF1) {
            double eta = 1.0 / (root_int(BIAS2 * dsm, gui<GW>(C->L)) + ADDON);
            eta = fmax(ETAMIN, eta);
            if (nef >= SMALL_NEF) eta = fmin(eta, ETAMXF);
            C->eta = eta;
            cv_rescale<CPL, GW>(C, V, lane);
            begin_attempt<CPL, GW>(C, V, lane, PREV_ERR_FAIL);
            return A_RHS;
        }
        if (q > 1) {
            C->eta = ETAMIN;
            cv_adjust_order<CPL, GW>(C, V, lane, -1);
            C->L = q; C->q = q - 1; C->qwait = q;
            cv_rescale<CPL, GW>(C, V, lane);
            begin_attempt<CPL, GW>(C, V, lane, PREV_ERR_FAIL);
            return A_RHS;
        }
        C->eta = ETAMIN;
        const double h = ud(C->h) * ETAMIN;
        C->h = h; C->hscale = h; C->qwait = LONG_WAIT;
#pragma unroll
        FOR_S V.at(V_Y, s) = V.at(0, s);
        C->phase = PH_EF1;
        return A_RHS;
    }
    // ---- cvCompleteStep
    BR_SUB_ADD(8, ps0);
    BR_QMARK(ps_complete);
    BR_SUB_T(ps1);
    // every controller scalar this part reads, loaded in one batch before the first Nordsieck store
    // (V shares LDS with the controller, so a load placed after a V store cannot be hoisted above
    // it: read in place, each one was its own LDS round trip)
    const int nst = gui<GW>(C->nst) + 1;
    const double h = ud(C->h);
    double tauv[QMAX + 1], lv[QMAX + 1];
#pragma unroll
    for (int i = 1; i <= QMAX; ++i) tauv[i] = ud(C->tau[i]);
#pragma unroll
    for (int j = 0; j <= QMAX; ++j) lv[j] = ud(C->l[j]);
    int qwait = gui<GW>(C->qwait) - 1;
    const double etamax = ud(C->etamax), tq1 = ud(C->tq[1]), tq2 = ud(C->tq[2]), tq3 = ud(C->tq[3]);
    const double tq5 = ud(C->tq[5]);
    double saved_tq5 = ud(C->saved_tq5);
    const int L = gui<GW>(C->L);
    const int nstloc = gui<GW>(C->nstloc) + 1;
    const double tn = ud(C->tn), tstop = ud(C->tstop), ulimit = ud(C->ulimit);
    C->nst = nst;
    double tau2 = tauv[2];   // tau[2] after the shift
#pragma unroll
    for (int i = QMAX; i >= 2; --i) if (i <= q) C->tau[i] = tauv[i - 1];
    if (q >= 2 || nst > 1) tau2 = tauv[1];
    if ((q == 1) && (nst > 1)) C->tau[2] = tauv[1];
    C->tau[1] = h;
#pragma unroll
    FOR_S acor[s] = V.at(V_ACOR, s);
#pragma unroll
    for (int j = 0; j <= QMAX; ++j) {
        if (j <= q) {
#pragma unroll
            FOR_S V.at(j, s) += lv[j] * acor[s];
        }
    }
    if ((qwait == 1) && (q != QMAX)) {
#pragma unroll
        FOR_S V.at(QMAX, s) = acor[s];
        saved_tq5 = tq5;
        C->saved_tq5 = tq5;
    }
    // ---- cvPrepareNextStep
    BR_QMARK(ps_prepare);
    double eta = 1.0, hprime = h;
    int qprime = q;
    if (etamax == 1.0) {
        qwait = qwait > 2 ? qwait : 2;
    } else {
        // the three step-size ratios (etaq, and at an order decision etaqm1 / etaqp1) in ONE root and
        // division sequence: lane 0 of each DPP row takes etaq's argument, lane 1 etaqm1's, lane 2
        // etaqp1's (root_int and the division per lane; a row broadcast returns each); C2: etaq's
        // root + division alone was 4.6 % of the kernel's VALU (profiles/r06_quad_valu_split.json)
        const int t = lane & 15;
        double xm = 1.0, xp = 1.0;     // benign arguments for lanes whose ratio is not needed
        bool hm = false, hp = false;
        if (qwait == 0) {
            if (q > 1) {
                double zq[CPL];
#pragma unroll
                FOR_S zq[s] = vget<CPL>(V, q, s);
                const double ddn = wrms_l<CPL, GW>(zq, ewt, lane, n) * tq1;
                xm = BIAS1 * ddn;
                hm = true;
            }
            if (q != QMAX && saved_tq5 != 0.0) {
                const double cquot = (tq5 / saved_tq5) * pow_int(h / tau2, L);
                double tempv[CPL];
#pragma unroll
                FOR_S tempv[s] = acor[s] - cquot * V.at(QMAX, s);
                const double dup = wrms_l<CPL, GW>(tempv, ewt, lane, n) * tq3;
                xp = BIAS3 * dup;
                hp = true;
            }
        }
        const double xa = t == 1 ? xm : (t == 2 ? xp : BIAS2 * dsm);
        const int La = t == 1 ? (hm ? q : L) : (t == 2 ? (hp ? L + 1 : L) : L);
        const double er = 1.0 / (root_int(xa, La) + ADDON);
        const double etaq = row_lane<0>(er);
        BR_XC_AFTER_ETAQ();
        if (qwait != 0) { eta = etaq; }
        else {
            qwait = 2;
            const double etaqm1 = hm ? row_lane<1>(er) : 0.0;
            const double etaqp1 = hp ? row_lane<2>(er) : 0.0;
            const double etam = fmax(etaqm1, fmax(etaq, etaqp1));
            if (etam < THRESH) { eta = 1.0; }
            else if (etam == etaq) { eta = etaq; }
            else if (etam == etaqm1) { eta = etaqm1; qprime = q - 1; }
            else {
                eta = etaqp1; qprime = q + 1;
#pragma unroll
                FOR_S V.at(QMAX, s) = acor[s];
            }
        }
        if (eta < THRESH) { eta = 1.0; hprime = h; }                // cvSetEta
        else {
            eta = fmin(eta, etamax);
            if (a.hmax_inv > 0) eta /= fmax(1.0, fabs(h) * a.hmax_inv * eta);   // (/ 1.0 otherwise)
            hprime = h * eta;
        }
    }
    C->qwait = qwait;
    C->etamax = (nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
#pragma unroll
    FOR_S V.at(V_ACOR, s) = acor[s] * tq2;
    C->nstloc = nstloc;
    double z0[CPL];
#pragma unroll
    FOR_S z0[s] = V.at(0, s);
    C->eta = eta; C->hprime = hprime; C->qprime = qprime;
    BR_SUB_ADD(9, ps1);
    BR_QMARK(ps_unstable);
    BR_SUB_T(ps2);
    {   // SciML unstable_check: NaN state (ulimit = inf), or opt-in runaway (br_opts.unstable_factor);
        // first, as in the oracle: an unstable step writes no trace row and no dense output
        double zm = 0.0;
#pragma unroll
        FOR_S if (CS < n) { const double a = fabs(z0[s]); zm = fmax(zm, a == a ? a : INFINITY); }
        const double mx = guni<GW>(gmax<GW>(zm));
        if (!(mx < INFINITY) || mx > ulimit) { C->status = BR_ERR_UNSTABLE; return A_DONE; }
    }
    if (a.trace) {
        double yl[CPL];
#pragma unroll
        FOR_S yl[s] = V.at(V_Y, s);                     // the last RHS was evaluated at y
        trace_row<CPL, GW>(C, a, lane, nst, tn, z0, yl);
    }
    BR_QMARK(ps_ignition);
    if (a.ign >= 0) track_ignition<CPL, GW>(C, a, lane, tn, z0);
    BR_QMARK(ps_dense);
    if (a.nout) dense_output<CPL, GW>(C, V, a, lane, tn, h, q, tn);
    // CVode ONE_STEP + tstop handling
    BR_QMARK(ps_tstop);
    const double troundoff = FUZZ * UROUND * (fabs(tn) + fabs(h));
    if (fabs(tn - tstop) <= troundoff) {                     // CVodeGetDky(tstop, 0)
        if (a.nout) dense_output<CPL, GW>(C, V, a, lane, tn, h, q, tstop);
        const double sk = (tstop - tn) / h;
#pragma unroll
        FOR_S {
            double yv = vget<CPL>(V, q, s);
#pragma unroll
            for (int j = QMAX - 1; j >= 0; --j) if (j < q) yv = V.at(j, s) + sk * yv;
            V.at(V_Y, s) = yv;
            if (a.trace && nst <= a.trace_cap) {
                auto row = a.trace + ((size_t)a.rid * (a.trace_cap + 1) + nst) * (2 * n + 4);
                if (lane == 0 && s == 0) row[0] = tstop;
                if (CS < n) row[4 + CS] = yv;
            }
        }
        return A_DONE;
    }
    if ((tn + hprime - tstop) * h > 0.0) {
        hprime = (tstop - tn) * (1.0 - 4.0 * UROUND);
        C->hprime = hprime;
        C->eta = hprime / h;
    }
    if (nstloc >= a.max_steps) { C->status = BR_ERR_MAXSTEPS; return A_DONE; }
    BR_SUB_ADD(10, ps2);
    BR_QMARK(ps_to_begin);
    begin_step<CPL, GW>(C, V, lane, a);
    BR_QMARK(ps_end);
    return A_RHS;
}

// ---- CVODE's dense difference-quotient Jacobian (cvLsDenseDQJac; CVODE_BDF()'s default, no `jac`
// is passed to ODEProblem at src/BatchReactor.jl:140,:204): at the setup point (y = z0, fy = F(y)),
// column j = (F(y + inc_j e_j) - fy) / inc_j with inc_j = max(sqrt(uround) |y_j|, minInc / ewt_j),
// minInc = 1000 |h| uround n ||fy||_WRMS (1 if that norm is 0). One RHS per column, run through the
// kernel's single RHS call site (k_integrate: the column index `dqj` routes the result here).
constexpr double DQ_SRUR = 1.4901161193847656e-08;   // sqrt(UROUND) = 2^-26
constexpr double DQ_MIN_INC_MULT = 1000.0;
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void dq_begin(LCtl* C, VA<CPL, GW, VS>& V, int lane, const double (&f)[CPL]) {
    const int n = gui<GW>(C->a_n);
    double ewt[CPL];
#pragma unroll
    FOR_S {
        ewt[s] = V.at(V_EWT, s);
        V.at(V_TEMP, s) = f[s];                      // fy, kept for the n columns
    }
    const double fnorm = wrms_l<CPL, GW>(f, ewt, lane, n);
    C->dq_mininc = (fnorm != 0.0) ? (DQ_MIN_INC_MULT * fabs(ud(C->h)) * UROUND * n * fnorm) : 1.0;
}
// increment of this lane's components (the one for component j is used by column j)
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void dq_incs(LCtl* C, VA<CPL, GW, VS>& V, int lane, double (&inc)[CPL]) {
    const double mininc = ud(C->dq_mininc);
#pragma unroll
    FOR_S inc[s] = fmax(DQ_SRUR * fabs(V.at(V_Z0, s)), mininc / V.at(V_EWT, s));
}
// column j of the saved J from F(y + inc_j e_j) = f (rows as jacobian(): JW per column)
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void dq_column(LCtl* C, VA<CPL, GW, VS>& V, int lane, int j, const double (&f)[CPL], double* Jsave) {
    constexpr int JW = CPL == 2 ? 80 : 64;
    double inc[CPL];
    dq_incs<CPL, GW>(C, V, lane, inc);
    const double ij = (j < 64) ? gbcast<GW>(inc[0], j) : gbcast<GW>(inc[CPL - 1], j - 64);
    const double ii = 1.0 / ij;
    BR_GLOBAL double* col = launder(Jsave) + (size_t)j * JW;
    const int n = gui<GW>(C->a_n);
    // rows >= n stored as 0 (with 32-wide vectors lanes 32..63 read lane - 32's V_TEMP, and f is 0
    // there: no consumer of Jsave has to mask them)
#pragma unroll
    FOR_S {
        const double v = CS < n ? ii * f[s] - ii * V.at(V_TEMP, s) : 0.0;
        if (s == 0) col[lane] = v;
        else if (lane < 16) col[64 + lane] = v;
    }
    C->nfe_dq = gui<GW>(C->nfe_dq) + 1;
}
// the Newton right-hand side at the setup point again (cvNlsResidual with f = fy, as ctl_post_rhs)
template <int CPL, int GW = 64, int VS = GW>
__device__ __forceinline__ void dq_newton_rhs(LCtl* C, VA<CPL, GW, VS>& V, int lane, double (&b)[CPL]) {
    const double rl1 = ud(C->rl1), gamma = ud(C->gamma);
#pragma unroll
    FOR_S b[s] = -((rl1 * V.at(1, s) + V.at(V_ACOR, s)) - gamma * V.at(V_TEMP, s));
}

#include "brhip_lane.hpp"   // one reactor per lane (small gas mechanisms)
#include "brhip_group.hpp"   // group engines: 4 / 2 reactors per wave (16- / 32-lane groups, n <= 32)

// ------------------------------------------------------------------------------------
// the integrator kernel: one reactor per 64-lane wavefront, `rpb` reactors per workgroup
// ------------------------------------------------------------------------------------
#ifndef BR_WPE
#define BR_WPE 2
#endif
// (Measured and not adopted, round 4-5; DESIGN.md section 3: the blocked LU with fp64 MFMA trailing
// updates -- GRI 88.8k / 92.0k vs 110.5k reactors/s, now in the variant library
// csrc/variants/brhip_lumf.hip -- and the 4 x 16 lane-grid LU with DPP-broadcast FMAs -- GRI -3.1 %,
// removed in round 6; it stays in the git history before that round.)
// upper bound of reactors (waves) per workgroup for the occupancy search: gas+surface (n > 64)
// needs 21 KB of LDS per reactor (+18 KB of tables), so only one workgroup of up to 6 reactors
// (tables staged once) fits a CU's 160 KB: 6 waves/CU instead of 4 with 1-reactor workgroups;
// n <= 64 keeps 256-thread workgroups (2 x 4 or 4 x 2 reactors, 8 waves/CU, VGPR-limited)
#ifndef BR_MAXRPB56
#define BR_MAXRPB56 16   // n in 33..64: one workgroup of up to 16 reactors per CU (tables staged once)
#endif
#ifndef BR_MAXRPB72
#define BR_MAXRPB72 12   // n > 64 (gas + surface): one workgroup of up to 12 reactors per CU (tables staged once)
#endif
__host__ __device__ constexpr int br_maxrpb(int nmax) {
    return nmax > 64 ? BR_MAXRPB72 : (nmax == 56 || nmax == 64) ? BR_MAXRPB56 : 4;
}
constexpr size_t LDS_PER_CU = 160 * 1024, LDS_GRANULE = 1280;   // gfx950 (granule: conservative)
#ifndef BR_WPE32
#define BR_WPE32 5   // n <= 32 (surface-only): 5 waves/SIMD (96 VGPRs, 80 B/lane spilled) -- with the 32-wide
                     // vectors (BR_VS32) five 4-reactor workgroups fit the LDS: 20 waves/CU, C4 232.8k vs
                     // 219.7k reactors/s at 16 (round 5); round 2: 3 waves/SIMD, 12 waves/CU, 130k -> 156k/s
#endif
// minimum waves per SIMD the register allocator must allow, per instance
#ifndef BR_WPE72
#define BR_WPE72 3   // n > 64: 3 waves/SIMD (168 VGPRs, 26 spilled; 11 reactors per CU by LDS: +3 % over 2 waves)
#endif
#ifndef BR_WPE56
#define BR_WPE56 4   // n in 33..64 (GRI): 4 waves/SIMD (<= 128 VGPRs; 16 x 8.8 KB + tables fit the LDS)
#endif
__host__ __device__ constexpr int br_wpe(int nmax) {
    return nmax == 32 ? BR_WPE32 : (nmax == 56 || nmax == 64) ? BR_WPE56 : nmax == 72 ? BR_WPE72 : BR_WPE;
}
template <int NMAX>
__global__ __launch_bounds__(64 * br_maxrpb(NMAX)) __attribute__((amdgpu_waves_per_eu(br_wpe(NMAX), 8))) void k_integrate(
    DevMech M, int N, int rpb, const double* __restrict__ Tv, const double* __restrict__ Asvv, double* __restrict__ U,
    const double* __restrict__ tfv, KOpts o, double* __restrict__ stats, double* __restrict__ Jws,
    double* __restrict__ trace) {
    constexpr int CPL = NMAX > 64 ? 2 : 1;   // components per lane
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx<CPL, NMAX>(M, smem_raw, rpb, Jws);
    // Reactor indices: with o.work every wave of the (resident-sized) grid keeps taking the next
    // index from the counter until the list is drained, so a wave whose reactor finishes early
    // starts another instead of idling until the slowest reactor of its workgroup is done; the
    // wave's workspace slot and LDS block are reused. Index -> reactor through rid_list when set
    // (the deferred reactors of a k_lane pass).
    const int widx = W.rid;               // workspace slot of this wave
    const int nidx = o.rid_list ? min(*o.rid_count, N) : N;
    auto next_index = [&]() -> int {
        int v = 0;
        if (W.lane == 0) v = atomicAdd(o.work, 1);
        return __builtin_amdgcn_readlane(v, 0);
    };
    for (int idx = o.work ? next_index() : widx; idx < nidx; idx = o.work ? next_index() : nidx) {
    int rid = o.rid_list ? uni(o.rid_list[idx]) : idx;
    wave_sync();
    const int lane = W.lane;
    const Tab& tb = W.tb;
    const size_t roff = (size_t)(W.rbase - smem_raw);
    LCtl* C = (LCtl*)(smem_raw + roff);
    const VA<CPL, 64, vec_stride(NMAX)> Vm{(LDbl*)(smem_raw + roff + CTL_BYTES), lane};
    VA<CPL, 64, vec_stride(NMAX)> V = Vm;
    const RView& S = W.R;
    const int n = M.n;
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    double* Jsave = Jws + (size_t)widx * ws_doubles(NMAX, M.nrg);   // J, LU factors, Jacobian scratch
    double* LUsave = Jsave + NMAX * col_rows(NMAX);
    double* jscr = LUsave;   // (aliases the factors: see rxd_ws_off)
    C->a_rtol = o.rtol; C->a_atol = o.atol; C->a_hmax_inv = o.hmax_inv; C->a_ufac = o.ufac;
    C->a_max_steps = o.max_steps; C->a_trace_cap = o.trace_cap; C->a_trace = trace; C->a_rid = rid; C->a_n = n;
    C->a_ign = o.ign; C->a_nout = o.nout; C->a_tout = o.tout; C->a_yout = o.yout;

    init_tconst<CPL>(M, tb, S, T, lane);

    // ---- CVodeInit
    double u0[CPL], su = 0.0;
#pragma unroll
    FOR_S {
        const bool act = CS < n;
        u0[s] = act ? U[(size_t)rid * n + CS] : 0.0;
#pragma unroll
        for (int j = 0; j < NVEC; ++j) V.at(j, s) = 0.0;
        V.at(0, s) = u0[s];
        V.at(V_Y, s) = u0[s];
        V.at(V_EWT, s) = act ? 1.0 / (o.rtol * fabs(u0[s]) + o.atol) : 1.0;
        su += act ? fabs(u0[s]) : 0.0;
    }
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
    const double t0 = o.rid_t0 ? uni(o.rid_t0[idx]) : 0.0;   // > 0: continue a deferred lane reactor
    C->tn = t0;
    C->ulimit = o.ufac > 0.0 ? o.ufac * uni(wave_sum(su)) : INFINITY;
    C->q = 1; C->qprime = 1; C->L = 2; C->qwait = 2;
    C->nst = 0; C->nfe = 0; C->nsetups = 0; C->nje = 0; C->nni = 0; C->ncfn = 0; C->netf = 0; C->nstlp = 0;
    C->nstlj = 0; C->ncf = 0; C->nef = 0; C->nstloc = 0; C->status = 0; C->m_it = 0; C->convfail = 0;
    C->count1 = 0; C->phase = PH_F0; C->callSetup = 0; C->jbad = 0; C->jcur_nls = 0; C->hnewOK = 0; C->newj = 0;
    C->p_last = 0.0;
    C->iout = 0; C->ign_t = t0; C->ign_rate = -INFINITY; C->t_ign = NAN; C->ign_x = 0.0; C->ign_dt = NAN;
    C->dq_mininc = 1.0; C->nfe_dq = 0;
    if (o.ign >= 0) C->ign_x = uni(mole_frac_of<CPL>(u0, lane, o.ign));
    // counters and ignition marker of the lane pass (deferred reactors) to continue from
    double st_in[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (o.rid_t0 && stats) {
#pragma unroll
        for (int k = 0; k < 7; ++k) st_in[k] = uni(stats[(size_t)rid * BR_NSTAT + k]);
        st_in[7] = uni(stats[(size_t)rid * BR_NSTAT + 19]);   // nfe_dq
        // the step limit is on the whole run (SciML maxiters): the lane pass's steps count against it
        C->a_max_steps = max(o.max_steps - (int)st_in[0], 0);
        if (o.ign >= 0) {
            C->ign_rate = uni(stats[(size_t)rid * BR_NSTAT + 17]);
            C->t_ign = uni(stats[(size_t)rid * BR_NSTAT + 16]);
            C->ign_dt = uni(stats[(size_t)rid * BR_NSTAT + 18]);
        }
    }
    if (o.nout) {                                           // outputs at t <= t0: the initial state
        int io = 0;
        while (io < o.nout && !(o.tout[io] > t0)) {
            if (!o.rid_t0)                                  // (a continued reactor wrote them already)
#pragma unroll
                FOR_S if (CS < n) o.yout[((size_t)rid * o.nout + io) * n + CS] = u0[s];
            ++io;
        }
        C->iout = io;
    }

#if BR_ASM_MARKS   // analysis builds: phase markers in the ISA listing (they are scheduling barriers)
#define BR_CLK(v) asm volatile("; BR_PHASE_BEGIN " #v)
#define BR_ACC(acc, v) asm volatile("; BR_PHASE_END " #acc)
#elif BR_PHASE_CLOCKS
    unsigned long long cyc_rhs = 0, cyc_jac = 0, cyc_lu = 0, cyc_sol = 0, cyc_ctl = 0;
    const unsigned long long clk0 = clock64();
#define BR_CLK(v) const unsigned long long v = clock64()
#define BR_ACC(acc, v) acc += clock64() - v
#else
#define BR_CLK(v)
#define BR_ACC(acc, v)
#endif
    const unsigned long long cyc0 = wall_clock64();
    int perm[CPL];
#pragma unroll
    FOR_S perm[s] = CS;
    LDSd* scr = (LDSd*)(S.sp + Lay<CPL>::ACCW);   // solve / LU scratch: the production sums are idle then
    double* p_last = reinterpret_cast<double*>(W.rbase);   // Ctl::p_last is the first field
    int dqj = -1;   // >= 0: building DQ Jacobian column dqj (this RHS is at y + inc_dqj e_dqj)
    for (;;) {
        double y[CPL], f[CPL];
#pragma unroll
        FOR_S y[s] = V.at(V_Y, s);
        if (dqj >= 0) {
            double inc[CPL];
            dq_incs<CPL>(C, V, lane, inc);
#pragma unroll
            FOR_S if (CS == dqj) y[s] += inc[s];
        }
        {
            BR_CLK(c0);
            rhs<CPL>(M, tb, S, T, Asv, Asv_th, y, lane, p_last, f);
            BR_X_AFTER_RHS();
            BR_ACC(cyc_rhs, c0);
        }
        double b[CPL];
        int act_code;
        bool jac_ready = false;
        if (dqj >= 0) {   // a DQ column (its RHS counts in nfe_dq, not nfe)
            BR_CLK(c0);
            dq_column<CPL>(C, V, lane, dqj, f, Jsave);
            BR_ACC(cyc_jac, c0);
            if (++dqj < n) continue;
            dqj = -1;
            dq_newton_rhs<CPL>(C, V, lane, b);
            act_code = A_SETUP;
            jac_ready = true;
        } else {
            BR_CLK(c2);
            BR_SUB_T(pr0);
            act_code = ctl_post_rhs<CPL>(C, V, lane, f, b);
            BR_SUB_ADD(3, pr0);
            BR_ACC(cyc_ctl, c2);
            if (act_code == A_RHS) continue;
            if (act_code == A_DONE) break;
            if (act_code == A_SETUP && o.dq_jac && ui(C->newj)) {
                dq_begin<CPL>(C, V, lane, f);
                dqj = 0;
                continue;
            }
        }
        int lu_fail = 0;
        if (act_code == A_SETUP) {
            if (!jac_ready && ui(C->newj)) {
                BR_CLK(c0);
                jacobian<CPL>(M, tb, S, T, Asv, Asv_th, y, lane, Jsave, jscr);
                BR_X_AFTER_JAC();
                BR_ACC(cyc_jac, c0);
            }
            BR_CLK(c1);
            if constexpr (CPL == 1) lu_fail = lu_factor<NMAX>(Jsave, LUsave, ud(C->gamma), n, lane, perm[0]);
            else lu_fail = lu_factor2<NMAX>(Jsave, LUsave, scr, ud(C->gamma), n, lane, perm);
            BR_ACC(cyc_lu, c1);
        }
        double delta[CPL];
#pragma unroll
        FOR_S delta[s] = 0.0;
        if (!lu_fail) {
            BR_CLK(c0);
            if constexpr (CPL == 1) {
                delta[0] = lu_solve<NMAX>(LUsave, n, lane, perm[0], b[0], scr);
                BR_X_AFTER_SOLVE();
            } else {
                lu_solve2<NMAX>(LUsave, scr, n, lane, perm, b);
                delta[0] = b[0];
                delta[1] = b[1];
            }
            BR_ACC(cyc_sol, c0);
        }
        BR_X_AFTER_ITER();
        BR_CLK(c3);
        act_code = ctl_post_solve<CPL>(C, V, lane, delta, lu_fail);
        BR_ACC(cyc_ctl, c3);
        if (act_code == A_DONE) break;
    }
    const int status = ui(C->status);
#pragma unroll
    FOR_S {
        const double u_out = status ? V.at(0, s) : V.at(V_Y, s);
        if (CS < n) U[(size_t)rid * n + CS] = u_out;
    }
    if (stats && lane == 0) {
        double* st = stats + (size_t)rid * BR_NSTAT;
        st[0] = st_in[0] + ui(C->nst); st[1] = st_in[1] + ui(C->nfe); st[2] = st_in[2] + ui(C->nje);
        st[3] = st_in[3] + ui(C->nsetups); st[4] = st_in[4] + ui(C->nni); st[5] = st_in[5] + ui(C->ncfn);
        st[6] = st_in[6] + ui(C->netf); st[7] = (double)status;
        st[8] = (double)(wall_clock64() - cyc0);
#if BR_PHASE_CLOCKS
        st[9] = (double)cyc_rhs; st[10] = (double)cyc_jac; st[11] = (double)cyc_lu; st[12] = (double)cyc_sol;
        st[14] = (double)cyc_ctl; st[15] = (double)(clock64() - clk0);
#else
        st[9] = st[10] = st[11] = st[12] = st[14] = st[15] = 0.0;
#endif
        st[13] = ud(C->tn);
        st[16] = o.ign >= 0 ? ud(C->t_ign) : NAN; st[17] = o.ign >= 0 ? ud(C->ign_rate) : NAN;
        st[18] = o.ign >= 0 ? ud(C->ign_dt) : NAN; st[19] = st_in[7] + ui(C->nfe_dq);
    }
    }   // next reactor
}

// ------------------------------------------------------------------------------------
// parity kernels: rates, rhs, jacobian (one reactor per wave)
// ------------------------------------------------------------------------------------
template <int CPL>
__global__ __launch_bounds__(256) void k_rates(DevMech M, int N, int rpb, const double* Tv, const double* pv,
                                               const double* X, const double* TH, double* W_, double* SD, double* Jws) {
    typedef Lay<CPL> L;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx<CPL, CPL == 2 ? 72 : 64>(M, smem_raw, rpb, Jws);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    const RView& S = W.R;
    const double T = Tv[rid], p = pv[rid];
    init_tconst<CPL>(M, W.tb, S, T, lane);
    double cg = 0.0;
#pragma unroll
    FOR_S {
        const int k = CS;
        double c = 0.0;
        if (k < M.ng) c = p * X[(size_t)rid * M.ng + k] / (R_GAS * T);
        else if (k < M.n) c = TH ? TH[(size_t)rid * M.ns + (k - M.ng)] : 0.0;
        if (k < M.n) { S.sp[L::CONC + k] = c; S.sp[L::ACCW + k] = 0.0; S.sp[L::ACCS + k] = 0.0; }
        cg += k < M.ng ? c : 0.0;
    }
    const double Ctot = wave_sum(cg);
    wave_sync();
    third_body_sets<CPL>(M, W.tb, S.sp, Ctot, lane);
    wave_sync();
    production<CPL>(M, W.tb, S, R_GAS * T, lane, rx_prefetch(S, lane));
    wave_sync();
#pragma unroll
    FOR_S {
        const int k = CS;
        const double w = k < M.n ? S.sp[L::ACCW + k] : 0.0;
        const double sd = k < M.n ? S.sp[L::ACCS + k] : 0.0;
        if (k < M.ng) W_[(size_t)rid * M.ng + k] = w;
        if (SD && k < M.n) SD[(size_t)rid * M.n + k] = sd;
    }
}

template <int CPL>
__global__ __launch_bounds__(256) void k_rhs(DevMech M, int N, int rpb, const double* Tv, const double* Asvv,
                                             const double* U, double* DU, double* Jws) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx<CPL, CPL == 2 ? 72 : 64>(M, smem_raw, rpb, Jws);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    const RView& S = W.R;
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst<CPL>(M, W.tb, S, T, lane);
    double u[CPL], du[CPL];
#pragma unroll
    FOR_S u[s] = CS < M.n ? U[(size_t)rid * M.n + CS] : 0.0;
    rhs<CPL>(M, W.tb, S, T, Asv, Asv_th, u, lane, reinterpret_cast<double*>(W.rbase), du);
#pragma unroll
    FOR_S if (CS < M.n) DU[(size_t)rid * M.n + CS] = du[s];
}

template <int NMAX>
__global__ __launch_bounds__(256) void k_jac(DevMech M, int N, int rpb, const double* Tv, const double* Asvv,
                                             const double* U, double* J, double* Jws) {
    constexpr int CPL = NMAX > 64 ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const WaveCtx W = wave_ctx<CPL, NMAX>(M, smem_raw, rpb, Jws);
    const int rid = W.rid;
    if (rid >= N) return;
    const int lane = W.lane;
    const RView& S = W.R;
    const double T = Tv[rid];
    const double Asv = Asvv ? Asvv[rid] : 1.0;
    const double Asv_th = (M.conv & 4) ? 1.0 : Asv;
    init_tconst<CPL>(M, W.tb, S, T, lane);
    double u[CPL];
#pragma unroll
    FOR_S u[s] = CS < M.n ? U[(size_t)rid * M.n + CS] : 0.0;
    double* Jsave = Jws + (size_t)rid * ws_doubles(NMAX, M.nrg);
    jacobian<CPL>(M, W.tb, S, T, Asv, Asv_th, u, lane, Jsave, Jsave + NMAX * col_rows(NMAX));
#pragma unroll
    FOR_S {
        if (CS < M.n) {
            double* row = J + ((size_t)rid * M.n + CS) * M.n;
            for (int j = 0; j < M.n; ++j) row[j] = Jsave[j * col_rows(NMAX) + CS];
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
// the group-engine instances (brhip_group.hpp)
static const void* grp_kernel(int gl, int nm) {
    if (gl == 16) return nm == 9 ? (const void*)k_group<16, 9> : (const void*)k_group<16, 16>;
    return nm == 24 ? (const void*)k_group<32, 24> : (const void*)k_group<32, 32>;
}

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
    // one-reactor-per-lane engine (brhip_lane.hpp): 0 = not eligible, else the register width NM
    int lane_nm = 0, lane_blocks = 0;
    size_t lane_shmem = 0;
    double* lws = nullptr;     // saved Jacobians, slot-major [NM*NM][slots]
    size_t lws_bytes = 0;
    int* queue = nullptr;      // work counter
    // group engine (brhip_group.hpp): gl = 0 not eligible, else the group width (16: quad, 32: pair)
    // and the register width NM of k_group<gl, NM>
    int grp_gl = 0, grp_nm = 0, grp_blocks = 0;
    size_t grp_shmem = 0;
    double* qws = nullptr;     // saved Jacobians, 16 x 16 per group slot
    size_t qws_bytes = 0;
    int* wq = nullptr;         // k_integrate work counter
    double* defer_t0 = nullptr; // start time of each deferred lane reactor (DEFER_CAP)
    int ncu = 0;
};

static thread_local std::string g_err;
// error message from the host mechanism compiler (mech_host.cpp, same library)
extern "C" __attribute__((visibility("hidden"))) void br_set_last_error(const char* msg) { g_err = msg; }
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

// engine selection for br_integrate* (untraced): BRHIP_ENGINE = wave | lane | quad | pair forces one
// (when the mechanism is eligible); default: the group engine for eligible mechanisms (quad, n <= 16:
// C2 H2/O2 882k reactors/s against 477k for the lane engine and 470k for the wavefront engine, round
// 4; pair, 16 < n <= 32, when BR_PAIR_DEFAULT: off, surface-only Ni/CH4 194.8k vs 217.7k for the
// wavefront engine), else the lane engine, else the wavefront engine.
// Codes: 0 wavefront, NM > 0 lane, -(100 gl + NM) group.
#ifndef BR_QUAD_DEFAULT
#define BR_QUAD_DEFAULT 1
#endif
#ifndef BR_PAIR_DEFAULT
#define BR_PAIR_DEFAULT 0
#endif
static int pick_engine(const br_mech* m) {
    const char* eng = getenv("BRHIP_ENGINE");
    if (eng && strcmp(eng, "wave") == 0) return 0;
    if (eng && strcmp(eng, "lane") == 0) return m->lane_nm;
    const int gcode = -(100 * m->grp_gl + m->grp_nm);
    if (m->grp_gl == 16 && ((eng && strcmp(eng, "quad") == 0) || (!eng && BR_QUAD_DEFAULT))) return gcode;
    if (m->grp_gl == 32 && ((eng && strcmp(eng, "pair") == 0) || (!eng && BR_PAIR_DEFAULT))) return gcode;
    return m->lane_nm;
}
int br_mech_engine(const br_mech* m) {
    if (!m) return fail(BR_ERR_INPUT, "null mechanism");
    return pick_engine(m);
}

int br_mech_launch_info(const br_mech* m, int* rpb, int* waves_per_cu, long long* lds_bytes) {
    if (!m) return fail(BR_ERR_INPUT, "null mechanism");
    // the geometry of the engine br_integrate launches (pick_engine), not always the wavefront one
    const int e = pick_engine(m);
    const int ncu = m->ncu > 0 ? m->ncu : 1;
    int r = m->rpb, w = m->waves_per_cu;
    long long l = (long long)m->shmem;
    if (e < 0) {          // group engine: BR_QWPB waves per workgroup, 64 / GL reactors per wave
        r = BR_QWPB * (64 / m->grp_gl);
        w = m->grp_blocks / ncu * BR_QWPB;
        l = (long long)m->grp_shmem;
    } else if (e > 0) {   // reactor-per-lane engine: one wave of 64 reactors per workgroup
        r = 64;
        w = m->lane_blocks / ncu;
        l = (long long)m->lane_shmem;
    }
    if (rpb) *rpb = r;
    if (waves_per_cu) *waves_per_cu = w;
    if (lds_bytes) *lds_bytes = l;
    return 0;
}

int br_mech_create(const br_mech_desc* d, int device, br_mech** out) {
    if (!d || !out) return fail(BR_ERR_INPUT, "null argument");
    const int ng = d->ng, ns = d->ns, nrg = d->nrg, nrs = d->nrs, n = ng + ns;
    if (ng <= 0 || ns < 0 || nrg < 0 || nrs < 0) return fail(BR_ERR_INPUT, "bad sizes");
    if (n > 72) return fail(BR_ERR_UNSUPPORTED, "n > 72 components is not supported by this build");
    HIPCHK(hipSetDevice(device));
    br_mech* m = new br_mech();
    m->device = device; m->ng = ng; m->ns = ns; m->nrg = nrg; m->nrs = nrs; m->n = n;
    m->nmax = n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 56 ? 56 : (n <= 64 ? 64 : 72)));
    DevMech& M = m->dm;
    M.ng = ng; M.ns = ns; M.n = n; M.nrg = nrg; M.nrs = nrs; M.conv = d->conv;
    M.cpl = n > 64 ? 2 : 1;
    const int SPW = M.cpl == 2 ? Lay<2>::SPW : Lay<1>::SPW;       // species slots
    const int SP_ONE = M.cpl == 2 ? Lay<2>::ONE : Lay<1>::ONE;    // pad species: conc = 1
    const int IMG_RX_OFF = M.cpl == 2 ? Lay<2>::IMG_RX : Lay<1>::IMG_RX;
    M.p_std = d->p_std > 0 ? d->p_std : 1e5;
    M.G = d->site_density * 1e4;
    auto pack4 = [](const int* v, int cnt, int pad = 255) {
        uint32_t w = 0;
        for (int e = 0; e < 4; ++e) w |= (uint32_t)(e < cnt ? (v[e] & 255) : pad) << (8 * e);
        return w;
    };
    // net-stoichiometry scatter list of a reaction: up to 6 (species, nu != 0) pairs packed in
    // 4 words (brhip_device.hpp sl_off / sl_nu): w0..w2 = byte offsets species * 8 of slots 0..5,
    // two 16-bit fields per word; w3 = 4-bit signed nu x 6 | count << 24
    auto sl_put = [](uint32_t* w, int t, int sp, int nu) {
        w[t >> 1] |= (uint32_t)(sp * 8) << (16 * (t & 1));
        w[3] |= (uint32_t)(nu & 15) << (4 * t);
    };
    auto scatter_pack = [&sl_put](const int* f, int nf, const int* pr, int np, uint32_t* w) -> bool {
        int sp[12], nu[12], c = 0;
        auto add = [&](int k, int v) {
            for (int i = 0; i < c; ++i) if (sp[i] == k) { nu[i] += v; return; }
            sp[c] = k; nu[c] = v; ++c;
        };
        for (int e = 0; e < nf; ++e) add(f[e], -1);
        for (int e = 0; e < np; ++e) add(pr[e], 1);
        int mm = 0;
        w[0] = w[1] = w[2] = w[3] = 0;
        for (int i = 0; i < c; ++i) {
            if (nu[i] == 0) continue;
            if (mm >= 6 || nu[i] < -8 || nu[i] > 7 || sp[i] < 0 || sp[i] > 255) return false;
            sl_put(w, mm, sp[i], nu[i]);
            ++mm;
        }
        w[3] |= (uint32_t)mm << 24;
        return true;
    };
    // ---- gas reactions, evaluated in a permuted order (falloff, then +M, then elementary) so
    //      that the lanes of one pass take the same branch; results are per species, so the
    //      order is invisible outside the kernel
    std::vector<int> perm;
    for (int pass = 2; pass >= 0; --pass)
        for (int r = 0; r < nrg; ++r) if (d->g_tb[r] == pass) perm.push_back(r);
    int ntb = 0, nfo = 0;
    for (int i = 0; i < nrg; ++i) {
        if (d->g_tb[perm[i]] == 2) nfo++;
        if (d->g_tb[perm[i]]) ntb++;
    }
    if (ntb > 1023 || nfo > 1023) { delete m; return fail(BR_ERR_UNSUPPORTED, "too many third-body reactions"); }
    std::vector<uint32_t> rx(RX_WORDS * (size_t)nrg, 0);
    std::vector<double> gpar(4 * (size_t)std::max(nrg, 1), 0.0), fopar(8 * (size_t)std::max(nfo, 1), 0.0);
    std::vector<int> gdnu(std::max(nrg, 1), 0);
    std::vector<std::pair<int, double>> tbe;       // (species, eff - 1), per set
    std::vector<std::vector<double>> sets;         // distinct efficiency rows
    std::vector<uint32_t> tbs;                     // per set: start | count << 20
    std::vector<double> tbeff;                     // dense [nset][n]
    int tbi = 0, foi = 0;
    for (int i = 0; i < nrg; ++i) {
        const int r = perm[i];
        const int nf = d->g_nf[r], nr = d->g_nr[r], tb = d->g_tb[r];
        if (nf > 4 || nr > 4 || nf < 1) { delete m; return fail(BR_ERR_UNSUPPORTED, "reaction with >4 entries"); }
        uint32_t* rec = &rx[RX_WORDS * (size_t)i];
        rec[0] = pack4(d->g_f + r * 4, nf, SP_ONE);
        rec[1] = pack4(d->g_r + r * 4, nr, SP_ONE);
        if (!scatter_pack(d->g_f + r * 4, nf, d->g_r + r * 4, nr, rec + 4)) {
            delete m; return fail(BR_ERR_UNSUPPORTED, "reaction touches more than 6 species");
        }
        for (int c = 0; c < 3; ++c) gpar[4 * (size_t)i + c] = d->g_arr[r * 3 + c];
        gpar[4 * (size_t)i + 3] = (d->conv & BR_CONV_KC_UNIT_SLIP) ? std::pow(1e6, (double)(nr - nf)) : 1.0;
        gdnu[i] = nr - nf;
        int troe = 0, fo = 0, tbidx = 0;
        if (tb) {   // third-body efficiency set (deduplicated: GRI's 41 reactions use 10 sets)
            std::vector<double> row(d->g_eff + (size_t)r * ng, d->g_eff + (size_t)r * ng + ng);
            int sidx = -1;
            for (size_t q = 0; q < sets.size(); ++q) if (sets[q] == row) { sidx = (int)q; break; }
            if (sidx < 0) {
                sidx = (int)sets.size();
                sets.push_back(row);
                const int start = (int)tbe.size();
                for (int k = 0; k < ng; ++k) if (row[k] != 1.0) tbe.push_back({k, row[k] - 1.0});
                const int cnt = (int)tbe.size() - start;
                if (start >= (1 << 20) || cnt >= (1 << 12)) { delete m; return fail(BR_ERR_UNSUPPORTED, "third-body list too long"); }
                tbs.push_back((uint32_t)start | ((uint32_t)cnt << 20));
                for (int k = 0; k < n; ++k) tbeff.push_back(k < ng ? row[k] : 0.0);
            }
            tbidx = sidx;
            tbi++;
        }
        if (tb == 2) {
            fo = foi++;
            troe = d->g_troe_n[r];
            for (int c = 0; c < 3; ++c) fopar[8 * (size_t)fo + c] = d->g_low[r * 3 + c];
            for (int c = 0; c < 4; ++c) fopar[8 * (size_t)fo + 3 + c] = d->g_troe[r * 4 + c];
            fopar[8 * (size_t)fo + 7] = troe;
        }
        rec[2] = (uint32_t)(nf | (nr << 3) | ((d->g_rev[r] ? 1 : 0) << 6) | (tb << 7) | ((troe & 7) << 9) |
                            (fo << 12) | (tbidx << 22));
    }
    M.ntb = ntb; M.nfo = nfo; M.ntbe = (int)tbe.size(); M.nset = (int)sets.size();
    M.nu4 = 0;
    for (int r = 0; r < nrg; ++r) if (d->g_nf[r] > 3 || d->g_nr[r] > 3) M.nu4 = 1;
    if (M.nset > 64) { delete m; return fail(BR_ERR_UNSUPPORTED, "more than 64 third-body efficiency sets"); }
    // ---- surface reactions
    std::vector<uint32_t> sx(SX_WORDS * (size_t)nrs, 0);
    std::vector<double> sxe(SXE_DOUBLES * (size_t)nrs, 0.0), spar(4 * (size_t)std::max(nrs, 1), 0.0);
    for (int r = 0; r < nrs; ++r) {
        const int nf = d->s_nf[r], np = d->s_np[r], nc = d->s_ncov[r];
        if (nf > 6 || np > 6 || nc > 4) { delete m; return fail(BR_ERR_UNSUPPORTED, "surface reaction too large"); }
        uint32_t* rec = &sx[SX_WORDS * (size_t)r];
        int e6[6];
        for (int e = 0; e < 6; ++e) e6[e] = e < nf ? d->s_f[r * 6 + e] : SP_ONE;
        rec[0] = pack4(e6, 4);
        rec[1] = pack4(e6 + 4, 2, SP_ONE);
        // constant site factor of the rate: Gamma/sigma per surface reactant (concentration
        // theta*Gamma/sigma), 1 for gas reactants and for sticking reactions (theta only)
        double fold = 1.0;
        for (int e = 0; e < nf; ++e) {
            const int sp = d->s_f[r * 6 + e];
            if (sp >= ng && !d->s_stick[r]) fold *= M.G / (d->sigma ? d->sigma[sp - ng] : 1.0);
        }
        sxe[SXE_DOUBLES * (size_t)r + 4] = fold;
        int p6[6];
        for (int e = 0; e < 6; ++e) p6[e] = e < np ? d->s_p[r * 6 + e] : 255;
        rec[2] = pack4(p6, 4);
        rec[3] = pack4(p6 + 4, 2);
        if (!scatter_pack(d->s_f + r * 6, nf, d->s_p + r * 6, np, rec + 6)) {
            delete m; return fail(BR_ERR_UNSUPPORTED, "surface reaction touches more than 6 species");
        }
        int cs[4] = {0, 0, 0, 0};
        for (int c = 0; c < nc; ++c) { cs[c] = d->s_cov_sp[r * 4 + c]; sxe[SXE_DOUBLES * (size_t)r + c] = d->s_cov_eps[r * 4 + c]; }
        rec[5] = pack4(cs, 4);
        int g = -1;
        for (int e = 0; e < nf; ++e) if (d->s_f[r * 6 + e] < ng) g = d->s_f[r * 6 + e];
        if (d->s_stick[r] && g < 0) { delete m; return fail(BR_ERR_INPUT, "sticking reaction without gas reactant"); }
        rec[4] = (uint32_t)(nf | (np << 3) | ((d->s_stick[r] ? 1 : 0) << 6) | (nc << 7) | ((g < 0 ? 0 : g) << 10));
        for (int c = 0; c < 3; ++c) spar[4 * (size_t)r + c] = d->s_arr[r * 3 + c];
        spar[4 * (size_t)r + 3] = g >= 0 ? d->molwt[g] : 1.0;
    }
    // ---- scatter-slot order: the production sums are accumulated with one LDS atomic instruction per
    //      list slot e over the 64 reactions of a pass (lanes), so a species that sits in the same
    //      slot of many of those reactions serialises that instruction (LDS address conflicts; GRI's
    //      H, O, OH, H2O ...). Per group of 64 reactions, each reaction's list is permuted so that its
    //      species land in the slots where they are least used so far (greedy, exhaustive over the
    //      <= 720 orders of one list). Only the order of the per-species sums changes.
    auto spread_slots = [&sl_put](std::vector<uint32_t>& recs, int words, int off, int nrec) {
        for (int g0 = 0; g0 < nrec; g0 += WAVE) {
            static thread_local int cnt[6][256];
            memset(cnt, 0, sizeof(cnt));
            for (int i = g0; i < std::min(nrec, g0 + WAVE); ++i) {
                uint32_t* w = &recs[(size_t)words * i + off];
                const int m = (int)(w[3] >> 24);
                int sp[6], nu[6], ord[6], best[6];
                for (int e = 0; e < m; ++e) {
                    sp[e] = (int)(((w[e >> 1] >> (16 * (e & 1))) & 0xffffu) >> 3);
                    nu[e] = ((int)(w[3] << (28 - 4 * e))) >> 28;
                    ord[e] = e;
                }
                long bc = -1;
                do {   // ord[slot] = entry placed in that slot
                    long c = 0;
                    for (int t = 0; t < m; ++t) { const long v = cnt[t][sp[ord[t]]] + 1; c += v * v; }
                    if (bc < 0 || c < bc) { bc = c; std::copy(ord, ord + m, best); }
                } while (std::next_permutation(ord, ord + m));
                uint32_t nw[4] = {0, 0, 0, w[3] & 0xFF000000u};
                for (int t = 0; t < m; ++t) {
                    const int e = best[t];
                    sl_put(nw, t, sp[e], nu[e]);
                    cnt[t][sp[e]]++;
                }
                for (int q = 0; q < 4; ++q) w[q] = nw[q];
            }
        }
    };
    {
        const char* ss = getenv("BRHIP_SPREAD");   // "0": lists in first-appearance order (A/B)
        if (!(ss && atoi(ss) == 0)) {
            spread_slots(rx, RX_WORDS, 4, nrg);
            spread_slots(sx, SX_WORDS, 6, nrs);
        }
    }
    // ---- Jacobian column lists: reactions whose rate depends on component j
    std::vector<int> colptr(1, 0), colrx;
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < nrg; ++i) {
            const int r = perm[i];
            bool dep = false;
            for (int e = 0; e < d->g_nf[r]; ++e) dep |= d->g_f[r * 4 + e] == j;
            for (int e = 0; e < d->g_nr[r]; ++e) dep |= d->g_r[r * 4 + e] == j;
            if (d->g_tb[r] && j < ng && d->g_eff[(size_t)r * ng + j] != 0.0) dep = true;
            if (dep) colrx.push_back(i);
        }
        for (int r = 0; r < nrs; ++r) {
            bool dep = false;
            for (int e = 0; e < d->s_nf[r]; ++e) dep |= d->s_f[r * 6 + e] == j;
            for (int c = 0; c < d->s_ncov[r]; ++c) dep |= d->s_cov_sp[r * 4 + c] == j;
            if (dep) colrx.push_back(nrg + r);
        }
        colptr.push_back((int)colrx.size());
    }
    // ---- gas-only fast Jacobian (jacobian_fast): reactant / product column lists (no third-body
    //      entries: that dependence goes through the efficiency sets), staged in the LDS image
    std::vector<int> cmp(1, 0);
    std::vector<uint16_t> cmr;
    const char* jf_env = getenv("BRHIP_JFAST");   // "0": the general column-list Jacobian (A/B)
    const bool jfast = (ns == 0) && (M.cpl == 1) && (M.nset <= JF_MAXSET) && (ntb <= WAVE) && (nrg < 65536) &&
                       !(jf_env && atoi(jf_env) == 0);
    if (jfast) {
        for (int j = 0; j < n; ++j) {
            for (int i = 0; i < nrg; ++i) {
                const int r = perm[i];
                bool dep = false;
                for (int e = 0; e < d->g_nf[r]; ++e) dep |= d->g_f[r * 4 + e] == j;
                for (int e = 0; e < d->g_nr[r]; ++e) dep |= d->g_r[r * 4 + e] == j;
                if (dep) cmr.push_back((uint16_t)i);
            }
            cmp.push_back((int)cmr.size());
        }
    }
    // ---- LDS table image: molwt[SPW] | sigma[SPW] | RX | SX | SXE | TBE | TBS | CMP | CMR
    auto al16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t off = IMG_RX_OFF + al16(RX_WORDS * 4 * (size_t)nrg);
    M.sx_off = (int)off;
    off += al16(SX_WORDS * 4 * (size_t)nrs);
    M.sxe_off = (int)off;
    off += al16(8 * SXE_DOUBLES * (size_t)nrs);
    M.tbe_off = (int)off;
    off += al16(16 * tbe.size());
    M.tbs_off = (int)off;
    off += al16(4 * tbs.size());
    M.jfast = jfast ? 1 : 0;
    M.ntbr = ntb;
    M.cmp_off = (int)off;
    off += jfast ? al16(4 * cmp.size()) : 0;
    M.cmr_off = (int)off;
    off += jfast ? al16(2 * cmr.size()) : 0;
    // per gas species, the efficiency sets with eff != 1 (jacobian_fast's third-body columns)
    std::vector<int> tjp(1, 0);
    std::vector<std::pair<int, double>> tje;
    if (jfast) {
        for (int j = 0; j < n; ++j) {
            for (size_t q = 0; q < sets.size(); ++q)
                if (j < ng && sets[q][j] != 1.0) tje.push_back({(int)q, sets[q][j] - 1.0});
            tjp.push_back((int)tje.size());
        }
    }
    M.tjp_off = (int)off;
    off += jfast ? al16(4 * tjp.size()) : 0;
    M.tje_off = (int)off;
    off += jfast ? al16(16 * tje.size()) : 0;
    M.img_bytes = (int)al16(off);
    std::vector<unsigned char> img(M.img_bytes, 0);
    {
        double* mw = reinterpret_cast<double*>(img.data());
        for (int k = 0; k < SPW; ++k) { mw[k] = 1.0; mw[SPW + k] = 1.0; }
        for (int k = 0; k < ng; ++k) mw[k] = d->molwt[k];
        for (int i = 0; i < ns; ++i) mw[SPW + ng + i] = d->sigma ? d->sigma[i] : 1.0;
        if (nrg) {
            uint32_t* ra = reinterpret_cast<uint32_t*>(img.data() + IMG_RX_OFF);
            for (int i = 0; i < nrg; ++i)
                for (int w = 0; w < RX_WORDS; ++w) ra[(w < 4 ? 4 * i : 4 * nrg + 4 * i) + (w & 3)] = rx[(size_t)RX_WORDS * i + w];
        }
        if (nrs) memcpy(img.data() + M.sx_off, sx.data(), sx.size() * 4);
        if (nrs) memcpy(img.data() + M.sxe_off, sxe.data(), sxe.size() * 8);
        if (!tbs.empty()) memcpy(img.data() + M.tbs_off, tbs.data(), tbs.size() * 4);
        if (jfast) {
            memcpy(img.data() + M.cmp_off, cmp.data(), cmp.size() * 4);
            if (!cmr.empty()) memcpy(img.data() + M.cmr_off, cmr.data(), cmr.size() * 2);
            memcpy(img.data() + M.tjp_off, tjp.data(), tjp.size() * 4);
            for (size_t q = 0; q < tje.size(); ++q) {
                memcpy(img.data() + M.tje_off + 16 * q, &tje[q].first, 4);
                memcpy(img.data() + M.tje_off + 16 * q + 8, &tje[q].second, 8);
            }
        }
        for (size_t i = 0; i < tbe.size(); ++i) {
            unsigned char* e = img.data() + M.tbe_off + 16 * i;
            const int sp = tbe[i].first;
            memcpy(e, &sp, 4);
            memcpy(e + 8, &tbe[i].second, 8);
        }
    }
    M.fod_off = fod_off_bytes(nrg);
    M.skd_off = skd_off_bytes(nrg, nfo);
    M.rblock_bytes = rblock_bytes(nrg, nfo, nrs, M.cpl);
    std::vector<double> nasa((size_t)ng * 15);
    for (size_t i = 0; i < (size_t)ng * 15; ++i) nasa[i] = d->nasa[i];
    if (tbeff.empty()) tbeff.push_back(0.0);
    if (colrx.empty()) colrx.push_back(0);
    std::vector<uint4> imgv(M.img_bytes / 16);
    memcpy(imgv.data(), img.data(), M.img_bytes);
    int rc = 0;
    rc |= upload(m, imgv, &M.img);
    rc |= upload(m, nasa, &M.nasa); rc |= upload(m, gpar, &M.g_par); rc |= upload(m, gdnu, &M.g_dnu);
    rc |= upload(m, fopar, &M.fo_par); rc |= upload(m, spar, &M.s_par);
    rc |= upload(m, tbeff, &M.tb_eff); rc |= upload(m, colptr, &M.col_ptr); rc |= upload(m, colrx, &M.col_rx);
    if (rc) { br_mech_destroy(m); return rc; }
    // ---- reactors (waves) per workgroup: the value that maximises resident waves per CU,
    //      from the occupancy calculator (VGPRs, LDS: tables once per workgroup + one block
    //      per reactor); ties go to the smaller workgroup
    const void* kfn = m->nmax == 16 ? (const void*)k_integrate<16>
                    : m->nmax == 32 ? (const void*)k_integrate<32>
                    : m->nmax == 56 ? (const void*)k_integrate<56>
                    : m->nmax == 64 ? (const void*)k_integrate<64> : (const void*)k_integrate<72>;
    int best = 0, best_w = 0;
    for (int rpb = 1; rpb <= br_maxrpb(m->nmax); ++rpb) {
        const size_t b = wg_lds_bytes(M, rpb);
        if (b > LDS_PER_CU) break;
        if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b) != hipSuccess) break;
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, 64 * rpb, b) != hipSuccess) break;
        // the calculator ignores the LDS allocation granule: 3 x 54.5 KB workgroups were reported
        // resident but only 2 were (measured: 6 of 9 waves/CU); count whole granules per CU
        nb = std::min(nb, (int)(LDS_PER_CU / ((b + LDS_GRANULE - 1) / LDS_GRANULE * LDS_GRANULE)));
        if (nb * rpb > best_w) { best_w = nb * rpb; best = rpb; }
    }
    if (best_w == 0) { br_mech_destroy(m); return fail(BR_ERR_UNSUPPORTED, "mechanism too large for LDS"); }
    m->rpb = best;
    m->waves_per_cu = best_w;
    HIPCHK(hipDeviceGetAttribute(&m->ncu, hipDeviceAttributeMultiprocessorCount, device));
    m->shmem = wg_lds_bytes(M, best);
    m->shmem1 = wg_lds_bytes(M, 1);
    // ---- one-reactor-per-lane engine for small gas-only mechanisms (brhip_lane.hpp)
    if (ns == 0 && n <= 12) {
        m->lane_nm = n <= 9 ? 9 : 12;
        const void* lfn = m->lane_nm == 9 ? (const void*)k_lane<9> : (const void*)k_lane<12>;
        m->lane_shmem = lane_lds_bytes(m->lane_nm, n, M.nset, nrg, M.nfo);
        int nb = 0;
        if (m->lane_shmem > 64 * 1024 ||
            hipFuncSetAttribute(lfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->lane_shmem) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lfn, 64, m->lane_shmem) != hipSuccess || nb <= 0) {
            m->lane_nm = 0;   // does not fit: the wave engine integrates it
        } else {
            int ncu = 0;
            HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
            m->lane_blocks = nb * ncu;
        }
    }
    // ---- group engines (brhip_group.hpp): 4 reactors per wave for n <= 16, 2 for n <= 32
    if (n <= 32 && M.nset <= grp::MAX_SETS) {
        m->grp_gl = n <= 16 ? 16 : 32;
        m->grp_nm = n <= 9 ? 9 : (n <= 16 ? 16 : (n <= 24 ? 24 : 32));
        const void* gfn = grp_kernel(m->grp_gl, m->grp_nm);
        m->grp_shmem = (size_t)M.img_bytes + (size_t)BR_QWPB * (64 / m->grp_gl) * grp::block_bytes(m->grp_gl, m->grp_nm, nrg, M.nfo, nrs);
        int nb = 0;
        if (m->grp_shmem > LDS_PER_CU ||
            hipFuncSetAttribute(gfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->grp_shmem) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gfn, 64 * BR_QWPB, m->grp_shmem) != hipSuccess || nb <= 0) {
            m->grp_gl = m->grp_nm = 0;
        } else {
            nb = std::min(nb, (int)(LDS_PER_CU / ((m->grp_shmem + LDS_GRANULE - 1) / LDS_GRANULE * LDS_GRANULE)));
            m->grp_blocks = nb * m->ncu;
        }
    }
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
    if (m->lws) hipFree(m->lws);
    if (m->qws) hipFree(m->qws);
    if (m->queue) hipFree(m->queue);
    if (m->wq) hipFree(m->wq);
    if (m->defer_t0) hipFree(m->defer_t0);
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
constexpr int DEFER_CAP = 4096;   // reactors one k_lane pass may hand to the wavefront engine
static int ensure_jws(br_mech* m, int N) {
    const size_t bytes = (size_t)N * ws_doubles(std::max(m->nmax, 64), m->nrg) * sizeof(double);
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
    rc = ensure_jws(m, N);   // per-reactor slots: {kf, kr} per gas reaction
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
    if (m->dm.cpl == 2) {
        HIPCHK(hipFuncSetAttribute((const void*)k_rates<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_rates<2>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, dp, dx, ns ? dth : nullptr, dw, ds, m->jws);
    } else {
        HIPCHK(hipFuncSetAttribute((const void*)k_rates<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_rates<1>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, dp, dx, ns ? dth : nullptr, dw, ds, m->jws);
    }
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
    rc = ensure_jws(m, N);   // per-reactor slots: {kf, kr} per gas reaction
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* du_ = dA + N;
    double* ddu = du_ + (size_t)N * n;
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    if (m->dm.cpl == 2) {
        HIPCHK(hipFuncSetAttribute((const void*)k_rhs<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_rhs<2>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, Asv ? dA : nullptr, du_, ddu, m->jws);
    } else {
        HIPCHK(hipFuncSetAttribute((const void*)k_rhs<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_rhs<1>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, Asv ? dA : nullptr, du_, ddu, m->jws);
    }
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
    if (m->dm.cpl == 2) {
        HIPCHK(hipFuncSetAttribute((const void*)k_jac<72>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_jac<72>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, pA, du_, dJ, m->jws);
    } else {
        HIPCHK(hipFuncSetAttribute((const void*)k_jac<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem1));
        hipLaunchKernelGGL(k_jac<64>, dim3(N), dim3(64), m->shmem1, 0, m->dm, N, 1, dT, pA, du_, dJ, m->jws);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(J, dJ, (size_t)N * n * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

static int integrate_dev(br_mech* m, int N, const double* dT, const double* dAsv, double* du, const double* dtf,
                         const br_opts* opts, br_stats* dstats, void* stream, double* trace) {
    if (!m || N < 0 || !dT || !du || !dtf) return fail(BR_ERR_INPUT, "bad argument");
    if (N == 0) return 0;
    HIPCHK(hipSetDevice(m->device));
    KOpts o;
    o.rtol = (opts && opts->rtol > 0) ? opts->rtol : 1e-6;
    o.atol = (opts && opts->atol > 0) ? opts->atol : 1e-10;
    o.max_steps = (opts && opts->max_steps > 0) ? opts->max_steps : 100000;
    o.hmax_inv = (opts && opts->hmax > 0) ? 1.0 / opts->hmax : 0.0;
    o.trace_cap = (opts && trace) ? opts->trace_cap : 0;
    o.ufac = opts ? opts->unstable_factor : 0.0;          // <= 0: NaN check only (SciML default)
    o.ign = (opts && opts->ignition_species > 0 && opts->ignition_species <= m->ng) ? opts->ignition_species - 1 : -1;
    o.nout = (opts && opts->nout > 0 && opts->tout && opts->yout) ? opts->nout : 0;
    o.tout = o.nout ? opts->tout : nullptr;
    o.yout = o.nout ? opts->yout : nullptr;
    o.dq_jac = (opts && opts->dq_jacobian) ? 1 : 0;
    o.defer_steps = o.max_steps;
    o.rid_list = nullptr;
    o.rid_count = nullptr;
    o.rid_t0 = nullptr;
    o.work = nullptr;
    hipStream_t s = (hipStream_t)stream;
    const int engine = trace ? 0 : pick_engine(m);   // traced runs: the wavefront engine
    if (engine < 0) {
        // 2 or 4 reactors per wave (one per 32- / 16-lane group), persistent grid over the resident
        // workgroups, reactors from a work counter
        const int GL = m->grp_gl;
        const int gpb = BR_QWPB * (64 / GL);
        const int blocks = std::max(1, std::min((N + gpb - 1) / gpb, m->grp_blocks));
        const size_t need = (size_t)blocks * gpb * grp::slot_doubles(GL, m->nrg) * sizeof(double);
        if (m->qws_bytes < need) {
            if (m->qws) hipFree(m->qws);
            m->qws = nullptr; m->qws_bytes = 0;
            HIPCHK(hipMalloc((void**)&m->qws, need));
            m->qws_bytes = need;
        }
        if (!m->queue) HIPCHK(hipMalloc((void**)&m->queue, (2 + DEFER_CAP) * sizeof(int)));
        HIPCHK(hipMemsetAsync(m->queue, 0, 2 * sizeof(int), s));
        o.work = m->queue;
        const void* gfn = grp_kernel(GL, m->grp_nm);
        HIPCHK(hipFuncSetAttribute(gfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->grp_shmem));
        HIPCHK(hipEventRecord(m->ev0, s));
        const DevMech dm = m->dm;
        double* st_ = (double*)dstats;
        double* qws = m->qws;
        void* args[] = {(void*)&dm, (void*)&N, (void*)&dT, (void*)&dAsv, (void*)&du, (void*)&dtf, (void*)&o, (void*)&st_, (void*)&qws};
        HIPCHK(hipLaunchKernel(gfn, dim3(blocks), dim3(64 * BR_QWPB), args, m->grp_shmem, s));
        HIPCHK(hipEventRecord(m->ev1, s));
        m->ev_recorded = true;
        return 0;
    }
    if (engine > 0) {
        // one reactor per lane; reactors still running after defer_steps steps (a few per 1e4 on
        // H2/O2, some of them up to max_steps) are handed to a follow-up wavefront pass, whose
        // per-step latency for a lone reactor is far lower than a wave's with one live lane
        const int NM = m->lane_nm;
        const int blocks = std::max(1, std::min((N + 63) / 64, m->lane_blocks));
        const size_t need = (size_t)lane_lay(NM, m->n, m->dm.nset, m->nrg, m->dm.nfo).g_rows * blocks * 64 * sizeof(double);
        if (need >= 0x7fffffffull) return fail(BR_ERR_UNSUPPORTED, "lane workspace exceeds the 2 GB buffer range");
        if (m->lws_bytes < need) {
            if (m->lws) hipFree(m->lws);
            m->lws = nullptr; m->lws_bytes = 0;
            HIPCHK(hipMalloc((void**)&m->lws, need));
            m->lws_bytes = need;
        }
        const char* ds = getenv("BRHIP_DEFER_STEPS");
        o.defer_steps = ds ? atoi(ds) : 5000;
        if (o.defer_steps <= 0 || o.defer_steps >= o.max_steps) o.defer_steps = o.max_steps;
        const int cap = std::min(N, DEFER_CAP);
        int rc = ensure_jws(m, cap);
        if (rc) return rc;
        if (!m->queue) HIPCHK(hipMalloc((void**)&m->queue, (2 + DEFER_CAP) * sizeof(int)));
        if (!m->defer_t0) HIPCHK(hipMalloc((void**)&m->defer_t0, DEFER_CAP * sizeof(double)));
        HIPCHK(hipMemsetAsync(m->queue, 0, 2 * sizeof(int), s));
        HIPCHK(hipEventRecord(m->ev0, s));
        if (NM == 9) {
            HIPCHK(hipFuncSetAttribute((const void*)k_lane<9>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->lane_shmem));
            hipLaunchKernelGGL(k_lane<9>, dim3(blocks), dim3(64), m->lane_shmem, s, m->dm, N, dT, du, dtf, o, (double*)dstats, m->lws, m->queue, m->defer_t0, cap);
        } else {
            HIPCHK(hipFuncSetAttribute((const void*)k_lane<12>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->lane_shmem));
            hipLaunchKernelGGL(k_lane<12>, dim3(blocks), dim3(64), m->lane_shmem, s, m->dm, N, dT, du, dtf, o, (double*)dstats, m->lws, m->queue, m->defer_t0, cap);
        }
        HIPCHK(hipGetLastError());
        if (o.defer_steps < o.max_steps) {   // the deferred reactors continue on the wavefront engine
            KOpts o2 = o;
            o2.defer_steps = o.max_steps;
            o2.rid_list = m->queue + 2;
            o2.rid_count = m->queue + 1;
            o2.rid_t0 = m->defer_t0;
            const int rpb = m->rpb;
            HIPCHK(hipFuncSetAttribute((const void*)k_integrate<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
            hipLaunchKernelGGL(k_integrate<16>, dim3((cap + rpb - 1) / rpb), dim3(64 * rpb), m->shmem, s, m->dm, cap, rpb, dT,
                               dAsv, du, dtf, o2, (double*)dstats, m->jws, (double*)nullptr);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(m->ev1, s));
        m->ev_recorded = true;
        return 0;
    }
    const int rpb = m->rpb;
    // persistent grid: as many workgroups as are resident at once, reactors from a work counter
    // (BRHIP_STATIC=1: one reactor per wave over ceil(N / rpb) workgroups)
    const char* st_env = getenv("BRHIP_STATIC");
    const bool dyn = !(st_env && atoi(st_env) == 1) && m->ncu > 0 && m->waves_per_cu >= rpb;
    const int nwg_all = (N + rpb - 1) / rpb;
    const int nwg = dyn ? std::min(nwg_all, m->ncu * (m->waves_per_cu / rpb)) : nwg_all;
    int rc = ensure_jws(m, nwg * rpb);
    if (rc) return rc;
    if (dyn) {
        if (!m->wq) HIPCHK(hipMalloc((void**)&m->wq, sizeof(int)));
        HIPCHK(hipMemsetAsync(m->wq, 0, sizeof(int), s));
        o.work = m->wq;
    }
    HIPCHK(hipEventRecord(m->ev0, s));
    const dim3 grid(nwg), block(64 * rpb);
    if (m->nmax == 16) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<16>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else if (m->nmax == 32) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<32>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else if (m->nmax == 56) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<56>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<56>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else if (m->nmax == 64) {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<64>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
    } else {
        HIPCHK(hipFuncSetAttribute((const void*)k_integrate<72>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m->shmem));
        hipLaunchKernelGGL(k_integrate<72>, grid, block, m->shmem, s, m->dm, N, rpb, dT, dAsv, du, dtf, o, (double*)dstats, m->jws, trace);
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
    const size_t ntr = trace ? (size_t)N * (cap + 1) * (2 * n + 4) : 0;
    const int nout = (opts && opts->nout > 0 && opts->tout && opts->yout) ? opts->nout : 0;
    const size_t nyo = (size_t)N * nout * n;
    const size_t nd = (size_t)N * (3 + n + BR_NSTAT) + ntr + nout + nyo;
    int rc = ensure_ws(m, nd * sizeof(double));
    if (rc) return rc;
    double* dT = (double*)m->ws;
    double* dA = dT + N;
    double* dtf = dA + N;
    double* du_ = dtf + N;
    double* dst = du_ + (size_t)N * n;
    double* dtr = dst + (size_t)N * BR_NSTAT;
    double* dto = dtr + ntr;
    double* dyo = dto + nout;
    br_opts od;
    if (opts) od = *opts;
    if (nout) {
        for (int i = 1; i < nout; ++i)
            if (!(opts->tout[i] >= opts->tout[i - 1])) return fail(BR_ERR_INPUT, "tout must be ascending");
        HIPCHK(hipMemcpy(dto, opts->tout, nout * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dyo, opts->yout, nyo * sizeof(double), hipMemcpyHostToDevice));
        od.tout = dto;
        od.yout = dyo;
    }
    HIPCHK(hipMemcpy(dT, T, N * sizeof(double), hipMemcpyHostToDevice));
    if (Asv) HIPCHK(hipMemcpy(dA, Asv, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dtf, tf, N * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(du_, u, (size_t)N * n * sizeof(double), hipMemcpyHostToDevice));
    if (trace) HIPCHK(hipMemset(dtr, 0, ntr * sizeof(double)));
    rc = integrate_dev(m, N, dT, Asv ? dA : nullptr, du_, dtf, opts ? &od : nullptr, (br_stats*)dst, nullptr,
                       trace ? dtr : nullptr);
    if (rc) return rc;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(u, du_, (size_t)N * n * sizeof(double), hipMemcpyDeviceToHost));
    if (stats) HIPCHK(hipMemcpy(stats, dst, (size_t)N * BR_NSTAT * sizeof(double), hipMemcpyDeviceToHost));
    if (trace) HIPCHK(hipMemcpy(trace, dtr, ntr * sizeof(double), hipMemcpyDeviceToHost));
    if (nout) HIPCHK(hipMemcpy(opts->yout, dyo, nyo * sizeof(double), hipMemcpyDeviceToHost));
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

int br_integrate_multi(br_mech* const* mechs, int ndev, int N, const double* T, const double* Asv, double* u,
                       const double* tf, const br_opts* opts, br_stats* stats) {
    if (!mechs || ndev < 1 || N < 0 || !T || !u || !tf) return fail(BR_ERR_INPUT, "bad argument");
    for (int d = 0; d < ndev; ++d) {
        if (!mechs[d] || mechs[d]->n != mechs[0]->n) return fail(BR_ERR_INPUT, "handles differ in size");
        for (int e = 0; e < d; ++e)
            if (mechs[e] == mechs[d]) return fail(BR_ERR_INPUT, "one handle per shard (handles hold workspaces)");
    }
    const int n = mechs[0]->n;
    const int nout = (opts && opts->nout > 0 && opts->tout && opts->yout) ? opts->nout : 0;
    std::vector<int> rc(ndev, 0);
    std::vector<std::string> msg(ndev);
    std::vector<std::thread> th;
    const int base = N / ndev, extra = N % ndev;
    for (int d = 0; d < ndev; ++d) {
        const int start = d * base + std::min(d, extra), cnt = base + (d < extra ? 1 : 0);
        th.emplace_back([&, d, start, cnt]() {
            br_opts od{};
            if (opts) od = *opts;
            if (nout) od.yout = opts->yout + (size_t)start * nout * n;
            rc[d] = integrate_host(mechs[d], cnt, T + start, Asv ? Asv + start : nullptr, u + (size_t)start * n,
                                   tf + start, opts ? &od : nullptr, stats ? stats + start : nullptr, nullptr);
            if (rc[d]) msg[d] = g_err;
        });
    }
    for (auto& t : th) t.join();
    for (int d = 0; d < ndev; ++d)
        if (rc[d]) return fail(rc[d], "shard " + std::to_string(d) + ": " + msg[d]);
    return 0;
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
    __shared__ double prow[256];
    double* Jt = ws + (size_t)rid * (NMAX * WAVE + lu_ws_doubles(NMAX));
    double* LU = Jt + NMAX * WAVE;
    for (int j = 0; j < NMAX; ++j) Jt[j * WAVE + lane] = (lane < n && j < n) ? J[((size_t)rid * n + lane) * n + j] : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    // twice, as in the integrator: the first factorization loads the rows in natural order (pivot
    // search + gather path), the second in the first one's pivot order (every pivot on its own lane:
    // the factors come out in step order, no gather); the solve uses the second one's factors
    int perm = lane;
    auto factor = [&]() __attribute__((always_inline)) { return lu_factor<NMAX>(Jt, LU, g[rid], n, lane, perm); };
    int f = factor();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    f = factor();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    const double r = lu_solve<NMAX>(LU, n, lane, perm, lane < n ? b[(size_t)rid * n + lane] : 0.0, (LDSd*)prow);
    if (lane < n) x[(size_t)rid * n + lane] = r;
    if (lane == 0) fail[rid] = f;
}
template <int NMAX>
__global__ __launch_bounds__(64) void k_lu_check2(int N, int n, const double* J, const double* g, const double* b,
                                                  double* x, double* ws, int* fail) {
    constexpr int JW = CR2;
    __shared__ double scr[256];
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    double* Jt = ws + (size_t)rid * (NMAX * JW + lu_ws_doubles(NMAX));
    double* LU = Jt + NMAX * JW;
    for (int j = 0; j < NMAX; ++j)
        for (int s = 0; s < 2; ++s) {
            const int row = lane + 64 * s;
            if (row < JW) Jt[j * JW + row] = (row < n && j < n) ? J[((size_t)rid * n + row) * n + j] : 0.0;
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    // twice, as k_lu_check: natural order first (gather path), then the first one's pivot order
    // (the no-gather path when every pivot stays on its position); the solve uses the second
    int perm[2] = {lane, lane + 64};
    int f = lu_factor2<NMAX>(Jt, LU, (LDSd*)scr, g[rid], n, lane, perm);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    f = lu_factor2<NMAX>(Jt, LU, (LDSd*)scr, g[rid], n, lane, perm);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    double r[2];
    for (int s = 0; s < 2; ++s) r[s] = (lane + 64 * s < n) ? b[(size_t)rid * n + lane + 64 * s] : 0.0;
    lu_solve2<NMAX>(LU, (LDSd*)scr, n, lane, perm, r);
    for (int s = 0; s < 2; ++s) if (lane + 64 * s < n) x[(size_t)rid * n + lane + 64 * s] = r[s];
    if (lane == 0) fail[rid] = f;
}
}  // namespace

// device buffers of the diagnostic entry points below, freed on every exit path (HIPCHK returns early)
namespace {
struct DevScratch {
    std::vector<void*> p;
    ~DevScratch() {
        for (void* q : p) hipFree(q);
    }
    template <class T>
    hipError_t alloc(T** out, size_t bytes) {
        void* q = nullptr;
        const hipError_t e = hipMalloc(&q, bytes);
        if (e == hipSuccess) { p.push_back(q); *out = (T*)q; }
        return e;
    }
};
}  // namespace

extern "C" int br_debug_lu_solve(int N, int n, const double* J, const double* gamma, const double* b, double* x,
                                 int* fail_out) {
    if (N <= 0 || n <= 0 || n > 72) return fail_code_input();
    const int nmax = n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 56 ? 56 : (n <= 64 ? 64 : 72)));
    double *dJ, *dg, *db, *dx, *dws;
    int* df;
    DevScratch S;
    HIPCHK(S.alloc(&dJ, (size_t)N * n * n * 8));
    HIPCHK(S.alloc(&dg, (size_t)N * 8));
    HIPCHK(S.alloc(&db, (size_t)N * n * 8));
    HIPCHK(S.alloc(&dx, (size_t)N * n * 8));
    HIPCHK(S.alloc(&dws, (size_t)N * (nmax * col_rows(nmax) + lu_ws_doubles(nmax)) * 8));
    HIPCHK(S.alloc(&df, (size_t)N * 4));
    HIPCHK(hipMemcpy(dJ, J, (size_t)N * n * n * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dg, gamma, (size_t)N * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(db, b, (size_t)N * n * 8, hipMemcpyHostToDevice));
    if (nmax == 16) hipLaunchKernelGGL(k_lu_check<16>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else if (nmax == 32) hipLaunchKernelGGL(k_lu_check<32>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else if (nmax == 56) hipLaunchKernelGGL(k_lu_check<56>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else if (nmax == 64) hipLaunchKernelGGL(k_lu_check<64>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else hipLaunchKernelGGL(k_lu_check2<72>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(x, dx, (size_t)N * n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(fail_out, df, (size_t)N * 4, hipMemcpyDeviceToHost));
    return 0;
}

#if BR_PHASE_CLOCKS
// diagnostic build only (not declared in brhip.h): read and reset the 16 sub-phase clock sums
// (BR_SUB_ADD slots of brhip_device.hpp)
extern "C" int br_diag_sub(double* out16) {
    std::vector<unsigned long long> v((size_t)brhip::SUB_MAXW * 16, 0ull);
    if (hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(brhip::g_sub), v.size() * 8) != hipSuccess) return -1;
    for (int i = 0; i < 16; ++i) out16[i] = 0.0;
    for (size_t w = 0; w < (size_t)brhip::SUB_MAXW; ++w)
        for (int i = 0; i < 16; ++i) out16[i] += (double)v[w * 16 + i];
    std::fill(v.begin(), v.end(), 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(brhip::g_sub), v.data(), v.size() * 8) != hipSuccess) return -1;
    return 0;
}
#endif
