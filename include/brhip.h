/*
 * brhip.h -- C-ABI of libbrhip.so, the MI355X (gfx950) batched stiff-kinetics engine that
 * sits behind BatchReactor.jl's hot path. Plain C types only; fp64 everywhere; int status
 * return (0 = OK, negative = error class, message via br_last_error()).
 *
 * Reference interfaces each entry point replaces (paths relative to the reference root):
 *   br_mech_create   <- compile_gaschemistry / SurfaceReactions.compile_mech /
 *                       IdealGas.create_thermo results (src/BatchReactor.jl:254,265,287):
 *                       the host flattens the compiled mechanism into br_mech_desc.
 *   br_mech_parse /  <- the same three compilers reading the mechanism library files
 *   br_mech_compile     (src/BatchReactor.jl:242-287); br_read_batch_xml <- input_data (:238-306)
 *   br_rates         <- GasphaseReactions.calculate_molar_production_rates!(g_state,gmd,thermo)
 *                       (call site src/BatchReactor.jl:355) and
 *                       SurfaceReactions.calculate_molar_production_rates!(s_state,thermo,smd)
 *                       (call site :344), batched over N states.
 *   br_rhs           <- residual!(du,u,p,t) (src/BatchReactor.jl:312-376), batched.
 *   br_jacobian      <- the dense Jacobian CVODE builds by finite differences inside
 *                       solve(..., CVODE_BDF()) (:138-141, :208-210); here analytic.
 *   br_integrate     <- solve(ODEProblem(residual!,u0,(0,tf),params), CVODE_BDF();
 *                       reltol=1e-6, abstol=1e-10, save_everystep=false)
 *                       (src/BatchReactor.jl:138-141 and :204-210), for N reactors at once.
 *   br_integrate_dev <- same, device-resident buffers on a caller stream (ensemble driver).
 *
 * Layout: per-reactor rows, reactor-major: u[N][n] with n = ng + ns and
 * u_k = rho*Y_k (kg/m3) for k < ng, theta_k for ng <= k < n (src/BatchReactor.jl:224-231).
 * A handle may be used by one host thread at a time; there is no global state.
 */
#ifndef BRHIP_H
#define BRHIP_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define BR_OK             0
#define BR_ERR_MAXSTEPS  -1   /* CVODE CV_TOO_MUCH_WORK  */
#define BR_ERR_ERRTEST   -3   /* CVODE CV_ERR_FAILURE     */
#define BR_ERR_CONV      -4   /* CVODE CV_CONV_FAILURE    */
#define BR_ERR_UNSTABLE  -7   /* NaN state (SciML ReturnCode.Unstable), or the opt-in runaway test of
                                 br_opts.unstable_factor */
#define BR_ERR_RHS       -8   /* CVODE CV_RHSFUNC_FAIL: a br_integrate_host right-hand side returned != 0 */
#define BR_ERR_INPUT    -10
#define BR_ERR_HIP      -20
#define BR_ERR_UNSUPPORTED -30

/* convention switches (bitmask); 0 = textbook CHEMKIN-II in SI units. BR_CONV_REFERENCE is what
 * the reference's GasphaseReactions does (identified from its golden output):
 * rates in mol/cm3 with Kc = Kp (p0/RT)^dnu in mol/m3, falloff rates also x [M] (mol/cm3), Troe
 * c = -4.0 - 0.67 log10 Fcent. */
#define BR_CONV_KC_UNIT_SLIP  1   /* Kc *= (1e6)^dnu for every reversible reaction          */
#define BR_CONV_FALLOFF_XM    2   /* falloff net rate *= [M] in mol/cm3 (1e-6 [M]_SI)       */
#define BR_CONV_DOC_COVG      4   /* no Asv on dtheta/dt (docs sample, predates :345)      */
#define BR_CONV_TROE_C4      16   /* Troe c = -4.0 - 0.67 log10 Fcent                       */
#define BR_CONV_REFERENCE    (BR_CONV_KC_UNIT_SLIP | BR_CONV_FALLOFF_XM | BR_CONV_TROE_C4)

typedef struct br_mech br_mech;

typedef struct br_mech_desc {
    int ng, ns, nrg, nrs;
    int conv;                 /* BR_CONV_* bitmask                                 */
    double p_std;             /* standard pressure for Kc [Pa]                     */
    const double* molwt;      /* [ng] kg/mol                                       */
    const double* nasa;       /* [ng][15]: Tmid, a_hi[7], a_lo[7] (NASA-7)         */
    /* gas reactions (CHEMKIN-II) */
    const int* g_nf;          /* [nrg] expanded reactant entries (<=4)             */
    const int* g_nr;          /* [nrg] expanded product entries  (<=4)             */
    const int* g_f;           /* [nrg][4] species index per entry, -1 pad          */
    const int* g_r;           /* [nrg][4]                                          */
    const int* g_rev;         /* [nrg] 1 reversible                                */
    const int* g_tb;          /* [nrg] 0 none, 1 third body (+M), 2 falloff (+M)   */
    const double* g_arr;      /* [nrg][3] A (SI), beta, Ea/R [K] (k_inf if falloff) */
    const double* g_low;      /* [nrg][3] k0: A (SI), beta, E/R                    */
    const int* g_troe_n;      /* [nrg] 0 Lindemann, else number of Troe params 3|4 */
    const double* g_troe;     /* [nrg][4] a, T***, T*, T**                         */
    const double* g_eff;      /* [nrg][ng] third-body efficiencies (tb rows)       */
    /* surface reactions */
    double site_density;      /* mol/cm2                                           */
    const double* sigma;      /* [ns] site coordination                           */
    const int* s_nf;          /* [nrs] <=6                                         */
    const int* s_np;          /* [nrs] <=6                                         */
    const int* s_f;           /* [nrs][6] combined index: gas 0..ng-1, surface ng.. */
    const int* s_p;           /* [nrs][6]                                          */
    const int* s_stick;       /* [nrs] 1 sticking coefficient reaction             */
    const double* s_arr;      /* [nrs][3] A (SI) or s0, beta, Ea [J/mol]           */
    const int* s_ncov;        /* [nrs] coverage-dependent terms (<=4)              */
    const int* s_cov_sp;      /* [nrs][4] combined species index                  */
    const double* s_cov_eps;  /* [nrs][4] J/mol                                    */
} br_mech_desc;

typedef struct br_opts {
    double rtol, atol;        /* default 1e-6 / 1e-10 (src/BatchReactor.jl:141,:210) */
    int max_steps;            /* default 100000 (Sundials.jl maxiters)             */
    int device;               /* HIP device ordinal for br_mech_create             */
    double hmax;              /* 0 = unbounded                                     */
    int trace_cap;            /* br_integrate_traced: max accepted steps recorded  */
    double unstable_factor;   /* > 0: also stop a reactor with BR_ERR_UNSTABLE once max_k |u_k|
                                 exceeds factor * sum_k |u0_k| (not a reference behaviour;
                                 default 0 = only a NaN state stops it, as SciML's check) */
    int ignition_species;     /* 1-based gas species index k+1 whose max dX_k/dt over the accepted
                                 steps marks ignition (br_stats.t_ign; OH for the reference's
                                 ignition marker); 0 = not tracked                          */
    int nout;                 /* dense output: number of output times (0 = none)            */
    const double* tout;       /* [nout] ascending output times, shared by all reactors; the
                                 state there is CVODE's CV_NORMAL output (CVodeGetDky(t, 0) on
                                 the step that passes t), the step sequence is unchanged     */
    double* yout;             /* [N][nout][n] states at tout (host memory for br_integrate,
                                 device memory for br_integrate_dev); rows with tout > tf are
                                 left untouched                                             */
    int dq_jacobian;          /* 1: CVODE's dense difference-quotient Jacobian (cvLsDenseDQJac:
                                 the reference's CVODE_BDF() setting, src/BatchReactor.jl:140,
                                 :204), n extra RHS per Jacobian, in every engine (lane,
                                 group, wavefront); 0 (default): the analytic Jacobian       */
} br_opts;

#define BR_NSTAT 20
typedef struct br_stats {     /* per reactor; counters as CVODE's, then device cycles */
    double nsteps, nfe, nje, nsetups, nni, ncfn, netf, status;
    double cyc_total;         /* wall clock ticks (100 MHz) for the whole reactor  */
    double cyc_rhs, cyc_jac, cyc_lu, cyc_sol;  /* shader clocks in each phase      */
    double t_end;             /* time reached                                      */
    double cyc_ctl;           /* shader clocks in the step controller (diagnostic build) */
    double cyc_clk;           /* shader clocks for the whole reactor (diagnostic build)  */
    double t_ign;             /* ignition time: midpoint of the accepted step with the largest
                                 dX_k/dt, k = br_opts.ignition_species (NaN if not tracked) */
    double ign_rate;          /* that largest dX_k/dt [1/s]                                */
    double ign_dt;            /* width of that step (the resolution of t_ign) [s]            */
    double nfe_dq;            /* RHS evaluations of the DQ Jacobian (CVODE's nfeDQ; not in nfe) */
} br_stats;

int         br_version(void);
const char* br_last_error(void);
int         br_device_count(void);

int br_mech_create(const br_mech_desc* desc, int device, br_mech** out);

/* ---- host mechanism compiler (C++, no GPU): the data formats the reference reads, flattened into
 * br_mech_desc. Replaces, as one step:
 *   compile_gaschemistry(get_path(lib_dir, <gas_mech>))       src/BatchReactor.jl:251-255
 *   IdealGas.create_thermo(gasphase, get_path(lib_dir, "therm.dat"))                   :242-243,:265
 *   SurfaceReactions.compile_mech(get_path(lib_dir, <surface_mech>), thermo, gasphase) :283-287
 * gas_mech_path: CHEMKIN-II mechanism, or NULL/"" for surface-only runs, whose gas species are then
 * the space-separated names of `gasphase` (the <gasphase> tag, :256-260). surf_mech_path: surface
 * XML or NULL. conv: BR_CONV_* bits (BR_CONV_REFERENCE = the reference's gas kinetics). The
 * tables are bit-identical to the Python host compiler's (batchreactor.jl_amd/mechanism.py). */
typedef struct br_host_mech br_host_mech;
int br_mech_parse(const char* gas_mech_path, const char* therm_path, const char* surf_mech_path,
                  const char* gasphase, int conv, br_host_mech** out);
/* desc's pointers point into h: valid until br_host_mech_free(h) */
int br_host_mech_desc(const br_host_mech* h, br_mech_desc* desc);
int br_host_mech_sizes(const br_host_mech* h, int* ng, int* ns, int* nrg, int* nrs);
/* name of species i (gas species 0..ng-1 in mechanism order, then surface species), upper case */
int br_host_mech_species(const br_host_mech* h, int i, char* buf, size_t n);
/* initial coverages of the surface species (<site><initial>, the u0 tail of :228-230) */
int br_host_mech_theta0(const br_host_mech* h, double* theta0 /*[ns]*/);
int br_host_mech_free(br_host_mech* h);
/* br_mech_parse + br_mech_create in one call */
int br_mech_compile(const char* gas_mech_path, const char* therm_path, const char* surf_mech_path,
                    const char* gasphase, int conv, int device, br_mech** out);

/* batch.xml (input_data, src/BatchReactor.jl:238-306; schema docs/src/index.md:80-123). Asv is 1
 * when the tag is missing (the reference's behaviour). The composition is the
 * <molefractions> list (comp_is_mass = 0) or else <massfractions> (1), names upper case. */
#define BR_BATCH_MAXCOMP 64
typedef struct br_batch_input {
    char gas_mech[256];
    char surface_mech[256];
    char gasphase[1024];      /* space-separated gas species names (surface-only runs) */
    double T, p, Asv, time;
    int has_T, has_p, has_Asv, has_time;
    int ncomp, comp_is_mass;
    char comp_names[BR_BATCH_MAXCOMP][32];
    double comp_values[BR_BATCH_MAXCOMP];
} br_batch_input;
int br_read_batch_xml(const char* path, br_batch_input* out);
int br_mech_destroy(br_mech* m);
int br_mech_info(const br_mech* m, int* ng, int* ns, int* nrg, int* nrs);
/* integrator engine br_integrate* uses for this mechanism: 0 = one reactor per wavefront
 * (k_integrate), NM > 0 = one reactor per lane with NM-wide register tiles (k_lane, gas-only
 * mechanisms with n <= 12), -(100 GL + NM) < 0 = a group engine, one reactor per GL-lane group of a
 * wavefront with NM-wide register tiles (k_group<GL, NM>; GL = 16 "quad", n <= 16, the default for
 * such mechanisms; GL = 32 "pair", 16 < n <= 32; gas and surface chemistry, <= 32 third-body
 * efficiency sets). All of them take br_opts.dq_jacobian. Traced integrations always use the
 * wavefront engine; env BRHIP_ENGINE = wave | lane | quad | pair forces one where the mechanism is
 * eligible. */
int br_mech_engine(const br_mech* m);
/* launch geometry of the engine br_integrate uses for this mechanism (br_mech_engine; diagnostics):
 * reactors per workgroup, resident waves per CU (occupancy calculator: VGPRs and LDS), LDS bytes
 * per workgroup (staged tables + one block per reactor or group). Any pointer may be NULL. */
int br_mech_launch_info(const br_mech* m, int* rpb, int* waves_per_cu, long long* lds_bytes);

/* host-buffer entry points (copy in/out); arrays are reactor-major */
int br_rates(br_mech* m, int N, const double* T, const double* p, const double* x /*[N][ng]*/,
             const double* theta /*[N][ns] or NULL*/, double* wdot /*[N][ng]*/,
             double* sdot /*[N][ng+ns] or NULL*/);
int br_rhs(br_mech* m, int N, const double* T, const double* Asv, const double* u /*[N][n]*/,
           double* du /*[N][n]*/);
int br_jacobian(br_mech* m, int N, const double* T, const double* Asv, const double* u,
                double* J /*[N][n][n] row-major d(du_i)/d(u_j)*/);
int br_integrate(br_mech* m, int N, const double* T, const double* Asv, double* u /*in/out*/,
                 const double* tf, const br_opts* opts, br_stats* stats /*[N] or NULL*/);

/* as br_integrate, and also records the state after every accepted step (the rows
 * save_data writes, src/BatchReactor.jl:383-402): trace[N][trace_cap+1][2n+4] with
 * row = (t, h, q, p_last, u[0..n-1], y[0..n-1]): u is the accepted state, y and p_last the state
 * and pressure of the last RHS evaluation of that step (save_data reads x, p and coverages from
 * the last RHS call and rho from u). Row 0 is t=0; unused rows are left as zeros. The last
 * written row is the tstop row (t = tf). */
int br_integrate_traced(br_mech* m, int N, const double* T, const double* Asv, double* u,
                        const double* tf, const br_opts* opts, br_stats* stats, double* trace);

/* multi-GPU ensemble: N reactors split into ndev contiguous slices (sizes
 * differ by at most one), slice d integrated on mechs[d] -- one handle per GPU, created with
 * br_mech_create(desc, device d, ...) -- concurrently (one host thread per handle), results
 * written back into the caller's host arrays in ensemble order. No inter-GPU traffic: every
 * slice is copied straight back to host memory. Arguments as br_integrate (opts->yout, when set,
 * is [N][nout][n] for the whole ensemble). Replaces running the reference's solve() once per
 * reactor (src/BatchReactor.jl:138-141). */
int br_integrate_multi(br_mech* const* mechs, int ndev, int N, const double* T, const double* Asv, double* u,
                       const double* tf, const br_opts* opts, br_stats* stats);

/* device-buffer entry point: all pointers are device memory on m's device; `stream` is a
 * hipStream_t (NULL = default stream). Asynchronous: returns after the launch. Calls on one
 * handle share its workspaces (work counter, Jacobian / LU slots, timing events): they must be
 * ordered on one stream (or synchronised); concurrent integrations need one handle each. */
int br_integrate_dev(br_mech* m, int N, const double* dT, const double* dAsv, double* du,
                     const double* dtf, const br_opts* opts, br_stats* dstats, void* stream);

/* dense-solver check (tests): factor I - gamma_i*J_i with the engine's batched LU and solve
 * x_i = (I - gamma_i J_i)^-1 b_i. J[N][n][n] row-major; fail[i] = 0 or (k+1) for a zero pivot. */
int br_debug_lu_solve(int N, int n, const double* J, const double* gamma, const double* b, double* x, int* fail);

/* User-defined chemistry: replaces solve(ODEProblem(residual!, u0, (0, tf), params), CVODE_BDF();
 * reltol, abstol, save_everystep=false, callback=FunctionCallingCallback(save_data)) with the userchem
 * residual! (src/BatchReactor.jl:51-54,:197-200,:204-210,:358-360,:371-372). The user's RHS is host
 * code (a Julia or Python function: it cannot run in a kernel), so this runs on the CPU: the same
 * CVODE 5.x restatement as the engine, with CVODE's DQ Jacobian (the reference supplies none).
 * f(user, t, u, du) returns 0 (non-zero ends the solve with BR_ERR_RHS); cb(cb_user, t, u) after every
 * accepted step and at t = 0 and t = tf (save_data's rows). u: u0 in, u(tf) out (the last accepted
 * state on failure); stats[BR_NSTAT] as br_stats. Returns 0 or a BR_ERR_* status. No GPU. */
typedef int (*br_rhs_fn)(void* user, double t, const double* u, double* du);
typedef void (*br_step_fn)(void* user, double t, const double* u);
int br_integrate_host(int n, br_rhs_fn f, void* user, double* u, double tf, double rtol, double atol, int max_steps,
                      br_step_fn cb, void* cb_user, double* stats);

/* timing helper for roofline accounting: duration (ms) of the last integrate kernel,
 * measured with HIP events on the stream it was launched on (after the stream syncs). */
int br_last_kernel_ms(br_mech* m, double* ms);

#ifdef __cplusplus
}
#endif
#endif
