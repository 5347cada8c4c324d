/*
 * oracle.h -- CPU restatement of BatchReactor.jl's hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the checker for the HIP engine (libbrhip.so). Only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it. The
 * product path never links, imports or falls back to it.
 *
 * What it restates (reference = /root/reference, v0.1.4):
 *   - residual!(du,u,p,t)                    src/BatchReactor.jl:312-376
 *   - initial state (rho_k = Y_k*rho0, theta0) src/BatchReactor.jl:224-232, :130-135
 *   - final conversion Y -> x                  src/BatchReactor.jl:142-145
 *   - gas production rates  (GasphaseReactions.calculate_molar_production_rates!, call
 *     site :355; package not vendored -> CHEMKIN-II contract + named convention switches,
 *     SURVEY.md A.4)
 *   - surface production rates (SurfaceReactions.calculate_molar_production_rates!, call
 *     site :344; not vendored -> SURVEY.md A.2 contract, pinned by docs/src/index.md:160-185)
 *   - the integrator: solve(..., CVODE_BDF(), reltol=1e-6, abstol=1e-10) (:138-141,:208-210)
 *     -> a restatement of SUNDIALS CVODE 5.x (Sundials_jll 5.2, pinned through
 *     Sundials.jl 4.x, Project.toml:24): Nordsieck BDF q<=5, modified Newton (maxcor 3),
 *     dense DQ Jacobian (cvLsDenseDQJac) or analytic Jacobian, dense LU with partial
 *     pivoting, WRMS error control, cvHin initial step, tstop handling.
 * Parity pins: tests/golden/* (subsampled from test/batch_gas_and_surf/*.csv and the
 * doc rows docs/src/index.md:160-185). Gas-phase conventions are only partially pinned
 * (see DESIGN.md "Parity status").
 */
#ifndef BR_ORACLE_H
#define BR_ORACLE_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* convention switches (bitmask); 0 = textbook CHEMKIN-II (SI throughout).
 * ORC_CONV_REFERENCE = the conventions of the GasphaseReactions version that produced the
 * reference's golden (test/batch_gas_and_surf/gas_profile.csv), identified in round 2 from the
 * golden's first 40 accepted steps (tests/test_oracle.py::test_golden_early_rows_all_species):
 *   KC_UNIT_SLIP  rates in mol/cm3 but Kc = exp(-dG/RT) (p0/RT)^dnu in mol/m3, i.e. in SI terms
 *                 Kc *= (1e6)^dnu for every reversible reaction;
 *   FALLOFF_XM    (+M) falloff rates are also multiplied by [M] (in mol/cm3 = 1e-6 [M]_SI);
 *   TROE_C4       Troe c = -4.0 - 0.67 log10(Fcent) (instead of -0.4). */
#define ORC_CONV_KC_UNIT_SLIP   1
#define ORC_CONV_FALLOFF_XM     2
#define ORC_CONV_DOC_COVG       4  /* no Asv on dtheta/dt (docs sample predates :345)          */
#define ORC_CONV_TROE_C4       16
#define ORC_CONV_REFERENCE     (ORC_CONV_KC_UNIT_SLIP | ORC_CONV_FALLOFF_XM | ORC_CONV_TROE_C4)

typedef struct orc_mech orc_mech;

typedef struct {
    double rtol, atol;     /* 1e-6, 1e-10 (:141,:210) */
    int    analytic_jac;   /* 0 = CVODE DQ Jacobian (reference), 1 = analytic */
    int    max_steps;      /* Sundials.jl maxiters default 1e5 */
    double hmax;           /* 0 = inf */
    double unstable_factor;/* > 0: abort (status -7) once max|u_k| > factor * sum|u0| (opt-in, not a
                              reference behaviour); always: a NaN state -> -7 (SciML unstable_check) */
    int    ignition_species;/* 1-based gas species index whose max dX/dt marks ignition; 0 = off */
} orc_opts;

typedef struct {
    long nsteps, nfe, nje, nsetups, nni, ncfn, netf, nfeDQ;
    int  status;           /* 0 ok, -1 too much work, -3 err fail, -4 conv fail, -6 LU fail,
                              -7 unstable (runaway state) */
    int  qlast;
    double hlast, tcur;
    double t_ign, ign_rate;/* midpoint of the accepted step with the largest dX_ign/dt, and that rate */
    double ign_dt;         /* width of that step */
} orc_stats;

/* per-accepted-step callback: t, u (solver state), and the "last RHS" state
 * (p, x[ng], theta[ns]) exactly as save_data (src/BatchReactor.jl:383-402) sees it */
typedef void (*orc_step_cb)(void* user, double t, const double* u, double p_last,
                            const double* x_last, const double* th_last);

/* load: gas_mech may be NULL (surface-only; then gas_species lists the <gasphase> tag),
 * surf_mech may be NULL (gas-only). Returns NULL on error (message in orc_errmsg()). */
orc_mech* orc_load(const char* gas_mech, const char* therm, const char* surf_mech,
                   const char* gas_species /* space separated, or NULL */, int conv, double p_std);
void        orc_free(orc_mech* m);
const char* orc_errmsg(void);
int  orc_ng(const orc_mech* m);
int  orc_ns(const orc_mech* m);
int  orc_nrg(const orc_mech* m);
int  orc_nrs(const orc_mech* m);
const char* orc_species_name(const orc_mech* m, int k);   /* gas 0..ng-1, then surface */
double orc_molwt(const orc_mech* m, int k);
double orc_site_density(const orc_mech* m);               /* mol/cm2 */
void   orc_initial_coverage(const orc_mech* m, double* th);
void   orc_set_conv(orc_mech* m, int conv);
/* test hook: multiply gas reaction i's forward / reverse terms (default 1.0) */
void   orc_set_rxn_mult(orc_mech* m, int i, double fmul, double rmul);

/* rho_k from mole fractions (src/BatchReactor.jl:224-232 / IdealGas.density) */
void orc_initial_state(const orc_mech* m, double T, double p, const double* x, double* u);
/* rates at (T,p,x,theta): wdot[ng] mol/m3/s, sdot[ng+ns] mol/m2/s (no Asv) */
void orc_rates(const orc_mech* m, double T, double p, const double* x, const double* th,
               double* wdot, double* sdot);
/* per-reaction rates of progress (gas qg[nrg], surface qs[nrs]) */
void orc_rop(const orc_mech* m, double T, double p, const double* x, const double* th,
             double* qg, double* qs);
/* residual! : du = f(u); also returns the diagnosed p and x (may be NULL) */
void orc_rhs(const orc_mech* m, double T, double Asv, const double* u, double* du,
             double* p_out, double* x_out);
/* analytic Jacobian d(du)/du, row-major n x n */
void orc_jac(const orc_mech* m, double T, double Asv, const double* u, double* J);
/* integrate one reactor 0 -> tf; u is in/out */
int  orc_integrate(const orc_mech* m, double T, double Asv, double* u, double tf,
                   const orc_opts* o, orc_stats* st, orc_step_cb cb, void* user);
/* same, plus the state at nout ascending output times (CV_NORMAL + CVodeGetDky); yout[nout][n] */
int  orc_integrate_out(const orc_mech* m, double T, double Asv, double* u, double tf, const orc_opts* o,
                       orc_stats* st, int nout, const double* tout, double* yout);
/* diagnostic: perturb every rate of progress by a relative +-eps (0 = off; not thread-safe) */
void orc_set_rop_jitter(double eps);
void orc_set_rop_jitter_seed(unsigned long long seed);   /* jitter realisation (streams per reactor index) */
/* diagnostic: pivot-order statistics of the factorizations (this thread; orc_lu_diag(1) resets and
 * enables): out4 = factorizations, those whose pivot order differs from the previous one's, steps,
 * row interchanges needed when the rows are loaded in the previous pivot order, sum of their steps,
 * the same within a 32-column panel, the first factorization's interchanges, steps whose column max shares
 * its high word with another candidate */
void orc_lu_diag(int on);
void orc_lu_stats(long* out8);
/* ensemble (OpenMP over reactors): u[N][n] row per reactor */
int  orc_integrate_batch(const orc_mech* m, int N, const double* T, const double* Asv,
                         double* u, const double* tf, const orc_opts* o, orc_stats* st,
                         int nthreads);
/* same, plus each reactor's states at the nout output times: yout[N][nout][n] */
int  orc_integrate_batch_out(const orc_mech* m, int N, const double* T, const double* Asv,
                             double* u, const double* tf, const orc_opts* o, orc_stats* st,
                             int nthreads, int nout, const double* tout, double* yout);

#ifdef __cplusplus
}
#endif
#endif
