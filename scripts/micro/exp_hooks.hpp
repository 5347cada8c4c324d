// exp_hooks.hpp -- diagnostic-only experiment hooks for k_integrate (never in the product build).
// Build a variant library with
//   hipcc ... -DBR_EXPERIMENT_HOOKS='"../../scripts/micro/exp_hooks.hpp"' -DBR_EXP_DUP=1 ... brhip.hip
// (scripts/pmc_ab.sh). The macros expand inside k_integrate's Newton loop and use its locals.
//   BR_EXP_DUP=1/2/3 : the RHS / the linear solve / the Jacobian evaluated twice (SQ_INSTS_VALU of
//                      one phase = the difference to the plain build)
//   BR_EXP_VALU=K    : K independent dummy fp64 FMAs per Newton iteration (VALU-issue sensitivity)
//   BR_EXP_MEM=K     : K columns (512 B each) of the saved J re-read per Newton iteration (memory-
//                      side sensitivity)
//   BR_EXP_GDUP=1/2/3/4 : k_group (group engines): the RHS / the solve / the Jacobian / the LU run
//                      twice (scripts/gdup_valu.sh)
#pragma once

//   BR_EXP_CDUP=1/2    : in the 16-lane groups' controller, cvSet / the etaq ratio (root_int + the
//                      division) evaluated twice on opaque copies of their inputs
#if defined(BR_EXP_CDUP) && BR_EXP_CDUP == 1
#define BR_XC_AFTER_CVSET()                                                                  \
    do {                                                                                     \
        if constexpr (GW == 16) {                                                            \
            AttemptIn in2 = in;                                                              \
            asm volatile("" : "+v"(in2.q), "+v"(in2.qwait), "+v"(in2.nst), "+v"(in2.h));     \
            asm volatile("" : "+v"(in2.gammap), "+v"(in2.tau[1]), "+v"(in2.tau[2]));          \
            asm volatile("" : "+v"(in2.tau[3]), "+v"(in2.tau[4]), "+v"(in2.tau[5]), "+v"(in2.tau[6])); \
            double t4b, grb;                                                                 \
            cv_set_lp(C, in2, t4b, grb);                                                     \
            asm volatile("" ::"v"(t4b), "v"(grb));                                           \
        }                                                                                    \
    } while (0)
#endif
#if defined(BR_EXP_CDUP) && BR_EXP_CDUP == 3   // the wavefront engine's cvSet (GW = 64)
#define BR_XC_AFTER_CVSET()                                                                  \
    do {                                                                                     \
        if constexpr (GW == 64) {                                                            \
            AttemptIn in2 = in;                                                              \
            asm volatile("" : "+s"(in2.q), "+s"(in2.qwait), "+s"(in2.nst));                  \
            asm volatile("" : "+v"(in2.h), "+v"(in2.gammap), "+v"(in2.tau[1]), "+v"(in2.tau[2])); \
            asm volatile("" : "+v"(in2.tau[3]), "+v"(in2.tau[4]), "+v"(in2.tau[5]), "+v"(in2.tau[6])); \
            double t4b, grb;                                                                 \
            cv_set_lp(C, in2, t4b, grb);                                                     \
            asm volatile("" ::"v"(t4b), "v"(grb));                                           \
        }                                                                                    \
    } while (0)
#endif
#if defined(BR_EXP_CDUP) && BR_EXP_CDUP == 2
#define BR_XC_AFTER_ETAQ()                                                                   \
    do {                                                                                     \
        if constexpr (GW == 16) {                                                            \
            double x2 = BIAS2 * dsm;                                                         \
            int L2 = L;                                                                      \
            asm volatile("" : "+v"(x2), "+v"(L2));                                           \
            const double e2 = 1.0 / (root_int(x2, L2) + ADDON);                              \
            asm volatile("" ::"v"(e2));                                                      \
        }                                                                                    \
    } while (0)
#endif
#if defined(BR_EXP_CDUP)
#ifndef BR_XC_AFTER_CVSET
#define BR_XC_AFTER_CVSET()
#endif
#ifndef BR_XC_AFTER_ETAQ
#define BR_XC_AFTER_ETAQ()
#endif
#endif

#if defined(BR_EXP_GDUP) && BR_EXP_GDUP == 1
#define BR_XG_AFTER_RHS()                                                                    \
    do {                                                                                     \
        asm volatile("" ::: "memory");                                                       \
        double f2 = g_rhs<GL>(tb, sp, kd, fod, skd, T, Asv, Asv_th, yv, gl, p_last);         \
        asm volatile("" ::"v"(f2));                                                          \
    } while (0)
#else
#define BR_XG_AFTER_RHS()
#endif
#if defined(BR_EXP_GDUP) && BR_EXP_GDUP == 2
#define BR_XG_AFTER_SOLVE()                                                                  \
    do {                                                                                     \
        asm volatile("" ::"v"(delta[0]) : "memory");   /* the first solve stays live */      \
        double bb = b[0];                                                                    \
        asm volatile("" : "+v"(bb));   /* opaque: the two solves cannot be merged */           \
        double d2 = g_solve<GL, NM>(a, orig, dinv, n, gl, bb);                               \
        asm volatile("" : "+v"(d2));                                                         \
        delta[0] = d2;                                                                       \
    } while (0)
#else
#define BR_XG_AFTER_SOLVE()
#endif
#if defined(BR_EXP_GDUP) && BR_EXP_GDUP == 3
#define BR_XG_AFTER_JAC()                                                                    \
    do {                                                                                     \
        asm volatile("" ::: "memory");                                                       \
        g_jac_cols<GL>(tb, sp, kd, fod, skd, T, Asv, Asv_th, gl, jst);                       \
    } while (0)
#else
#define BR_XG_AFTER_JAC()
#endif
#if defined(BR_EXP_GDUP) && BR_EXP_GDUP == 4
#define BR_XG_AFTER_LU()                                                                     \
    do {                                                                                     \
        asm volatile("" ::: "memory");                                                       \
        lu_fail = g_lu<GL, NM>(jr, C->gamma, n, gl, a, orig, dinv);                          \
    } while (0)
#else
#define BR_XG_AFTER_LU()
#endif

#if defined(BR_EXP_DUP) && BR_EXP_DUP == 1
#define BR_X_AFTER_RHS()                                                \
    do {                                                                \
        asm volatile("" ::: "memory");                                  \
        rhs<CPL>(M, tb, S, T, Asv, Asv_th, y, lane, p_last, f);         \
    } while (0)
#else
#define BR_X_AFTER_RHS()
#endif

#if defined(BR_EXP_DUP) && BR_EXP_DUP == 3
#define BR_X_AFTER_JAC()                                                \
    do {                                                                \
        asm volatile("" ::: "memory");                                  \
        jacobian<CPL>(M, tb, S, T, Asv, Asv_th, y, lane, Jsave, jscr);  \
    } while (0)
#else
#define BR_X_AFTER_JAC()
#endif

#if defined(BR_EXP_DUP) && BR_EXP_DUP == 2
#define BR_X_AFTER_SOLVE()                                              \
    do {                                                                \
        asm volatile("" ::: "memory");                                  \
        double d2 = lu_solve<NMAX>(LUsave, n, lane, perm[0], b[0], scr); \
        asm volatile("" : "+v"(d2));                                    \
        delta[0] = d2;                                                  \
    } while (0)
#else
#define BR_X_AFTER_SOLVE()
#endif

#if defined(BR_EXP_VALU)
#define BR_X_AFTER_ITER()                                                                   \
    do {                                                                                    \
        double acc[8];                                                                      \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                     \
            acc[i] = delta[0] + i;                                                          \
            asm volatile("" : "+v"(acc[i]));                                                \
        }                                                                                   \
        _Pragma("unroll") for (int i = 0; i < BR_EXP_VALU / 8; ++i)                         \
            _Pragma("unroll") for (int j = 0; j < 8; ++j)                                   \
                asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(acc[j]));                    \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(acc[i]));       \
    } while (0)
#elif defined(BR_EXP_MEM)
#define BR_X_AFTER_ITER()                                                                   \
    do {                                                                                    \
        const BR_GLOBAL double* jg = launder((const double*)Jsave);                         \
        double d[BR_EXP_MEM];                                                               \
        _Pragma("unroll") for (int i = 0; i < BR_EXP_MEM; ++i) d[i] = jg[i * 64 * CPL + lane]; \
        _Pragma("unroll") for (int i = 0; i < BR_EXP_MEM; ++i) asm volatile("" ::"v"(d[i]));  \
    } while (0)
#else
#define BR_X_AFTER_ITER()
#endif
