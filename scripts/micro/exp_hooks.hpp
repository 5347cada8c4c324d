// exp_hooks.hpp -- diagnostic-only experiment hooks for k_integrate (never in the product build).
// Build a variant library with
//   hipcc ... -DBR_EXPERIMENT_HOOKS='"../../scripts/micro/exp_hooks.hpp"' -DBR_EXP_DUP=1 ... brhip.hip
// (scripts/pmc_ab.sh). The macros expand inside k_integrate's Newton loop and use its locals.
//   BR_EXP_DUP=1/2/3 : the RHS / the linear solve / the Jacobian evaluated twice (SQ_INSTS_VALU of
//                      one phase = the difference to the plain build)
//   BR_EXP_VALU=K    : K independent dummy fp64 FMAs per Newton iteration (VALU-issue sensitivity)
//   BR_EXP_MEM=K     : K columns (512 B each) of the saved J re-read per Newton iteration (memory-
//                      side sensitivity)
#pragma once

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
