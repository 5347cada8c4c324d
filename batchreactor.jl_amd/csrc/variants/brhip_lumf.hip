// brhip_lumf.hip -- VARIANT library libbrhip_lumf.so (not the product): the blocked LU of I - gamma J
// with fp64 MFMA trailing updates (v_mfma_f64_16x16x4f64), north_star: "fp64 MFMA only for the LU
// trailing update, and only if rocprof shows it beats VALU at that matrix size". Built into the
// integrator and measured in round 4 (profiles/r04_lu_mfma_ab.json: 88.8k / 92.0k vs 110.5k GRI
// reactors/s for the row-per-lane VALU LU), so the product keeps the VALU LU; this library keeps the
// MFMA LU built and tested (tests/test_gpu_parity.py::test_batched_lu_solve_mfma) against numpy and
// the lane-level emulation (scripts/emu/). Same solve (lu_solve) as the product.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <vector>

#include "../../../include/brhip.h"
#include "../brhip_device.hpp"

using namespace brhip;

namespace brhip {
// ------------------------------------------------------------------------------------
// Blocked LU for 32 < NMAX <= 64 (CPL = 1) with the trailing update on the fp64 matrix pipe
// (v_mfma_f64_16x16x4f64). Same pivoting rule, multipliers and stored factor form as lu_factor
// (SUNDIALS denseGETRF semantics; rows loaded in the previous pivot order; factors in M, step
// order after the gather); the trailing update is reassociated (bands, not bits, against the
// unblocked form).
//
// Panels of 16 columns, factored right-looking row-per-lane (pivot search and readlane
// broadcasts as lu_rl_steps). Alongside, each panel tracks E' (64 x 16, row per lane):
// E = the same elimination applied to [0; I] on the panel's pivot rows (E[p_j] = (L11^-1)_j,
// E[r] = -(L21 L11^-1)_r for rows not yet pivoted, 0 for rows pivoted earlier), E' = E - the
// pivot entries (E'[p_j][j] = 0). Then the whole right-looking update of the trailing columns by
// the panel's 16 steps is one GEMM over ALL rows, no mask:
//     X <- X + E' X[piv]   (pivot rows get L11^-1 X[piv] = U12, the other rows X - L21 U12).
// It runs transposed, X^T (cols x rows) += X[piv]^T (cols x 16) E'^T (16 x rows), so that the
// accumulator layout (col = 16c + (lane >> 4) + 4 i, row = 16t + (lane & 15)) addresses the
// column-major factor matrix M in 128-B row segments, and the trailing matrix lives in M itself:
// column j of X sits where factor column j will be written, and panel p reads its columns from
// there before its steps overwrite them with factors. Operands: A = X[piv]^T gathered from M
// (lane: col 16c + (lane & 15), k = 4s + (lane >> 4)); B = E'^T through LDS scratch (one 4-column
// chunk of E' at a time, 2 KB). Row tiles whose rows were all pivoted before the panel have E' = 0
// and are skipped (with the rows in the previous pivot order that is every earlier tile).
// ------------------------------------------------------------------------------------
typedef double d4v __attribute__((ext_vector_type(4)));

#ifndef BR_LU_PW
#define BR_LU_PW 8   // panel width of lu_factor_mf (8 or 16)
#endif

// one panel: columns c0 .. c0+PW-1 right-looking in a[] (row per lane), factor columns stored to
// M as each step completes, E' in e[] (WITH_E), the steps' pivot lanes in piv[]
template <int FR, int PW, bool WITH_E>
__device__ __forceinline__ void lu_mf_panel(double (&a)[PW], double (&e)[PW], int (&piv)[PW], int c0, int nlive,
                                            int lane, int prow, int& pstep, double& dinv, int& fail,
                                            __amdgpu_buffer_rsrc_t rs) {
    const unsigned fo8 = (lane < FR) ? (unsigned)lane * 8u : LU_OOB;
#pragma unroll
    for (int kk = 0; kk < PW; ++kk) {
        if (kk < nlive) {
            const int k = c0 + kk;
            const bool cand = pstep < 0;
            const int p = pivot_lane(a[kk], cand ? 0x7fffffffu : 0u, prow);
            piv[kk] = p;
            const double pv = bcast(a[kk], p);
            if (pv == 0.0 && !fail) fail = k + 1;
            const double rinv = 1.0 / pv;
            const bool isp = (lane == p);
            const bool rem = cand && !isp;
            const double l = rem ? a[kk] * rinv : 0.0;
            const double fv = rem ? l : (cand ? 0.0 : a[kk] * dinv);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, fv), rs, fo8, k * (FR * 8), 0);
            if (isp) { pstep = k; dinv = rinv; }
            if constexpr (WITH_E) {
#pragma unroll
                for (int j = 0; j < kk; ++j) e[j] = fma(-bcast_lu(e[j], p), l, e[j]);
                e[kk] = -l;
            }
            int nl = nlive;   // (opaque per step: scalar tests, see lu_factor)
            asm volatile("" : "+s"(nl));
#pragma unroll
            for (int j = kk + 1; j < PW; ++j)
                if (j < nl) a[j] = fma(-bcast_lu(a[j], p), l, a[j]);
        }
    }
}

template <int NMAX, int STOP = (1 << 20)>   // STOP: return after that panel's trailing update (debug kernel)
__device__ __forceinline__ int lu_factor_mf(const double* __restrict__ J_, double* __restrict__ ws, LDSd* scr,
                                            double gamma, int n, int lane, int& perm_io) {
    static_assert(NMAX > 32 && NMAX <= 64 && NMAX % 8 == 0, "lu_factor_mf: NMAX");
    constexpr int PW = BR_LU_PW;             // panel width
    constexpr int KS = PW / 4;               // MFMA k-steps per panel
    constexpr int FR = NMAX;                 // factor column stride (rows)
    constexpr int NRT = (NMAX + 15) / 16;    // row tiles
    constexpr int MAXCT = (NMAX - PW + 15) / 16;   // column tiles of the largest trailing block
    static_assert(PW == 8 || PW == 16, "lu_factor_mf: PW");
    const BR_GLOBAL double* J = launder(J_);
    BR_GLOBAL double* wsg = launder(ws);
    const LUWs F{wsg, wsg + NMAX * FR};
    const __amdgpu_buffer_rsrc_t rs = lu_rsrc(wsg, NMAX * FR);
    lane = launder_v(lane);
    n = launder_s(n);
    // the trailing block's pivot-row operand through a buffer of n columns: padding columns read 0
    const __amdgpu_buffer_rsrc_t rsn = lu_rsrc(wsg, n * FR);
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc((void*)J, (short)0, n * (WAVE * 8), 0x00020000);
    const int prow = launder_v(perm_io);
    const bool act = lane < n;
    const int g = lane >> 4, m = lane & 15;
    int pstep = act ? -1 : 1024;
    double dinv = 0.0;
    int fail = 0;
    const int np = (n + PW - 1) / PW;
    const unsigned fo8 = (lane < FR) ? (unsigned)lane * 8u : LU_OOB;
#pragma unroll 1
    for (int p = 0; p + 1 < np; ++p) {
        BR_SUB_T(lt0);
        const int c0 = PW * p;
        const unsigned long long live = __ballot(pstep < 0);   // rows not pivoted before this panel
        double a[PW], e[PW];
        int piv[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) e[j] = 0.0;
        if (p == 0) {
            const unsigned jo8 = act ? (unsigned)prow * 8u : LU_OOB;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const double jv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, jo8 + j * (WAVE * 8), 0, 0));
                a[j] = ((j == prow) ? 1.0 : 0.0) - gamma * jv;
            }
        } else {
#pragma unroll
            for (int j = 0; j < PW; ++j)
                a[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, fo8 + j * (FR * 8), c0 * (FR * 8), 0));
        }
        lu_mf_panel<FR, PW, true>(a, e, piv, c0, PW, lane, prow, pstep, dinv, fail, rs);
        // ---- E'^T operands through LDS, one 4-column chunk at a time: lane l of operand (t, s)
        // holds E'[16t + (l & 15)][4s + (l >> 4)]
        double bo[NRT][KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int q = 0; q < 4; ++q) scr[4 * lane + q] = e[4 * s + q];
            wave_sync();
#pragma unroll
            for (int t = 0; t < NRT; ++t) bo[t][s] = scr[4 * (16 * t + m) + g];
            wave_sync();
        }
        // A operand rows: the pivot row of step 4s + (lane >> 4); in the first panel the trailing
        // columns are still I - gamma J, read from J at the pivot's original row (aor)
        unsigned ao8[KS];
        int aor[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int pr = g == 0 ? piv[4 * s] : g == 1 ? piv[4 * s + 1] : g == 2 ? piv[4 * s + 2] : piv[4 * s + 3];
            if (p == 0) {
                aor[s] = __builtin_amdgcn_ds_bpermute(4 * pr, prow);
                ao8[s] = (unsigned)aor[s] * 8u + (unsigned)m * (WAVE * 8);
            } else {
                ao8[s] = (unsigned)(m * FR + pr) * 8u;
            }
        }
        // first trailing update: X = I - gamma J straight from the saved J; position 16t + m holds
        // original row orow[t] (-1: none; its J offset out of range)
        unsigned jt8[NRT];
        int orow[NRT];
        if (p == 0) {
#pragma unroll
            for (int t = 0; t < NRT; ++t) {
                orow[t] = __builtin_amdgcn_ds_bpermute(4 * (16 * t + m), act ? prow : -1);
                jt8[t] = orow[t] >= 0 ? (unsigned)orow[t] * 8u + (unsigned)g * (WAVE * 8) : LU_OOB;
            }
        }
        // accumulator rows 16t + m (out of range for rows >= FR)
        unsigned rb8[NRT];
#pragma unroll
        for (int t = 0; t < NRT; ++t) rb8[t] = (16 * t + m < FR) ? (unsigned)(g * FR + 16 * t + m) * 8u : LU_OOB;
        BR_SUB_ADD(0, lt0);
        BR_SUB_T(lt1);
        // ---- trailing update: columns c0 + PW .. n-1 in tiles of 16
        const int cs = c0 + PW;
#pragma unroll
        for (int ct = 0; ct < MAXCT; ++ct) {
            const int cb = cs + 16 * ct;
            if (cb < n) {
                double ao[KS];
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    if (p == 0) {
                        const double jv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, ao8[s] + cb * (WAVE * 8), 0, 0));
                        ao[s] = ((aor[s] == cb + m) ? 1.0 : 0.0) - gamma * jv;
                    } else {
                        ao[s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsn, ao8[s] + cb * (FR * 8), 0, 0));
                    }
                }
                d4v x[NRT];
#pragma unroll
                for (int t = 0; t < NRT; ++t) {
                    if ((live >> (16 * t)) & 0xffffull) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int cc = cb + 4 * i;   // columns cc .. cc + 3 (lane groups)
                            x[t][i] = 0.0;
                            if (cc < NMAX) {
                                if (p == 0) {
                                    const double jv = __builtin_bit_cast(double,
                                        __builtin_amdgcn_raw_buffer_load_b64(rj, jt8[t] + cc * (WAVE * 8), 0, 0));
                                    x[t][i] = ((orow[t] == cc + g) ? 1.0 : 0.0) - gamma * jv;
                                } else {
                                    x[t][i] = __builtin_bit_cast(double,
                                        __builtin_amdgcn_raw_buffer_load_b64(rs, rb8[t], cc * (FR * 8), 0));
                                }
                            }
                        }
                    }
                }
#pragma unroll
                for (int t = 0; t < NRT; ++t) {
                    if ((live >> (16 * t)) & 0xffffull) {
#pragma unroll
                        for (int s = 0; s < KS; ++s) x[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ao[s], bo[t][s], x[t], 0, 0, 0);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int cc = cb + 4 * i;
                            // (through a scalar copy: __builtin_bit_cast of a vector element reads element 0)
                            const double xv = x[t][i];
                            if (cc < NMAX)
                                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, xv), rs, rb8[t], cc * (FR * 8), 0);
                        }
                    }
                }
            }
        }
        BR_SUB_ADD(1, lt1);
        if (p == STOP) {
            perm_io = prow;
            return 0;
        }
    }
    {   // last panel: no trailing columns, no E'
        BR_SUB_T(lt0);
        const int c0 = PW * (np - 1);
        double a[PW], e[PW];
        int piv[PW];
        const int nlive = n - c0;
        if (np == 1) {
            const unsigned jo8 = act ? (unsigned)prow * 8u : LU_OOB;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const double jv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rj, jo8 + j * (WAVE * 8), 0, 0));
                a[j] = ((j == prow) ? 1.0 : 0.0) - gamma * jv;
            }
        } else {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                a[j] = 0.0;
                if (j < nlive)
                    a[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, fo8 + j * (FR * 8), c0 * (FR * 8), 0));
            }
        }
        lu_mf_panel<FR, PW, false>(a, e, piv, c0, nlive, lane, prow, pstep, dinv, fail, rs);
        BR_SUB_ADD(0, lt0);
    }
    BR_SUB_T(lt2);
    constexpr int CH = 8, NC = NMAX / CH;
    int perm;
    if (__ballot(act && pstep != lane) == 0) {
        // pivots in lane order: M is in step order already; padding columns n..NMAX-1 zeroed
        perm = prow;
        if (lane < FR)
            for (int c = n; c < NMAX; ++c) F.M[c * FR + lane] = 0.0;
        F.D[lane] = dinv;
    } else {
        // rows into step order, in place (as lu_factor; columns >= n: zeros)
        const int q = pivot_perm(pstep, lane, n);
        perm = __builtin_amdgcn_ds_bpermute(q * 4, prow);
        double gb[2][CH];
        auto gather = [&](double (&v)[CH], int c) {
#pragma unroll
            for (int i = 0; i < CH; ++i) v[i] = F.M[min(c + i, n - 1) * FR + min(q, FR - 1)];
        };
        gather(gb[0], 0);
#pragma unroll
        for (int t = 0; t < NC; ++t) {
            if (t + 1 < NC) gather(gb[(t + 1) & 1], (t + 1) * CH);
            __builtin_amdgcn_sched_barrier(0);
            if (lane < FR) {
#pragma unroll
                for (int i = 0; i < CH; ++i) F.M[(t * CH + i) * FR + lane] = (t * CH + i < n) ? gb[t & 1][i] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        F.D[lane] = lane_pull(dinv, q);
    }
    BR_SUB_ADD(2, lt2);
    perm_io = perm;
    return fail;
}

}  // namespace brhip

namespace {
__host__ __device__ inline size_t lumf_ws_doubles(int nmax) { return (size_t)nmax * nmax + WAVE; }   // factors + D^-1


template <int NMAX>
__global__ __launch_bounds__(64) void k_lu_check_mf(int N, int n, const double* J, const double* g, const double* b,
                                                    double* x, double* ws, int* fail) {
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    __shared__ double prow[256];
    double* Jt = ws + (size_t)rid * (NMAX * WAVE + lumf_ws_doubles(NMAX));
    double* LU = Jt + NMAX * WAVE;
    for (int j = 0; j < NMAX; ++j) Jt[j * WAVE + lane] = (lane < n && j < n) ? J[((size_t)rid * n + lane) * n + j] : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    // twice, as in the integrator: natural row order first, then the first one's pivot order
    int perm = lane;
    int f = lu_factor_mf<NMAX>(Jt, LU, (LDSd*)prow, g[rid], n, lane, perm);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    f = lu_factor_mf<NMAX>(Jt, LU, (LDSd*)prow, g[rid], n, lane, perm);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    const double r = lu_solve<NMAX>(LU, n, lane, perm, lane < n ? b[(size_t)rid * n + lane] : 0.0, (LDSd*)prow);
    if (lane < n) x[(size_t)rid * n + lane] = r;
    if (lane == 0) fail[rid] = f;
}

// the factor workspace [M | D^-1] and the step -> row map after one (twice = 0) or two factorizations,
// for the lane-level emulation (scripts/emu/lu_mf_emu.py, cmp_lu.py)
template <int NMAX, int STOP>
__global__ __launch_bounds__(64) void k_lu_factor_dbg(int N, int n, const double* J, const double* g, int twice,
                                                      double* ws, double* Fout, int* pout) {
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    __shared__ double scr[256];
    double* Jt = ws + (size_t)rid * (NMAX * WAVE + lumf_ws_doubles(NMAX));
    double* LU = Jt + NMAX * WAVE;
    for (int j = 0; j < NMAX; ++j) Jt[j * WAVE + lane] = (lane < n && j < n) ? J[((size_t)rid * n + lane) * n + j] : 0.0;
    for (int i = lane; i < (int)lumf_ws_doubles(NMAX); i += 64) LU[i] = __builtin_nan("");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    int perm = lane;
    for (int r = 0; r <= twice; ++r) {
        lu_factor_mf<NMAX, STOP>(Jt, LU, (LDSd*)scr, g[rid], n, lane, perm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
    }
    for (int i = lane; i < (int)lumf_ws_doubles(NMAX); i += 64) Fout[(size_t)rid * lumf_ws_doubles(NMAX) + i] = LU[i];
    pout[(size_t)rid * 64 + lane] = perm;
}

struct DevScratch {   // device buffers freed on every exit path
    std::vector<void*> p;
    ~DevScratch() {
        for (void* q : p) (void)hipFree(q);
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

#define MFCHK(x) do { if ((x) != hipSuccess) return -20; } while (0)

// br_debug_lu_solve with the MFMA-blocked LU, 32 < n <= 64: factor I - gamma J (J[N][n][n] row-major)
// and solve one right-hand side per matrix; fail_out[N] = 0 or the zero-pivot step + 1
extern "C" int br_debug_lu_solve_mf(int N, int n, const double* J, const double* gamma, const double* b, double* x,
                                    int* fail_out) {
    if (N <= 0 || n <= 32 || n > 64) return -10;
    const int nmax = n <= 56 ? 56 : 64;
    double *dJ, *dg, *db, *dx, *dws;
    int* df;
    DevScratch S;
    MFCHK(S.alloc(&dJ, (size_t)N * n * n * 8));
    MFCHK(S.alloc(&dg, (size_t)N * 8));
    MFCHK(S.alloc(&db, (size_t)N * n * 8));
    MFCHK(S.alloc(&dx, (size_t)N * n * 8));
    MFCHK(S.alloc(&dws, (size_t)N * (nmax * WAVE + lumf_ws_doubles(nmax)) * 8));
    MFCHK(S.alloc(&df, (size_t)N * 4));
    MFCHK(hipMemcpy(dJ, J, (size_t)N * n * n * 8, hipMemcpyHostToDevice));
    MFCHK(hipMemcpy(dg, gamma, (size_t)N * 8, hipMemcpyHostToDevice));
    MFCHK(hipMemcpy(db, b, (size_t)N * n * 8, hipMemcpyHostToDevice));
    if (nmax == 56) hipLaunchKernelGGL(k_lu_check_mf<56>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    else hipLaunchKernelGGL(k_lu_check_mf<64>, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, db, dx, dws, df);
    MFCHK(hipGetLastError());
    MFCHK(hipMemcpy(x, dx, (size_t)N * n * 8, hipMemcpyDeviceToHost));
    MFCHK(hipMemcpy(fail_out, df, (size_t)N * 4, hipMemcpyDeviceToHost));
    return 0;
}

// factor workspace after one or two MFMA factorizations (stop: return after panel 0 / 1's update)
extern "C" int br_debug_lu_factor(int N, int n, const double* J, const double* gamma, int twice, int stop, double* F,
                                  int* perm) {
    if (N <= 0 || n <= 32 || n > 64) return -10;
    const int nmax = n <= 56 ? 56 : 64;
    const size_t lw = lumf_ws_doubles(nmax);
    double *dJ, *dg, *dws, *dF;
    int* dp;
    DevScratch S;
    MFCHK(S.alloc(&dJ, (size_t)N * n * n * 8));
    MFCHK(S.alloc(&dg, (size_t)N * 8));
    MFCHK(S.alloc(&dws, (size_t)N * (nmax * WAVE + lw) * 8));
    MFCHK(S.alloc(&dF, (size_t)N * lw * 8));
    MFCHK(S.alloc(&dp, (size_t)N * 64 * 4));
    MFCHK(hipMemcpy(dJ, J, (size_t)N * n * n * 8, hipMemcpyHostToDevice));
    MFCHK(hipMemcpy(dg, gamma, (size_t)N * 8, hipMemcpyHostToDevice));
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(N), dim3(64), 0, 0, N, n, dJ, dg, twice, dws, dF, dp); };
    if (nmax == 56) {
        if (stop == 0) go(k_lu_factor_dbg<56, 0>);
        else if (stop == 1) go(k_lu_factor_dbg<56, 1>);
        else go(k_lu_factor_dbg<56, (1 << 20)>);
    } else go(k_lu_factor_dbg<64, (1 << 20)>);
    MFCHK(hipGetLastError());
    MFCHK(hipMemcpy(F, dF, (size_t)N * lw * 8, hipMemcpyDeviceToHost));
    MFCHK(hipMemcpy(perm, dp, (size_t)N * 64 * 4, hipMemcpyDeviceToHost));
    return 0;
}
