// coop_lusolve.hip -- VERDICT r05 item 3, measured at the level of the phases it changes: can a
// cooperative engine (one GRI reactor per 4-wave workgroup, the LU factors held in the four waves'
// registers) run the Newton linear algebra faster than the integrator's wavefront form at the same
// 16 waves/CU? The unit of work is one reactor's factorization of I - gamma J (n = 53, NMAX = 56)
// followed by `nsolve` triangular solves, the integrator's ratio (~9.2 solves per factorization,
// GRI C3), repeated `reps` times per reactor with the rows entering each LU in the previous one's
// pivot order, as in k_integrate.
//
//   k_base : the integrator's code itself (brhip_device.hpp lu_factor<56> / lu_solve<56>): one
//            reactor per wave, four per 256-thread workgroup, J and the factors in the reactor's
//            global workspace slot (the ~23 KB factor matrix re-read from the L2 / fabric by every
//            solve).
//   k_coop : one reactor per 256-thread workgroup. Wave w holds columns 16w .. 16w+15 of every row
//            (lane = row, as in lu_factor) in registers for the reactor's whole life. LU step k:
//            the owner wave of column k runs lu_rl_steps' pivot search (fast path included),
//            publishes the multipliers l (one per lane), the pivot lane and 1/pivot through LDS,
//            one s_barrier, then every wave applies the rank-1 update to its live columns with the
//            same FMA as lu_rl_steps (fma(-u_pj, l_i, a_ij), u_pj by v_readlane). The solves are the
//            integrator's DPP sweeps (tri_block_dpp: v_fmac_f64_dpp row_newbcast inside 16-lane
//            rows, one LDS copy per block) with the factor operands taken from registers: block B
//            is run by wave B and the right-hand side is handed to the next block's wave through
//            LDS (one s_barrier per block). No factor byte leaves the CU.
//
// Both produce bit-identical solutions (same pivots, multipliers, FMA order per element; checked
// by scripts/exp_coop.py against each other and against numpy). Occupancy is capped at 16 waves/CU
// for both with dynamic LDS (4 workgroups per CU), the integrator's k_integrate<56> residency:
// 16 reactors per CU for k_base, 4 for k_coop. A second coop launch without the cap shows what
// the phases would gain if the rest of a cooperative engine's state fitted in 64 VGPRs per wave.
// Not part of libbrhip.so.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <type_traits>

#include "../../include/brhip.h"
#include "../../batchreactor.jl_amd/csrc/brhip_device.hpp"

using namespace brhip;

namespace {

constexpr int NMAX = 56;
constexpr int NB = (NMAX + 15) / 16;   // 16-column blocks = waves of a coop workgroup
constexpr size_t SLOT = (size_t)NMAX * 64 + (size_t)NMAX * NMAX + 64;   // J (column-major) + factors + D^-1

// ---------------------------------------------------------------------------------------------
// baseline: the integrator's LU and solve, one reactor per wave
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_base(int N, int n, const double* __restrict__ J, int nj,
                                              const double* __restrict__ g, const double* __restrict__ b, double* ws,
                                              int reps, int nsolve, double* __restrict__ x, double* __restrict__ chk,
                                              int* __restrict__ fail) {
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int rid = blockIdx.x * 4 + w;
    if (rid >= N) return;   // no workgroup barrier below
    double* Jt = ws + (size_t)rid * SLOT;
    double* LU = Jt + NMAX * 64;
    const double* Jr = J + (size_t)(rid % nj) * n * n;
    for (int j = 0; j < NMAX; ++j) Jt[j * 64 + lane] = (lane < n && j < n) ? Jr[lane * n + j] : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    const double gm = g[rid];
    const double bv = lane < n ? b[(size_t)rid * n + lane] : 0.0;
    int perm = lane, f = 0;
    double acc = 0.0, r = 0.0;
    for (int rep = 0; rep < reps; ++rep) {
        f |= lu_factor<NMAX>(Jt, LU, gm, n, lane, perm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wave_sync();
        for (int s = 0; s < nsolve; ++s) {
            r = lu_solve<NMAX>(LU, n, lane, perm, bv * (double)(1 + s), (LDSd*)(sh + 64 * w));
            acc += r;
        }
    }
    if (lane < n) { x[(size_t)rid * n + lane] = r; chk[(size_t)rid * n + lane] = acc; }
    if (lane == 0) fail[rid] = f;
}

// ---------------------------------------------------------------------------------------------
// cooperative: one reactor per workgroup of NB = 4 waves, factors in registers
// ---------------------------------------------------------------------------------------------
struct CoopLds {
    double l[2][64];     // multipliers of step k (double-buffered on k & 1)
    double rinv[2];      // 1 / pivot
    int p[2];            // pivot lane
    double rhs[64];      // right-hand side handed from one block's wave to the next
    double x64[NB][64];  // per-wave scratch of the DPP sweeps (tri_block_dpp's x64)
    // PANEL form: a block's 16 steps published at once (double-buffered on the block)
    double pl[2][16][64];
    double prinv[2][16];
    int pp[2][16];
};

// compile-time loop: f(std::integral_constant<int, K>) for K = B0 .. E-1
template <int B0, int E, class F>
__device__ __forceinline__ void cfor(F&& f) {
    if constexpr (B0 < E) {
        f(std::integral_constant<int, B0>{});
        cfor<B0 + 1, E>(f);
    }
}

// rank-1 update of this wave's columns J0 .. 15 (compile time) by step k's pivot lane p and multipliers l
template <int J0>
__device__ __forceinline__ void coop_update(double (&a)[16], int p, double l) {
#pragma unroll
    for (int jj = J0; jj < 16; ++jj) a[jj] = fma(-bcast_lu(a[jj], p), l, a[jj]);
}

// the integrator's DPP block sweep (tri_block_dpp) for block B with the factor operands f[] from
// registers; r = this lane's right-hand side entry, x64 = the wave's LDS scratch
template <bool FWD, int B>
__device__ __forceinline__ void coop_block(double& r, const double (&f)[16], LDSd* x64, int lane) {
    constexpr int CW = (16 * B + 16 > NMAX) ? NMAX - 16 * B : 16;
    dpp_diag<FWD, CW, 1 << B, 0>(r, f);
    constexpr int ROWS = FWD ? (0xF << (B + 1)) & 0xF : (1 << B) - 1;
    if constexpr (ROWS != 0) {
        asm volatile("s_nop 1");
        x64[lane] = r;
        wave_sync();
        const double xv = x64[16 * B + (lane & 15)];
        dpp_off<FWD, CW, ROWS, 0>(r, xv, f);
        wave_sync();
    }
    asm volatile("s_nop 1");
}

template <int B>
__device__ __forceinline__ void coop_fwd(double& r, const double (&fl)[16], CoopLds* S, int w, int lane) {
    if constexpr (B < NB) {
        if (w == B) {
            if (B > 0) r = S->rhs[lane];
            coop_block<true, B>(r, fl, (LDSd*)S->x64[w], lane);
            if (B + 1 < NB) S->rhs[lane] = r;
        }
        if (B + 1 < NB) __syncthreads();
        coop_fwd<B + 1>(r, fl, S, w, lane);
    }
}
template <int B>
__device__ __forceinline__ void coop_bwd(double& r, const double (&fu)[16], CoopLds* S, int w, int lane) {
    if constexpr (B >= 0) {
        if (w == B) {
            if (B + 1 < NB) r = S->rhs[lane];
            coop_block<false, B>(r, fu, (LDSd*)S->x64[w], lane);
            if (B > 0) S->rhs[lane] = r;
        }
        if (B > 0) __syncthreads();
        coop_bwd<B - 1>(r, fu, S, w, lane);
    }
}

template <bool PANEL>
__global__ __launch_bounds__(256) void k_coop(int N, int n, const double* __restrict__ J, int nj,
                                              const double* __restrict__ g, const double* __restrict__ b, double* ws,
                                              int reps, int nsolve, double* __restrict__ x, double* __restrict__ chk,
                                              int* __restrict__ fail) {
    extern __shared__ __attribute__((aligned(16))) double sh[];
    CoopLds* S = reinterpret_cast<CoopLds*>(sh);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int rid = blockIdx.x;
    if (rid >= N) return;   // whole workgroup
    // J in the same column-major slot as k_base (wave w stages columns 16w..)
    double* Jt = ws + (size_t)rid * SLOT;
    const double* Jr = J + (size_t)(rid % nj) * n * n;
    for (int j = 16 * w; j < 16 * w + 16 && j < NMAX; ++j) Jt[j * 64 + lane] = (lane < n && j < n) ? Jr[lane * n + j] : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    const double gm = g[rid];
    const double bv = lane < n ? b[(size_t)rid * n + lane] : 0.0;
    const int tr = lane & 15, row = lane >> 4;
    int perm = lane, f = 0;
    double acc = 0.0, r = 0.0;
    double fl[16], fu[16];   // this wave's 16 factor columns, masked for the forward / backward sweep
    for (int rep = 0; rep < reps; ++rep) {
        // ---- rows in the previous factorization's pivot order (perm), as lu_factor
        const int prow = perm;
        const bool act = lane < n;
        double a[16];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int col = 16 * w + jj;
            const double jv = (act && col < NMAX) ? Jt[col * 64 + prow] : 0.0;
            a[jj] = ((col == prow) ? 1.0 : 0.0) - gm * jv;
        }
        int pstep = act ? -1 : 1024;
        double dinv = 0.0;
        int fl_k = 0;
        if constexpr (!PANEL) {
            // one s_barrier per step: the owner of column k publishes step k, every wave updates
#pragma unroll 1
            for (int B = 0; B < NB; ++B) {
                cfor<0, 16>([&](auto kc) {
                    constexpr int kk = decltype(kc)::value;
                    const int k = 16 * B + kk;
                    if (k < n) {
                        const bool cand = pstep < 0;
                        double l = 0.0;
                        if (w == B) {   // owner of column k: lu_rl_steps' pivot search and column k of the factors
                            const double ak = a[kk];
                            const double akk = bcast(ak, k);
                            const bool kcand = (__ballot(cand) >> k) & 1ull;
                            const bool fast = kcand && __ballot(cand && lane != k && !(fabs(ak) < fabs(akk))) == 0;
                            const int p = fast ? k : pivot_lane(ak, cand ? 0x7fffffffu : 0u, prow);
                            const double piv = fast ? akk : bcast(ak, p);
                            const double rinv = 1.0 / piv;
                            const bool isp = lane == p;
                            const bool rem = cand && !isp;
                            l = rem ? ak * rinv : 0.0;
                            a[kk] = rem ? l : (cand ? 0.0 : ak * dinv);
                            S->l[k & 1][lane] = l;
                            if (lane == 0) { S->p[k & 1] = p; S->rinv[k & 1] = rinv; }
                        }
                        __syncthreads();
                        const int p = S->p[k & 1];
                        const double rinv = S->rinv[k & 1];
                        if (w != B) l = S->l[k & 1][lane];
                        if (lane == p) { pstep = k; dinv = rinv; }
                        if (!fl_k && (rinv == INFINITY || rinv == -INFINITY)) fl_k = k + 1;   // zero pivot
                        if (w == B) coop_update<(kk + 1 < 16 ? kk + 1 : 16)>(a, p, l);
                        else if (w > B) coop_update<0>(a, p, l);
                    }
                });
            }
        } else {
            // one s_barrier per block: wave B factors its 16 columns alone (right-looking inside the
            // panel, the same per-element FMA sequence), publishes the block's 16 steps, then the
            // waves to its right apply them in step order (every element still receives its updates
            // in step order: bit-identical to the per-step form and to lu_factor)
#pragma unroll 1
            for (int B = 0; B < NB; ++B) {
                const int bb = B & 1;
                if (w == B) {
                    cfor<0, 16>([&](auto kc) {
                        constexpr int kk = decltype(kc)::value;
                        const int k = 16 * B + kk;
                        if (k < n) {
                            const bool cand = pstep < 0;
                            const double ak = a[kk];
                            const double akk = bcast(ak, k);
                            const bool kcand = (__ballot(cand) >> k) & 1ull;
                            const bool fast = kcand && __ballot(cand && lane != k && !(fabs(ak) < fabs(akk))) == 0;
                            const int p = fast ? k : pivot_lane(ak, cand ? 0x7fffffffu : 0u, prow);
                            const double piv = fast ? akk : bcast(ak, p);
                            const double rinv = 1.0 / piv;
                            const bool isp = lane == p;
                            const bool rem = cand && !isp;
                            const double l = rem ? ak * rinv : 0.0;
                            a[kk] = rem ? l : (cand ? 0.0 : ak * dinv);
                            S->pl[bb][kk][lane] = l;
                            if (lane == 0) { S->pp[bb][kk] = p; S->prinv[bb][kk] = rinv; }
                            if (isp) { pstep = k; dinv = rinv; }
                            if (!fl_k && piv == 0.0) fl_k = k + 1;
                            coop_update<(kk + 1 < 16 ? kk + 1 : 16)>(a, p, l);
                        }
                    });
                }
                __syncthreads();
                if (w != B) {
                    cfor<0, 16>([&](auto kc) {
                        constexpr int kk = decltype(kc)::value;
                        const int k = 16 * B + kk;
                        if (k < n) {
                            const int p = S->pp[bb][kk];
                            const double rinv = S->prinv[bb][kk];
                            if (lane == p) { pstep = k; dinv = rinv; }
                            if (!fl_k && (rinv == INFINITY || rinv == -INFINITY)) fl_k = k + 1;
                            if (w > B) coop_update<0>(a, p, S->pl[bb][kk][lane]);
                        }
                    });
                }
            }
        }
        f |= fl_k;
        // ---- rows into step order (lu_factor's gather), padding columns to zero
        if (__ballot(act && pstep != lane) != 0) {
            const int q = pivot_perm(pstep, lane, n);
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) a[jj] = lane_pull(a[jj], q);
            dinv = lane_pull(dinv, q);
            perm = __builtin_amdgcn_ds_bpermute(q * 4, prow);
        } else {
            perm = prow;
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const double v = (16 * w + jj < n) ? a[jj] : 0.0;
            const bool diag_row = row == w;   // this wave's diagonal 16 x 16 block
            fl[jj] = (diag_row && tr < jj) ? 0.0 : v;   // L below the diagonal (forward)
            fu[jj] = (diag_row && tr > jj) ? 0.0 : v;   // U' above it (backward)
        }
        __syncthreads();
        // ---- the solves: P b, forward over blocks 0..NB-1, D^-1, backward over NB-1..0
        for (int s = 0; s < nsolve; ++s) {
            if (w == 0) r = lane_pull(lane < n ? bv * (double)(1 + s) : 0.0, perm);
            coop_fwd<0>(r, fl, S, w, lane);
            if (w == NB - 1) r *= dinv;
            __syncthreads();
            coop_bwd<NB - 1>(r, fu, S, w, lane);
            if (w == 0) { r = (lane < n) ? r : 0.0; acc += r; }
            __syncthreads();
        }
    }
    if (w == 0) {
        if (lane < n) { x[(size_t)rid * n + lane] = r; chk[(size_t)rid * n + lane] = acc; }
        if (lane == 0) fail[rid] = f;
    }
}

}  // namespace

extern "C" {
// mode 0: k_base; k_coop with one barrier per 16-column block: 1 capped at 4 workgroups per CU
// (16 waves/CU), 2 uncapped; k_coop with one barrier per LU step: 3 capped, 4 uncapped.
// J: nj matrices n x n row-major (reactor r uses J[r % nj]); g[N], b[N][n]. Outputs x, chk [N][n],
// fail[N]; *ms = kernel time of the timed launch (one untimed launch first). Returns 0 or a HIP error.
int coop_run(int mode, int N, int n, const double* J, int nj, const double* g, const double* b, int reps, int nsolve,
             double* x, double* chk, int* fail, double* ms, int* vgprs) {
    if (n > NMAX || n < 1 || N < 1 || mode < 0 || mode > 4) return -1;
    double *dJ, *dg, *db, *dws, *dx, *dc;
    int* df;
    hipError_t e = hipSuccess;
    auto ck = [&](hipError_t v) { if (e == hipSuccess) e = v; };
    ck(hipMalloc(&dJ, sizeof(double) * nj * n * n));
    ck(hipMalloc(&dg, sizeof(double) * N));
    ck(hipMalloc(&db, sizeof(double) * N * n));
    ck(hipMalloc(&dws, sizeof(double) * SLOT * N));
    ck(hipMalloc(&dx, sizeof(double) * N * n));
    ck(hipMalloc(&dc, sizeof(double) * N * n));
    ck(hipMalloc(&df, sizeof(int) * N));
    if (e != hipSuccess) return (int)e;
    ck(hipMemcpy(dJ, J, sizeof(double) * nj * n * n, hipMemcpyHostToDevice));
    ck(hipMemcpy(dg, g, sizeof(double) * N, hipMemcpyHostToDevice));
    ck(hipMemcpy(db, b, sizeof(double) * N * n, hipMemcpyHostToDevice));
    // 4 workgroups per CU: 40 KB of LDS each (the kernels use 2 KB / 5.6 KB of it)
    const size_t cap = 40 * 1024;
    const bool capped = mode == 0 || mode == 1 || mode == 3;
    const size_t lds = capped ? cap : sizeof(CoopLds);
    const void* fn = mode == 0 ? (const void*)k_base : (mode <= 2 ? (const void*)k_coop<true> : (const void*)k_coop<false>);
    const int grid = mode == 0 ? (N + 3) / 4 : N;
    hipFuncAttributes at;
    if (hipFuncGetAttributes(&at, fn) == hipSuccess && vgprs) *vgprs = at.numRegs;
    hipEvent_t e0, e1;
    ck(hipEventCreate(&e0));
    ck(hipEventCreate(&e1));
    for (int it = 0; it < 2 && e == hipSuccess; ++it) {
        ck(hipEventRecord(e0, 0));
        if (mode == 0)
            hipLaunchKernelGGL(k_base, dim3(grid), dim3(256), lds, 0, N, n, dJ, nj, dg, db, dws, reps, nsolve, dx, dc, df);
        else if (mode <= 2)
            hipLaunchKernelGGL(k_coop<true>, dim3(grid), dim3(256), lds, 0, N, n, dJ, nj, dg, db, dws, reps, nsolve, dx, dc, df);
        else
            hipLaunchKernelGGL(k_coop<false>, dim3(grid), dim3(256), lds, 0, N, n, dJ, nj, dg, db, dws, reps, nsolve, dx, dc, df);
        ck(hipGetLastError());
        ck(hipEventRecord(e1, 0));
        ck(hipEventSynchronize(e1));
    }
    float t = 0.f;
    ck(hipEventElapsedTime(&t, e0, e1));
    *ms = t;
    ck(hipMemcpy(x, dx, sizeof(double) * N * n, hipMemcpyDeviceToHost));
    ck(hipMemcpy(chk, dc, sizeof(double) * N * n, hipMemcpyDeviceToHost));
    ck(hipMemcpy(fail, df, sizeof(int) * N, hipMemcpyDeviceToHost));
    (void)hipFree(dJ); (void)hipFree(dg); (void)hipFree(db); (void)hipFree(dws); (void)hipFree(dx); (void)hipFree(dc); (void)hipFree(df);
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    return (int)e;
}
}
