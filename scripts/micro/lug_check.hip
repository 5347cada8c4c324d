// Lane-grid LU (lu_factor_g, brhip_lug.hpp) against the row-per-lane LU (lu_factor): bit-identical
// factor workspaces, pivot orders and failure codes on random ill-scaled Newton matrices (natural row
// order first, then the first factorization's pivot order, as in the integrator), plus a throughput
// micro-benchmark at the integrator's occupancy (16 waves/CU, <= 128 VGPRs). Not part of libbrhip.so.
//   ./lug_check [reps]
#include "../../include/brhip.h"
#include "../../batchreactor.jl_amd/csrc/brhip_device.hpp"
#include "../../batchreactor.jl_amd/csrc/brhip_lug.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace brhip;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } \
    } while (0)

__host__ __device__ static size_t lws(int nmax) { return (size_t)nmax * nmax + 64; }

template <int NMAX, int KIND>
__device__ __forceinline__ int factor(double* Jt, double* LU, LDSd* scr, double g, int n, int lane, int& perm) {
    if constexpr (KIND == 0) return lu_factor<NMAX>(Jt, LU, g, n, lane, perm);
    else return lu_factor_g<NMAX>(Jt, LU, scr, g, n, lane, perm);
}

// one matrix per 64-thread block; J[N][n][n] row-major
template <int NMAX, int KIND>
__global__ __launch_bounds__(64) void k_fac(int N, int n, const double* J, const double* g, int twice, double* ws,
                                            double* Fout, int* pout, int* fout) {
    const int rid = blockIdx.x;
    if (rid >= N) return;
    const int lane = threadIdx.x;
    __shared__ double scr[256];
    double* Jt = ws + (size_t)rid * (NMAX * 64 + lws(NMAX));
    double* LU = Jt + NMAX * 64;
    for (int j = 0; j < NMAX; ++j) Jt[j * 64 + lane] = (lane < n && j < n) ? J[((size_t)rid * n + lane) * n + j] : 0.0;
    for (size_t i = lane; i < lws(NMAX); i += 64) LU[i] = __builtin_nan("");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    int perm = lane, f = 0;
    for (int r = 0; r <= twice; ++r) {
        f = factor<NMAX, KIND>(Jt, LU, (LDSd*)scr, g[rid], n, lane, perm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
    }
    for (size_t i = lane; i < lws(NMAX); i += 64) Fout[(size_t)rid * lws(NMAX) + i] = LU[i];
    pout[(size_t)rid * 64 + lane] = perm;
    if (lane == 0) fout[rid] = f;
}

// throughput: W waves per block (16 waves/CU), each factors matrix (w mod nm) `reps` times; with
// alt = 1 it alternates between two matrices (pivot orders differ: interchange path every LU)
template <int NMAX, int KIND>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_bench(
    int nw, int n, const double* J, const double* g, int nm, int reps, int alt, double* ws, int* fout) {
    const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));   // wave-uniform
    const int lane = threadIdx.x & 63;
    __shared__ double scr[4][192];
    if (w >= nw) return;
    double* base = ws + (size_t)w * (2 * NMAX * 64 + lws(NMAX));
    double* LU = base + 2 * NMAX * 64;
    for (int v = 0; v < 2; ++v) {
        const int m = (w + v) % nm;
        for (int j = 0; j < NMAX; ++j)
            base[v * NMAX * 64 + j * 64 + lane] = (lane < n && j < n) ? J[((size_t)m * n + lane) * n + j] : 0.0;
    }
    int perm = lane, f = 0;
    for (int r = 0; r < reps; ++r) {
        double* Jt = base + ((alt && (r & 1)) ? NMAX * 64 : 0);
        f |= factor<NMAX, KIND>(Jt, LU, (LDSd*)&scr[threadIdx.x >> 6][0], g[w % nm], n, lane, perm);
    }
    if (lane == 0) fout[w] = f;
}

template <int NMAX>
static int check(int n, int N, std::mt19937_64& rng, int reps) {
    std::normal_distribution<double> nd;
    std::uniform_real_distribution<double> ud(-8, 8), ug(-12, -2);
    std::vector<double> J((size_t)N * n * n), g(N);
    for (int i = 0; i < N; ++i) {
        for (int a = 0; a < n; ++a) {
            const double s = std::exp(ud(rng));
            for (int b = 0; b < n; ++b) J[((size_t)i * n + a) * n + b] = nd(rng) * s;
        }
        g[i] = std::exp(ug(rng));
        if (i % 4 == 3) {   // exact ties in a column: duplicated rows (scaled by -1)
            for (int b = 0; b < n; ++b) J[((size_t)i * n + 1) * n + b] = -J[((size_t)i * n + 0) * n + b];
        }
        if (i % 8 == 5) {   // a zero column (singular unless gamma J has the identity there)
            for (int a = 0; a < n; ++a) J[((size_t)i * n + a) * n + 2] = 0.0;
        }
    }
    double *dJ, *dg, *dws, *dF[2];
    int *dp[2], *df[2];
    CK(hipMalloc(&dJ, J.size() * 8));
    CK(hipMalloc(&dg, N * 8));
    CK(hipMalloc(&dws, (size_t)N * (NMAX * 64 + lws(NMAX)) * 8));
    for (int k = 0; k < 2; ++k) {
        CK(hipMalloc(&dF[k], (size_t)N * lws(NMAX) * 8));
        CK(hipMalloc(&dp[k], (size_t)N * 64 * 4));
        CK(hipMalloc(&df[k], (size_t)N * 4));
    }
    CK(hipMemcpy(dJ, J.data(), J.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, g.data(), N * 8, hipMemcpyHostToDevice));
    int bad = 0;
    for (int twice = 0; twice < 2; ++twice) {
        hipLaunchKernelGGL((k_fac<NMAX, 0>), dim3(N), dim3(64), 0, 0, N, n, dJ, dg, twice, dws, dF[0], dp[0], df[0]);
        hipLaunchKernelGGL((k_fac<NMAX, 2>), dim3(N), dim3(64), 0, 0, N, n, dJ, dg, twice, dws, dF[1], dp[1], df[1]);
        CK(hipDeviceSynchronize());
        std::vector<double> F0((size_t)N * lws(NMAX)), F1(F0.size());
        std::vector<int> p0((size_t)N * 64), p1(p0.size()), f0(N), f1(N);
        CK(hipMemcpy(F0.data(), dF[0], F0.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(F1.data(), dF[1], F1.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(p0.data(), dp[0], p0.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(p1.data(), dp[1], p1.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(f0.data(), df[0], N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(f1.data(), df[1], N * 4, hipMemcpyDeviceToHost));
        int nf = 0, shown = 0;
        for (int i = 0; i < N; ++i) {
            if (f0[i]) ++nf;
            bool ok = f0[i] == f1[i];
            if (!f0[i]) {   // the factors are only defined for a successful factorization
                for (int l = 0; l < 64 && ok; ++l) ok = p0[(size_t)i * 64 + l] == p1[(size_t)i * 64 + l];
                size_t first = 0;
                for (size_t e = 0; e < lws(NMAX) && ok; ++e) {
                    const double a = F0[(size_t)i * lws(NMAX) + e], b = F1[(size_t)i * lws(NMAX) + e];
                    if (memcmp(&a, &b, 8) != 0) { ok = false; first = e; }
                }
                if (!ok && shown < 4) {
                    ++shown;
                    const size_t e = first;
                    printf("  n=%d twice=%d matrix %d: first difference at %zu (col %zu row %zu): %.17g vs %.17g; perm0[0..7]",
                           n, twice, i, e, e / NMAX, e % NMAX, F0[(size_t)i * lws(NMAX) + e], F1[(size_t)i * lws(NMAX) + e]);
                    for (int l = 0; l < 8; ++l) printf(" %d/%d", p0[(size_t)i * 64 + l], p1[(size_t)i * 64 + l]);
                    printf("\n");
                }
            }
            if (!ok) ++bad;
        }
        printf("n=%2d NMAX=%d twice=%d: %d / %d matrices differ (%d singular)\n", n, NMAX, twice, bad, N, nf);
    }
    // throughput
    if (reps > 0) {
        const int nw = 256 * 16, nm = N;
        double* wsb;
        int* fb;
        CK(hipMalloc(&wsb, (size_t)nw * (2 * NMAX * 64 + lws(NMAX)) * 8));
        CK(hipMalloc(&fb, nw * 4));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int alt = 0; alt < 2; ++alt) {
            float ms[2][2];
            for (int kind = 0; kind < 2; ++kind) {
                for (int rr = 0; rr < 2; ++rr) {       // rr = 0: one LU (setup cost), 1: 1 + reps LUs
                    const int nr = rr ? 1 + reps : 1;
                    for (int it = 0; it < 2; ++it) {
                        CK(hipEventRecord(e0));
                        if (kind == 0) hipLaunchKernelGGL((k_bench<NMAX, 0>), dim3(nw / 4), dim3(256), 0, 0, nw, n, dJ, dg, nm, nr, alt, wsb, fb);
                        else hipLaunchKernelGGL((k_bench<NMAX, 2>), dim3(nw / 4), dim3(256), 0, 0, nw, n, dJ, dg, nm, nr, alt, wsb, fb);
                        CK(hipEventRecord(e1));
                        CK(hipEventSynchronize(e1));
                        CK(hipEventElapsedTime(&ms[kind][rr], e0, e1));
                    }
                }
            }
            const double t0 = (ms[0][1] - ms[0][0]) * 1e3 / reps, t1 = (ms[1][1] - ms[1][0]) * 1e3 / reps;
            printf("n=%2d %s: row-per-lane %.2f us, grid %.2f us per LU round (%d waves, 16/CU; %d LUs each, setup "
                   "subtracted), ratio %.3f\n", n, alt ? "alternating pivot orders" : "stable pivot order", t0, t1, nw, reps, t1 / t0);
        }
        hipFree(wsb);
        hipFree(fb);
    }
    hipFree(dJ); hipFree(dg); hipFree(dws);
    for (int k = 0; k < 2; ++k) { hipFree(dF[k]); hipFree(dp[k]); hipFree(df[k]); }
    return bad;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::mt19937_64 rng(12345);
    int bad = 0;
    bad += check<32>(20, 512, rng, 0);
    bad += check<32>(32, 512, rng, 0);
    bad += check<56>(33, 512, rng, 0);
    bad += check<56>(47, 512, rng, 0);
    bad += check<56>(53, 1024, rng, reps);
    bad += check<56>(56, 512, rng, 0);
    bad += check<64>(57, 512, rng, 0);
    bad += check<64>(64, 512, rng, 0);
    bad += check<32>(20, 1024, rng, reps);
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
