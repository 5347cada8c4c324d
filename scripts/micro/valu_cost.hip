// Throughput of the VALU forms the integrator's LU / solve use (gfx950), 16 waves per CU:
// v_fma_f64, v_readlane_b32 pairs (fp64 broadcast), v_fmac_f64_dpp row_newbcast, v_mov_b64_dpp.
// Each wave runs 8 independent chains, ITERS x 8 ops per chain. Prints ns per wave-op per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096
template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, double seed) {
    const int lane = threadIdx.x & 63;
    double a[8], f = seed * (lane + 1) * 1e-3;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed + i + lane;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MODE == 0) {          // plain fp64 FMA
                a[i] = __builtin_fma(a[i], f, 1e-9);
            } else if constexpr (MODE == 1) {   // readlane pair (fp64 broadcast) + FMA
                const long long b = __double_as_longlong(a[(i + 1) & 7]);
                const int lo = __builtin_amdgcn_readlane((int)b, i), hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
                const double x = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
                a[i] = __builtin_fma(-x, f, a[i]);
            } else if constexpr (MODE == 2) {   // DPP fp64 FMA with row_newbcast
                asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                             : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(f));
            } else if constexpr (MODE == 3) {   // v_mov_b64_dpp + FMA
                const double x = __builtin_amdgcn_mov_dpp(a[(i + 1) & 7], 0x153, 0xF, 0xF, true);
                a[i] = __builtin_fma(-x, f, a[i]);
            } else if constexpr (MODE == 4) {   // readlane pair only (feeding an integer xor to keep it live)
                const long long b = __double_as_longlong(a[(i + 1) & 7]);
                const int lo = __builtin_amdgcn_readlane((int)b, i), hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
                a[i] = __longlong_as_double(__double_as_longlong(a[i]) ^ (((long long)hi << 32) | (unsigned)lo));
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int MODE>
float run(double* d, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<MODE><<<blocks, 256>>>(d, 1.0);
    hipEventRecord(e0);
    k<MODE><<<blocks, 256>>>(d, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}
int main() {
    int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = ncu * 4;   // 4 x 256 threads = 16 waves per CU = 4 per SIMD
    double* d; hipMalloc(&d, (size_t)blocks * 256 * 8);
    const char* nm[] = {"fma_f64", "readlane2+fma", "fmac_f64_dpp", "mov_b64_dpp+fma", "readlane2+xor"};
    float t[5] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks)};
    // per SIMD: 4 waves x ITERS x 8 wave-ops
    for (int m = 0; m < 5; ++m)
        printf("%-18s %8.3f ms  %6.3f ns per wave-op per SIMD\n", nm[m], t[m], t[m] * 1e6 / (4.0 * ITERS * 8));
    return 0;
}
