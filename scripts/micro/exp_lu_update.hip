// exp_lu_update.hip -- the north_star's MFMA question, measured: does fp64 MFMA
// (v_mfma_f64_16x16x4_f64) beat the VALU for the LU trailing update at the integrator's matrix
// sizes? One 64 x 64 matrix per wave (n = 53..64 padded), the rank-16 trailing update of the first
// panel, C[16:64, 16:64] -= L[16:64, 0:16] * U[0:16, 16:64] (L = columns 0..15, U = rows 0..15 of
// A: the largest panel update of a blocked LU), repeated `reps` times per wave:
//
//   k_upd_valu : row-per-lane layout, the engine's form (brhip_device.hpp lu_rl_steps / lu_factor):
//                lane i holds row i; 16 rank-1 steps, each pivot-row element broadcast by
//                v_readlane (2 per double) into an FMA;
//   k_upd_mfma : tile layout, A held as 4 x 4 tiles of 16 x 16 in the f64 MFMA accumulator layout
//                (col = lane & 15, row = (lane >> 4) + 4 r); the L panel is re-laid into MFMA
//                A-operands through LDS and the 16 pivot rows into B-operands through LDS (with
//                partial pivoting the pivot rows are arbitrary rows, so both go through LDS), then
//                3 x 3 output tiles x 4 k-steps = 36 MFMAs.
//
// Both produce the same C (checked by the driver, scripts/exp_mfma_lu.py). Built as
// libexp_lu.so (not part of libbrhip.so); timed with HIP events and rocprofv3 --kernel-trace.
#include <hip/hip_runtime.h>

#include <cstdio>

namespace {

constexpr int NM = 64;   // padded matrix size
constexpr int PW = 16;   // panel width

__device__ __forceinline__ double rdl(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// A: [nmat][64][64] row-major; out: same
__global__ __launch_bounds__(256, 2) void k_upd_valu(const double* __restrict__ A, double* __restrict__ out, int nmat,
                                                  int reps) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= nmat) return;
    const double* a0 = A + (size_t)w * NM * NM + (size_t)lane * NM;
    double l[PW], u[NM - PW], c[NM - PW];
#pragma unroll
    for (int k = 0; k < PW; ++k) l[k] = lane >= PW ? a0[k] : 0.0;   // rows 0..15 are the pivot rows
#pragma unroll
    for (int j = 0; j < NM - PW; ++j) { u[j] = a0[PW + j]; c[j] = u[j]; }
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < PW; ++k)
#pragma unroll
            for (int j = 0; j < NM - PW; ++j) c[j] = fma(-rdl(u[j], k), l[k], c[j]);
    }
    double* o = out + (size_t)w * NM * NM + (size_t)lane * NM;
#pragma unroll
    for (int k = 0; k < PW; ++k) o[k] = a0[k];
#pragma unroll
    for (int j = 0; j < NM - PW; ++j) o[PW + j] = c[j];
}

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 2) void k_upd_mfma(const double* __restrict__ A, double* __restrict__ out, int nmat,
                                                  int reps) {
    __shared__ double lds[4][NM * PW + PW * (NM - PW)];   // per wave: L panel [64][16], U rows [16][48]
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int w = blockIdx.x * (blockDim.x >> 6) + wv;
    if (w >= nmat) return;
    double* Ls = lds[wv];
    double* Us = lds[wv] + NM * PW;
    const double* a0 = A + (size_t)w * NM * NM;
    const int col = lane & 15, g = lane >> 4;
    d4 T[4][4];   // tile (I, J): element (16I + g + 4r, 16J + col) in T[I][J][r]
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) T[I][J][r] = a0[(16 * I + g + 4 * r) * NM + 16 * J + col];
    // the operands (tile column 0 = L, tile row 0 = the pivot rows U) are not updated
    for (int r = 0; r < reps; ++r) {
        // L panel -> LDS row-major [64][16]; pivot rows (0..15) of columns 16..63 -> [16][48]
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
            for (int q = 0; q < 4; ++q) Ls[(16 * I + g + 4 * q) * PW + col] = T[I][0][q];
#pragma unroll
        for (int J = 1; J < 4; ++J)
#pragma unroll
            for (int q = 0; q < 4; ++q) Us[(g + 4 * q) * (NM - PW) + 16 * (J - 1) + col] = T[0][J][q];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's own LDS writes are visible
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            double av[4], bv[3];
#pragma unroll
            for (int I = 1; I < 4; ++I) av[I] = Ls[(16 * I + col) * PW + 4 * t + g];      // A[i = lane&15][k = lane>>4]
#pragma unroll
            for (int J = 0; J < 3; ++J) bv[J] = Us[(4 * t + g) * (NM - PW) + 16 * J + col];  // B[k = lane>>4][j = lane&15]
#pragma unroll
            for (int I = 1; I < 4; ++I)
#pragma unroll
                for (int J = 1; J < 4; ++J)
                    T[I][J] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[I], bv[J - 1], T[I][J], 0, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();
    }
    double* o = out + (size_t)w * NM * NM;
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[(16 * I + g + 4 * r) * NM + 16 * J + col] = T[I][J][r];
}

}  // namespace

extern "C" int exp_lu_update(int variant, const double* hA, double* hout, int nmat, int reps, int iters, float* ms) {
    double *dA = nullptr, *dO = nullptr;
    const size_t bytes = (size_t)nmat * NM * NM * sizeof(double);
    if (hipMalloc(&dA, bytes) != hipSuccess || hipMalloc(&dO, bytes) != hipSuccess) return -1;
    hipMemcpy(dA, hA, bytes, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 grid((nmat + 3) / 4), block(256);
    auto launch = [&]() {
        if (variant == 0) hipLaunchKernelGGL(k_upd_valu, grid, block, 0, 0, dA, dO, nmat, reps);
        else hipLaunchKernelGGL(k_upd_mfma, grid, block, 0, 0, dA, dO, nmat, reps);
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1);
    *ms = t / iters;
    const hipError_t err = hipGetLastError();
    hipMemcpy(hout, dO, bytes, hipMemcpyDeviceToHost);
    hipFree(dA);
    hipFree(dO);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return err == hipSuccess ? 0 : -2;
}
