// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// integrator uses (its workspace traffic is mostly 8-B-per-lane raw buffer loads: factor columns,
// J columns, {kf, kr} pairs as 16 B), against a known byte count. Every kernel streams `bytes` of a
// buffer once per launch, coalesced (lane l of wave w reads element w*64 + l per instruction).
//   mode 0: raw_buffer_load_b64 (8 B/lane)      mode 1: raw_buffer_load_b128 (16 B/lane)
//   mode 2: global_load_dwordx2 (8 B/lane)      mode 3: raw_buffer_store_b64 (8 B/lane)
// scripts/micro/fetch_calib.py runs each mode under rocprofv3 --pmc and prints counter / bytes.
#include <hip/hip_runtime.h>

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k_stream(double* __restrict__ p, size_t n, double* __restrict__ sink) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7fffffff, 0x00020000);
    const size_t per = MODE == 1 ? 2 : 1;               // doubles per lane per access
    const size_t stride = (size_t)gridDim.x * blockDim.x * per;
    double acc = 0.0;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * per; i < n; i += stride) {
        if constexpr (MODE == 0) {
            acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (unsigned)(i * 8), 0, 0));
        } else if constexpr (MODE == 1) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(i * 8), 0, 0);
            acc += __builtin_bit_cast(double, u32x2{v[0], v[1]}) + __builtin_bit_cast(double, u32x2{v[2], v[3]});
        } else if constexpr (MODE == 2) {
            acc += p[i];
        } else {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, (double)i), rs, (unsigned)(i * 8), 0, 0);
        }
    }
    if (acc == 12345.678) sink[0] = acc;   // keeps the loads
}

extern "C" int fetch_calib(int mode, size_t bytes, int reps) {
    double *p = nullptr, *sink = nullptr;
    if (bytes > 0x7fff0000ull) return -1;   // 2 GB buffer range
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return -2;
    if (hipMemset(p, 0, bytes) != hipSuccess) return -3;
    const size_t n = bytes / 8;
    for (int r = 0; r < reps; ++r) {
        if (mode == 0) hipLaunchKernelGGL(k_stream<0>, dim3(2048), dim3(256), 0, 0, p, n, sink);
        else if (mode == 1) hipLaunchKernelGGL(k_stream<1>, dim3(2048), dim3(256), 0, 0, p, n, sink);
        else if (mode == 2) hipLaunchKernelGGL(k_stream<2>, dim3(2048), dim3(256), 0, 0, p, n, sink);
        else hipLaunchKernelGGL(k_stream<3>, dim3(2048), dim3(256), 0, 0, p, n, sink);
    }
    const hipError_t e = hipDeviceSynchronize();
    hipFree(p);
    hipFree(sink);
    return e == hipSuccess ? 0 : -4;
}
