// mfma_f64_layout.hip -- one v_mfma_f64_16x16x4f64 per wave on lane-indexed inputs: a[lane], b[lane],
// c[reg][lane] in; d[reg][lane] out (checks the operand / accumulator lane maps the blocked LU uses)
#include <hip/hip_runtime.h>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* a, const double* b, const double* c, double* d) {
    const int l = threadIdx.x;
    d4 x;
    for (int i = 0; i < 4; ++i) x[i] = c[i * 64 + l];
    x = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], x, 0, 0, 0);
    for (int i = 0; i < 4; ++i) d[i * 64 + l] = x[i];
}
extern "C" int mfma_f64_layout(const double* a, const double* b, const double* c, double* d) {
    double *da, *db, *dc, *dd;
    hipMalloc(&da, 512); hipMalloc(&db, 512); hipMalloc(&dc, 2048); hipMalloc(&dd, 2048);
    hipMemcpy(da, a, 512, hipMemcpyHostToDevice);
    hipMemcpy(db, b, 512, hipMemcpyHostToDevice);
    hipMemcpy(dc, c, 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
    hipMemcpy(d, dd, 2048, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(dc); hipFree(dd);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
