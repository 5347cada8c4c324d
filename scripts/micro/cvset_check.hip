// cvset_check.hip -- device-side check that the 16-lane groups' lane-parallel cvSet (cv_set_lp) and
// step-size ratios give bit-for-bit the values of the generic forms (cv_set<16>, one root_int per
// ratio) on random controller states. Includes the whole integrator translation unit; not part of
// libbrhip.so.   python3 scripts/cvset_check.py
#include "../../batchreactor.jl_amd/csrc/brhip.hip"

namespace {
constexpr int NOUT = 16;   // doubles per case and variant
__global__ __launch_bounds__(64) void k_cvchk(int ncase, const double* __restrict__ din, const int* __restrict__ iin,
                                              double* __restrict__ out) {
    __shared__ Ctl cs[2][4];
    const int lane = threadIdx.x, g = lane >> 4, t = lane & 15;
    const int c = blockIdx.x * 4 + g;
    const int cc = c < ncase ? c : ncase - 1;
    AttemptIn in;
    in.q = iin[4 * cc]; in.qwait = iin[4 * cc + 1]; in.nst = iin[4 * cc + 2]; in.nstlp = 0;
    in.h = din[10 * cc]; in.tn = 0.0; in.tstop = 1.0; in.gammap = din[10 * cc + 1];
    for (int i = 0; i < QMAX + 2; ++i) in.tau[i] = din[10 * cc + 2 + i];
    LCtl* C0 = (LCtl*)&cs[0][g];
    LCtl* C1 = (LCtl*)&cs[1][g];
    if (t == 0) {
        for (int i = 0; i < 6; ++i) { C0->tq[i] = -1.0; C1->tq[i] = -1.0; }
        C0->gammap = -1.0; C1->gammap = -1.0;
    }
    wave_sync();
    double t4a, gra, t4b, grb;
    cv_set<16>(C0, in, t4a, gra);
    cv_set_lp(C1, in, t4b, grb);
    wave_sync();
    // the step-size ratios: lane 0 etaq (L), lane 1 etaqm1 (q), lane 2 etaqp1 (L + 1), as ctl_post_solve
    const double dsm = din[10 * cc + 9], ddn = 0.7 * dsm + 1e-3, dup = 1.3 * dsm + 2e-3;
    const int q = in.q, L = q + 1;
    const double xa = t == 1 ? BIAS1 * ddn : (t == 2 ? BIAS3 * dup : BIAS2 * dsm);
    const int La = t == 1 ? q : (t == 2 ? L + 1 : L);
    const double er = 1.0 / (root_int(xa, La) + ADDON);
    const double e0 = row_lane<0>(er), e1 = row_lane<1>(er), e2 = row_lane<2>(er);
    const double f0 = 1.0 / (root_int(BIAS2 * dsm, L) + ADDON);
    const double f1 = 1.0 / (root_int(BIAS1 * ddn, q) + ADDON);
    const double f2 = 1.0 / (root_int(BIAS3 * dup, L + 1) + ADDON);
    if (c < ncase) {
        double* o = out + (size_t)c * 2 * NOUT * 16 + t * 2 * NOUT;   // every lane's view
        for (int v = 0; v < 2; ++v) {
            LCtl* C = v ? C1 : C0;
            double* p = o + v * NOUT;
            for (int i = 0; i <= QMAX; ++i) p[i] = C->l[i];
            for (int i = 1; i <= 5; ++i) p[5 + i] = C->tq[i];
            p[11] = C->rl1; p[12] = C->gamma; p[13] = C->gamrat; p[14] = v ? t4b : t4a;
            p[15] = v ? (e0 + 2.0 * e1 + 4.0 * e2) : (f0 + 2.0 * f1 + 4.0 * f2);
        }
        (void)gra; (void)grb;
    }
}
}  // namespace

extern "C" int cvset_check(int ncase, const double* din, const int* iin, double* out) {
    double *dd, *dout;
    int* di;
    if (hipMalloc(&dd, sizeof(double) * 10 * ncase) != hipSuccess) return -1;
    if (hipMalloc(&di, sizeof(int) * 4 * ncase) != hipSuccess) return -1;
    const size_t no = (size_t)ncase * 2 * NOUT * 16;
    if (hipMalloc(&dout, sizeof(double) * no) != hipSuccess) return -1;
    (void)hipMemcpy(dd, din, sizeof(double) * 10 * ncase, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, iin, sizeof(int) * 4 * ncase, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_cvchk, dim3((ncase + 3) / 4), dim3(64), 0, 0, ncase, dd, di, dout);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipMemcpy(out, dout, sizeof(double) * no, hipMemcpyDeviceToHost);
    (void)hipFree(dd); (void)hipFree(di); (void)hipFree(dout);
    return (int)e;
}
