"""The north_star's MFMA question at the integrator's matrix size: time the rank-16 LU trailing
update of a 64 x 64 fp64 matrix per wave with the engine's VALU form (row per lane, v_readlane
broadcasts) and with v_mfma_f64_16x16x4_f64 (tile layout, operands staged through LDS), check that
both give the same matrix, print one JSON line. Usage: python scripts/exp_mfma_lu.py [nmat] [reps]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "scripts", "micro", "libexp_lu.so"))   # make -C scripts/micro libexp_lu.so
lib.exp_lu_update.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int,
                              C.POINTER(C.c_float)]
nmat = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rng = np.random.default_rng(0)
A = rng.standard_normal((nmat, 64, 64))
out = {}
res = {}
for v, name in ((0, "valu_readlane"), (1, "mfma_f64_16x16x4")):
    o = np.zeros_like(A)
    ms = C.c_float()
    rc = lib.exp_lu_update(v, A.ctypes.data_as(C.POINTER(C.c_double)), o.ctypes.data_as(C.POINTER(C.c_double)),
                           nmat, reps, 5, C.byref(ms))
    assert rc == 0, rc
    flop = nmat * reps * 2.0 * 48 * 16 * 48
    out[name] = {"ms": ms.value, "TFLOPs": flop / (ms.value * 1e-3) / 1e12,
                 "frac_fp64_peak": flop / (ms.value * 1e-3) / 78.6e12}
    res[name] = o
ref = A.copy()
ref[:, 16:, 16:] -= reps * (A[:, 16:, :16] @ A[:, :16, 16:])
for name in res:
    out[name]["max_rel_err_vs_numpy"] = float(np.max(np.abs(res[name] - ref)) / np.max(np.abs(ref)))
out["speedup_mfma_over_valu"] = out["valu_readlane"]["ms"] / out["mfma_f64_16x16x4"]["ms"]
out["workload"] = f"{nmat} matrices 64x64 fp64, one per wave, rank-16 trailing update x {reps}"
print(json.dumps(out))
