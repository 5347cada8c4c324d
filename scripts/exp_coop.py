"""VERDICT r05 item 3 measured on the phases it changes: the cooperative LU + solve (one GRI reactor
per 4-wave workgroup, factors in registers; scripts/micro/coop_lusolve.hip) against the integrator's
own lu_factor<56> / lu_solve<56> (one reactor per wave, factors in the global workspace), both at
16 waves/CU. Inputs are real GRI Newton matrices: analytic Jacobians (br_jacobian) at states taken
from an integration of the bench ensemble (CVODE dense output at 1e-6 .. 1 s), gamma log-uniform in
[1e-8, 1e-3] s. Unit = one factorization + NSOLVE solves (the integrator's ~9.2 solves per
factorization on GRI C3), REPS units per reactor with each LU entering in the previous pivot order.

  python3 scripts/exp_coop.py [N] [REPS] [NSOLVE] [TAG]   -> gpurun_out/coop_ab[_TAG].json
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import _pkgload  # noqa: E402
import bench  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    nsolve = int(sys.argv[3]) if len(sys.argv) > 3 else 9
    tag = ("_" + sys.argv[4]) if len(sys.argv) > 4 else ""
    pkg = _pkgload.load()
    mech = bench.make_mech(pkg, "gri")
    eng = pkg.Engine(mech)
    n = mech.n
    K = 512
    T, A, U0 = bench.ensemble_inputs(pkg, mech, "gri", K)
    tout = np.array([1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 1e-1, 1.0])
    _, st = eng.integrate(T, A, U0, 1.0, tout=tout)
    Y = st["yout"].reshape(-1, n)
    TT = np.repeat(T, len(tout))
    AA = np.repeat(A, len(tout))
    J = np.ascontiguousarray(eng.jacobian(TT, AA, Y))
    nj = J.shape[0]
    rng = np.random.default_rng(7)
    g = np.ascontiguousarray(10.0 ** rng.uniform(-8, -3, N))
    b = np.ascontiguousarray(rng.standard_normal((N, n)))
    lib = C.CDLL(os.path.join(ROOT, "scripts", "micro", "libcoop.so"))
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int)
    lib.coop_run.argtypes = [C.c_int, C.c_int, C.c_int, dp, C.c_int, dp, dp, C.c_int, C.c_int, dp, dp, ip, dp, ip]
    P = lambda a: a.ctypes.data_as(dp)  # noqa: E731
    res = {}
    outs = {}
    modes = ((0, "base_wavefront"), (1, "coop_panel_16w_per_cu"), (2, "coop_panel_uncapped"),
             (3, "coop_step_16w_per_cu"), (4, "coop_step_uncapped"))
    for mode, name in modes:
        x = np.zeros((N, n))
        chk = np.zeros((N, n))
        fail = np.zeros(N, dtype=np.int32)
        ms = C.c_double(0.0)
        vg = C.c_int(0)
        t0 = time.time()
        rc = lib.coop_run(mode, N, n, P(J), nj, P(g), P(b), reps, nsolve, P(x), P(chk), fail.ctypes.data_as(ip),
                          C.byref(ms), C.byref(vg))
        if rc != 0:
            raise SystemExit(f"{name}: coop_run returned {rc}")
        units = N * reps
        res[name] = {"ms": ms.value, "units_per_s": units / (ms.value * 1e-3), "vgprs": vg.value,
                     "fail": int(np.count_nonzero(fail)), "wall_s": time.time() - t0}
        outs[name] = (x, chk, fail)
        print(name, json.dumps(res[name]), flush=True)
    xb, cb, fb = outs["base_wavefront"]
    for _, name in modes[1:]:
        x, c, f = outs[name]
        res[name]["bit_identical_x"] = bool(np.array_equal(x.view(np.int64), xb.view(np.int64)))
        res[name]["bit_identical_checksum"] = bool(np.array_equal(c.view(np.int64), cb.view(np.int64)))
        res[name]["speed_vs_base"] = res[name]["units_per_s"] / res["base_wavefront"]["units_per_s"]
    # sanity against numpy on a sample (last solve's rhs = b * nsolve)
    errs = []
    for r in range(0, N, max(1, N // 64)) if nsolve else []:
        M = np.eye(n) - g[r] * J[r % nj]
        xs = np.linalg.solve(M, b[r] * nsolve)
        errs.append(float(np.max(np.abs(xb[r] - xs)) / max(np.max(np.abs(xs)), 1e-300)))
    out = {"experiment": "cooperative LU + solve vs the integrator's (VERDICT r05 item 3)", "N": N, "n": n,
           "reps": reps, "nsolve": nsolve, "matrices": nj, "gamma_range_s": [1e-8, 1e-3], "modes": res,
           "numpy_max_rel_err_sample": max(errs) if errs else None}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"coop_ab{tag}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
