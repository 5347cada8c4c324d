"""C5 gas+surface failure statistics on the GPU with both Jacobians (CVODE's CV_ERR_FAILURE, -3):
the bench ensemble of 1e5 reactors integrated with the analytic and with CVODE's DQ Jacobian, failure
counts and the step / Jacobian counts. Usage: python scripts/c5_failures.py [N] > out.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    import _pkgload
    import bench
    pkg = _pkgload.load()
    from batchreactor_amd import ensemble
    mech = bench.make_mech(pkg, "gas_surf")
    eng = pkg.Engine(mech)
    T, Asv, U0 = ensemble.make_inputs(mech, "gas_surf", 0, N)
    out = {"reactors": N, "config": "C5 gas+surface bench ensemble (ensemble.make_inputs, seed 0), tf 10 s, rtol 1e-6 / atol 1e-10"}
    for dq in (False, True):
        U, st = eng.integrate(T, Asv, U0, 10.0, dq_jacobian=dq)
        s = st["status"]
        out["dq" if dq else "analytic"] = {
            "failed": int(np.sum(s != 0)), "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(s, return_counts=True))},
            "kernel_ms": eng.last_kernel_ms(), "mean_steps": float(st["nsteps"].mean()), "mean_nje": float(st["nje"].mean()),
            "mean_nfe": float(st["nfe"].mean()), "mean_nfe_dq": float(st["nfe_dq"].mean()),
            "failed_ids_first": [int(i) for i in np.nonzero(s != 0)[0][:40]]}
    a, d = set(out["analytic"]["failed_ids_first"]), set(out["dq"]["failed_ids_first"])
    out["note"] = "which reactors fail is rounding-dependent; the rates compare the algorithms"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
