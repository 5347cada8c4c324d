"""Global error at tf of the GPU engine and of the oracle (analytic / DQ Jacobian) at the default
tolerances, against a tight-tolerance oracle solution. Usage: python scripts/diag_globalerr.py case N"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import _pkgload  # noqa: E402
import oracle  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
case, N = sys.argv[1], int(sys.argv[2])
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat"}[case]
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas)
om = oracle.Mech(os.path.join(LIB, gas), os.path.join(LIB, "therm.dat"))
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
eng = pkg.Engine(pm)
U, st = eng.integrate(T, Asv, U0, 10.0)
Ua, sa, _ = om.integrate_batch(T, Asv, U0, 10.0, analytic_jac=True, nthreads=8)
Ud, sd, _ = om.integrate_batch(T, Asv, U0, 10.0, analytic_jac=False, nthreads=8)
Ut, stt, _ = om.integrate_batch(T, Asv, U0, 10.0, rtol=1e-10, atol=1e-14, analytic_jac=True, nthreads=8)
ok = (st["status"] == 0) & np.array([s["status"] == 0 for s in sa]) & np.array([s["status"] == 0 for s in sd]) & \
     np.array([s["status"] == 0 for s in stt])


def gerr(X):
    e = np.abs(X - Ut) / (np.abs(Ut) + 1e-6 * np.abs(Ut).max(axis=1, keepdims=True))
    return e[ok].max(axis=1)


for name, X in (("gpu", U), ("oracle-analytic", Ua), ("oracle-DQ", Ud)):
    g = gerr(X)
    print(f"{name:16s} global rel err (species > 1e-6 of max): median {np.median(g):.2e} p90 {np.percentile(g, 90):.2e} "
          f"max {g.max():.2e}")
print("reactors compared", int(ok.sum()), "of", N)
