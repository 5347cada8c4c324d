"""GPU check: lane engine with the analytic per-lane Jacobian on a few H2/O2 reactors vs the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import _pkgload  # noqa: E402
import oracle  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
pm = pkg.Mechanism.from_files(LIB, gas_mech="h2o2.dat")
om = oracle.Mech(os.path.join(LIB, "h2o2.dat"), os.path.join(LIB, "therm.dat"))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T, Asv, U0 = ensemble.make_inputs(pm, "h2o2", 0, N)
eng = pkg.Engine(pm)
print("engine", eng.engine, flush=True)
U, st = eng.integrate(T, Asv, U0, 1e-2, rtol=1e-10, atol=1e-16)
print("status", np.unique(st["status"]), flush=True)
err = 0.0
for i in range(N):
    uo, so, _ = om.integrate(T[i], Asv[i], U0[i], 1e-2, analytic_jac=True, rtol=1e-10, atol=1e-16)
    err = max(err, float(np.max(np.abs(U[i] - uo) / (1e-6 * np.abs(uo) + 1e-14))))
print("tight err", err, "steps", st["nsteps"][:4], flush=True)
