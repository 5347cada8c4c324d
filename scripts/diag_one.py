"""Trace one synthetic-ensemble reactor on the GPU next to the CPU oracle.
Usage: python scripts/diag_one.py case index"""
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
case, idx = sys.argv[1], int(sys.argv[2])
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat"}[case]
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas)
om = oracle.Mech(os.path.join(LIB, gas), os.path.join(LIB, "therm.dat"))
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, idx + 1)
T, Asv, U0 = T[idx:], Asv[idx:], U0[idx:]
cap = 3000
U, st, tr = eng.integrate(T, Asv, U0, 10.0, trace_cap=cap)
uo, so, rows = om.integrate(T[0], Asv[0], U0[0], 10.0, analytic_jac=True, record=True)
print({k: float(st[k][0]) for k in pkg.STAT_FIELDS})
print(so)
ns = int(min(st["nsteps"][0], cap))
np.set_printoptions(precision=3, linewidth=200)
for s in range(1, ns + 1, max(1, ns // 60)):
    o = rows[s] if s < len(rows) else None
    print(f"{s:6d} gpu t={tr[0, s, 0]:.5e} h={tr[0, s, 1]:.3e} q={tr[0, s, 2]:.0f}  " +
          (f"orc t={o[0]:.5e}" if o else ""))
last = tr[0, ns, 4:]
print("gpu state at last traced step", last)
print("min component", last.min(), "sum", last.sum(), "u0 sum", U0[0].sum())
