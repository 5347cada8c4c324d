"""First divergence of the GPU accepted-step sequence from the oracle's (parity-test inputs).
Usage: python scripts/diag_trace.py case N index"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import _mechs, _ignition_inputs  # noqa: E402

pkg = _pkgload.load()
case, N, idx = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
pm, om = _mechs(pkg, oracle, case)
eng = pkg.Engine(pm)
T, Asv, U0 = _ignition_inputs(pm, case, N, 5)
cap = 3000
U, st, tr = eng.integrate(T[idx:idx + 1], Asv[idx:idx + 1], U0[idx:idx + 1], 10.0, trace_cap=cap)
uo, so, rows = om.integrate(T[idx], Asv[idx], U0[idx], 10.0, analytic_jac=True, record=True)
ns = int(min(st["nsteps"][0], len(rows) - 1, cap))
print("gpu steps", st["nsteps"][0], "orc", so["nsteps"])
first = None
for s in range(1, ns + 1):
    rel = abs(tr[0, s, 0] / rows[s][0] - 1)
    if rel > 1e-9 and first is None:
        first = s
    if first is not None and s < first + 12:
        print(f"step {s}: gpu t={tr[0, s, 0]:.12e} h={tr[0, s, 1]:.6e} q={tr[0, s, 2]:.0f} | orc t={rows[s][0]:.12e}")
print("first divergence (1e-9 in t):", first)
np.set_printoptions(precision=4, linewidth=200)
for s in [first - 1, first] if first else []:
    u_g, u_o = tr[0, s, 4:], rows[s][1]
    big = np.abs(u_o) > 1e-12
    print(s, "state rel diff", np.max(np.abs(u_g[big] / u_o[big] - 1)))
