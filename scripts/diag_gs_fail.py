"""GPU: step-by-step trace of one gas+surface reactor (t, h, q per accepted step) next to the
oracle's accepted-step times; prints where the two step sequences part."""
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
i = int(sys.argv[1])
pm = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat", surface_mech="ch4ni.xml")
om = oracle.Mech(os.path.join(LIB, "grimech.dat"), os.path.join(LIB, "therm.dat"), os.path.join(LIB, "ch4ni.xml"))
T, Asv, U0 = ensemble.make_inputs(pm, "gas_surf", 0, i + 1)
T, Asv, U0 = T[i:], Asv[i:], U0[i:]
U, st, tr = pkg.Engine(pm).integrate(T, Asv, U0, 10.0, trace_cap=3000)
nst = int(st["nsteps"][0])
print("gpu status", st["status"][0], "steps", nst, "netf", st["netf"][0], "t_end", st["t_end"][0])
uo, so, rows = om.integrate(T[0], Asv[0], U0[0], 10.0, analytic_jac=True, record=True)
to = np.array([r[0] for r in rows])
print("oracle status", so["status"], "steps", so["nsteps"], "netf", so["netf"])
tg = tr[0, :nst + 1, 0]
k = 1
while k < min(len(tg), len(to)) and abs(tg[k] / max(to[k], 1e-300) - 1) < 1e-8:
    k += 1
print("step sequences agree to 1e-8 for", k, "steps")
n = pm.n
for j in range(max(k - 3, 0), min(k + 12, nst + 1)):
    ug = tr[0, j, 4:4 + n]
    line = f"  {j:4d} gpu t={tg[j]:.10e} h={tr[0, j, 1]:.4e} q={tr[0, j, 2]:.0f}"
    if j < len(to):
        e = np.max(np.abs(ug - rows[j][1]) / (1e-6 * np.abs(rows[j][1]) + 1e-10))
        line += f" | orc t={to[j]:.10e}  state diff (1e-6 band) {e:.3g}"
    print(line)
print("oracle steps around the GPU's end:")
for j in range(len(to)):
    if 1.1e-4 < to[j] < 2.2e-4:
        print(f"  {j:4d} orc t={to[j]:.10e}")
print("gpu last steps:")
for j in range(max(nst - 12, 0), nst + 1):
    print(f"  {j:4d} t={tg[j]:.10e} h={tr[0, j, 1]:.4e} q={tr[0, j, 2]:.0f}")
