"""GPU diagnostic: one H2/O2 reactor of the C2 ensemble on the lane engine (DQ Jacobian) and the
wavefront engine (analytic), against the oracle with both Jacobians and a perturbed-u0 oracle run."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import _pkgload  # noqa: E402
import oracle  # noqa: E402
from parity_bands import OUT_T  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
idx = int(sys.argv[1])
pm = pkg.Mechanism.from_files(LIB, gas_mech="h2o2.dat")
om = oracle.Mech(os.path.join(LIB, "h2o2.dat"), os.path.join(LIB, "therm.dat"))
T, Asv, U0 = ensemble.make_inputs(pm, "h2o2", 0, idx + 1)
T, Asv, U0 = T[idx:], Asv[idx:], U0[idx:]
eng = pkg.Engine(pm)
U, st = eng.integrate(T, Asv, U0, 10.0, tout=OUT_T)
os.environ["BRHIP_ENGINE"] = "wave"
Uw, sw = eng.integrate(T, Asv, U0, 10.0, tout=OUT_T)
_, sd, Yd = om.integrate_out(T[0], Asv[0], U0[0], 10.0, OUT_T, analytic_jac=False)
_, sa, Ya = om.integrate_out(T[0], Asv[0], U0[0], 10.0, OUT_T, analytic_jac=True)
print("t_ign lane", st["t_ign"][0], "wave", sw["t_ign"][0], "orc dq", sd["t_ign"], "orc an", sa["t_ign"])
print("steps lane", st["nsteps"][0], "wave", sw["nsteps"][0], "orc dq", sd["nsteps"], "orc an", sa["nsteps"])
for j, t in enumerate(OUT_T[:8]):
    def e(a, b):
        return (np.abs(a - b) / (1e-4 * np.abs(b) + 1e-8)).max()
    print(f"t={t:.2e} lane-vs-orcDQ {e(st['yout'][0, j], Yd[j]):.3g} wave-vs-orcAN {e(sw['yout'][0, j], Ya[j]):.3g} "
          f"orcDQ-vs-orcAN {e(Yd[j], Ya[j]):.3g} lane-vs-orcAN {e(st['yout'][0, j], Ya[j]):.3g}")
    k = np.argmax(np.abs(st['yout'][0, j] - Yd[j]) / (1e-4 * np.abs(Yd[j]) + 1e-8))
    print("    ", pm.species[k], st['yout'][0, j, k], Yd[j, k], Ya[j, k], sw['yout'][0, j, k])
