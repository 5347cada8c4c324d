"""Gas+surface (n = 66, two components per lane) integration vs the oracle: statuses, counters,
and for the first reactor the GPU fails on, the step trace next to the oracle's."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import _pkgload  # noqa: E402
pkg = _pkgload.load()
import oracle  # noqa: E402  (checker)
from batchreactor_amd import ensemble  # noqa: E402
LIB = os.path.join(ROOT, "tests", "golden", "lib")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
pm = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat", surface_mech="ch4ni.xml")
om = oracle.Mech(os.path.join(LIB, "grimech.dat"), os.path.join(LIB, "therm.dat"), os.path.join(LIB, "ch4ni.xml"))
T, Asv, U0 = ensemble.make_inputs(pm, "gas_surf", 0, N)
eng = pkg.Engine(pm)
U, st, tr = eng.integrate(T, Asv, U0, 10.0, trace_cap=4000)
print("gpu status", st["status"].astype(int).tolist())
print("gpu nsteps", st["nsteps"].astype(int).tolist())
print("gpu netf", st["netf"].astype(int).tolist(), "ncfn", st["ncfn"].astype(int).tolist())
Ua, sta, _ = om.integrate_batch(T, Asv, U0, 10.0, analytic_jac=True, nthreads=8)
print("orc nsteps", [s["nsteps"] for s in sta])
bad = np.nonzero(st["status"] != 0)[0]
i = int(bad[0]) if len(bad) else 0
u, so, rows = om.integrate(T[i], Asv[i], U0[i], 10.0, analytic_jac=True, record=True)
ns = int(st["nsteps"][i])
print("reactor", i, "gpu steps", ns, "orc steps", so["nsteps"])
for k in list(range(0, min(ns, 40))) + list(range(max(0, ns - 30), ns + 1)):
    g = tr[i, k]
    o = rows[k] if k < len(rows) else None
    print(k, "gpu t=%.6e h=%.3e q=%d" % (g[0], g[1], g[2]), "orc t=%.6e" % o[0] if o else "")
