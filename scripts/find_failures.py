"""GPU: integrate a config's first N reactors and list the ones that do not return Success
(index, status, steps, t_end, T), writing them to gpurun_out/failures_<config>.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
case = sys.argv[1]
N = int(sys.argv[2])
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat", "surf": None, "gas_surf": "grimech.dat"}[case]
surf = "ch4ni.xml" if case in ("surf", "gas_surf") else None
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas, surface_mech=surf,
                              gasphase=None if gas else "CH4 H2O H2 CO CO2 O2 N2".split())
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
U, st = pkg.Engine(pm).integrate(T, Asv, U0, 10.0)
bad = np.nonzero(st["status"] != 0)[0]
rows = [dict(i=int(i), status=int(st["status"][i]), nsteps=int(st["nsteps"][i]), netf=int(st["netf"][i]),
             t_end=float(st["t_end"][i]), T=float(T[i])) for i in bad]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", f"failures_{case}.json"), "w"), indent=1)
print(len(bad), "failed of", N, rows[:10])
