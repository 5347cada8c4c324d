"""Per-reactor cost vs inputs for the strong-scaling tail analysis: integrates a config's
ensemble sample on the GPU and saves T, p, phi, counters and wall cycles per reactor to
gpurun_out/cost_<config>.npz.   Usage: python scripts/diag_cost.py [config] [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402
sys.path.insert(0, ROOT)
from bench import make_mech  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "gri"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
mech = make_mech(pkg, cfg)
eng = pkg.Engine(mech)
T, Asv, U0 = ensemble.make_inputs(mech, cfg, 0, N)
u0, u1, u2, u3 = ensemble._draws(0, N)
U, st = eng.integrate(T, Asv, U0, 10.0)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"cost_{cfg}.npz"), T=T, u0=u0, u1=u1, u2=u2, u3=u3,
         **{k: st[k] for k in ("nsteps", "nfe", "nje", "nsetups", "netf", "status", "cyc_total", "t_ign")})
print("saved", N, "mean cyc", st["cyc_total"].mean(), "max", st["cyc_total"].max())
