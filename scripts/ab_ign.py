"""Cost of the per-step ignition tracking (track_ignition: max dX_OH/dt, br_stats.t_ign) in the
integrator: kernel time with and without it (br_opts.ignition_species = 0), alternating.
  python3 scripts/ab_ign.py CONFIG N"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import _pkgload  # noqa: E402
import bench  # noqa: E402

cfg, N = sys.argv[1], int(sys.argv[2])
pkg = _pkgload.load()
mech = bench.make_mech(pkg, cfg)
eng = pkg.Engine(mech)
T, A, U0 = bench.ensemble_inputs(pkg, mech, cfg, N)
tf = bench.CONFIGS[cfg]["tf"]
ign = eng.ign1
res = {"on": [], "off": []}
eng.integrate(T, A, U0, tf)
for it in range(3):
    for k in ("on", "off"):
        eng.ign1 = ign if k == "on" else 0
        eng.integrate(T, A, U0, tf)
        res[k].append(eng.last_kernel_ms())
out = {"config": cfg, "N": N, "kernel_ms": res, "off_vs_on": min(res["on"]) / min(res["off"])}
print(json.dumps(out))
