"""Solver-counter and per-phase cycle breakdown of the HIP integrator on a synthetic ensemble.
Usage: python scripts/diag_perf.py [case] [N]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# per-phase shader clocks are compiled only into the diagnostic build
os.environ.setdefault("BRHIP_LIB", os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_diag.so"))
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
case = sys.argv[1] if len(sys.argv) > 1 else "gri"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat", "surf": None, "gas_surf": "grimech.dat"}[case]
surf = "ch4ni.xml" if case in ("surf", "gas_surf") else None
SG = "CH4 H2O H2 CO CO2 O2 N2".split()
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas, surface_mech=surf, gasphase=None if gas else SG)
eng = pkg.Engine(pm)
print("launch:", eng.launch_info)
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
t0 = time.perf_counter()
U, st = eng.integrate(T, Asv, U0, 10.0)
dt = time.perf_counter() - t0
print(f"{case} N={N}: {dt:.3f} s wall, {N/dt:.1f} reactors/s")
bad = np.nonzero(st["status"] != 0)[0]
print("failed:", bad[:20], st["status"][bad[:20]], "T", T[bad[:20]])
for k in ("nsteps", "nfe", "nje", "nsetups", "nni", "ncfn", "netf"):
    v = st[k]
    print(f"  {k:8s} mean {v.mean():9.1f} p50 {np.median(v):8.0f} p99 {np.percentile(v, 99):8.0f} max {v.max():8.0f}")
tot = st["cyc_total"] / 100e6
print(f"  wave time ms: mean {tot.mean()*1e3:.2f} p50 {np.median(tot)*1e3:.2f} max {tot.max()*1e3:.2f}")
clk = np.sum(st["cyc_clk"])
print(f"  shader clocks per reactor {clk/N:.4g} (clock ratio to 100 MHz wall: {clk/np.sum(st['cyc_total']):.1f})")
for ph, cnt in (("rhs", "nfe"), ("jac", "nje"), ("lu", "nsetups"), ("sol", "nni"), ("ctl", "nfe")):
    c = st["cyc_" + ph]
    print(f"  {ph:4s} cycles/call {np.sum(c)/max(np.sum(st[cnt]),1):10.0f}  share of clock {np.sum(c)/clk:.3f}")
rest = clk - sum(np.sum(st["cyc_" + ph]) for ph in ("rhs", "jac", "lu", "sol", "ctl"))
print(f"  rest (init, loop glue): share {rest/clk:.3f}")
i = int(np.argmax(st["nsteps"]))
print("slowest reactor", i, "T", T[i], {k: float(st[k][i]) for k in pkg.STAT_FIELDS})
