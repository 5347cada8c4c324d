"""GPU-vs-oracle step-by-step diagnostic: traces of accepted steps, solver counters and
per-phase cycle counts of the HIP kernel. Usage: python scripts/diag_integrate.py [case] [N]"""
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
case = sys.argv[1] if len(sys.argv) > 1 else "h2o2"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat", "surf": None}[case]
surf = "ch4ni.xml" if case == "surf" else None
SG = "CH4 H2O H2 CO CO2 O2 N2".split()
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas, surface_mech=surf, gasphase=None if gas else SG)
om = oracle.Mech(os.path.join(LIB, gas) if gas else None, os.path.join(LIB, "therm.dat"),
                 os.path.join(LIB, surf) if surf else None, gas_species=None if gas else SG)
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
cap = 4000
U, st, tr = eng.integrate(T, Asv, U0, 10.0, trace_cap=cap)
np.set_printoptions(precision=4, linewidth=160)
for i in range(N):
    uo, so, rows = om.integrate(T[i], Asv[i], U0[i], 10.0, analytic_jac=True, record=True)
    g = {k: st[k][i] for k in pkg.STAT_FIELDS}
    print(f"--- reactor {i} T={T[i]:.1f} status gpu {g['status']:.0f} orc {so['status']}")
    for k in ("nsteps", "nfe", "nje", "nsetups", "nni", "ncfn", "netf"):
        print(f"   {k:8s} gpu {g[k]:8.0f}  orc {so[k]:8d}")
    ct = g["cyc_total"] / 100e6
    print(f"   time {ct*1e3:.2f} ms  rhs {g['cyc_rhs']:.3e} jac {g['cyc_jac']:.3e} lu {g['cyc_lu']:.3e} "
          f"sol {g['cyc_sol']:.3e} cycles; per-call rhs {g['cyc_rhs']/max(g['nfe'],1):.0f} "
          f"jac {g['cyc_jac']/max(g['nje'],1):.0f} lu {g['cyc_lu']/max(g['nsetups'],1):.0f} "
          f"sol {g['cyc_sol']/max(g['nni'],1):.0f}")
    # first divergence in the accepted-step sequence
    ns = int(min(g["nsteps"], so["nsteps"], cap))
    first = None
    for s in range(1, ns + 1):
        tg, to = tr[i, s, 0], rows[s][0]
        if abs(tg / to - 1) > 1e-6:
            first = s
            break
    if first is None:
        print(f"   step times agree to 1e-6 for all {ns} compared steps")
    else:
        s = first
        print(f"   first step-time divergence at step {s}: gpu t={tr[i, s, 0]:.6e} h={tr[i, s, 1]:.3e} q={tr[i, s, 2]:.0f}"
              f" | orc t={rows[s][0]:.6e}; prev gpu t={tr[i, s-1, 0]:.6e} orc {rows[s-1][0]:.6e}")
        ug, uo_ = tr[i, s - 1, 4:], rows[s - 1][1]
        big = np.abs(uo_) > 1e-8 * np.abs(uo_).max()
        print(f"   state rel diff at step {s-1}: {np.max(np.abs(ug[big]/uo_[big]-1)):.3e}")
    big = np.abs(uo) > 1e-8 * np.abs(uo).max()
    print(f"   final rel diff {np.max(np.abs(U[i][big] / uo[big] - 1)):.3e}")
