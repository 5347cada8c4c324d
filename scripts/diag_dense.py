"""GPU diagnostic: per-output-time errors of the engine against the oracle (dense output through
br_opts.tout), step counts and ignition times, for a few reactors of one config."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402
import oracle  # noqa: E402

pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
SG = "CH4 H2O H2 CO CO2 O2 N2".split()
case = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat", "gas_surf": "grimech.dat", "surf": None}[case]
surf = "ch4ni.xml" if case in ("gas_surf", "surf") else None
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas, surface_mech=surf, gasphase=None if gas else SG)
om = oracle.Mech(os.path.join(LIB, gas) if gas else None, os.path.join(LIB, "therm.dat"),
                 os.path.join(LIB, surf) if surf else None, gas_species=None if gas else SG)
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
tout = np.concatenate([[1e-6, 1e-5, 1e-4], np.logspace(-3, 1, 25)])
U, st = eng.integrate(T, Asv, U0, 10.0, tout=tout)
for i in range(N):
    uo, so, Yo = om.integrate_out(T[i], Asv[i], U0[i], 10.0, tout, analytic_jac=eng.engine == "wave")
    Y = st["yout"][i]
    e = (np.abs(Y - Yo) / (1e-4 * np.abs(Yo) + 1e-8)).max(axis=1)
    k = (np.abs(Y - Yo) / (1e-4 * np.abs(Yo) + 1e-8)).argmax(axis=1)
    print(f"reactor {i} engine {eng.engine} steps {st['nsteps'][i]:.0f}/{so['nsteps']} nfe {st['nfe'][i]:.0f}/{so['nfe']} "
          f"netf {st['netf'][i]:.0f}/{so['netf']} nje {st['nje'][i]:.0f}/{so['nje']} t_ign {st['t_ign'][i]:.6e}/{so['t_ign']:.6e}")
    for j in range(len(tout)):
        print(f"   t={tout[j]:.3e} err={e[j]:.3e} sp={pm.species[k[j]]} gpu={Y[j, k[j]]:.6e} orc={Yo[j, k[j]]:.6e} "
              f"sumgpu={np.abs(Y[j]).sum():.6e}")
print("final U err", np.max(np.abs(U - np.array([om.integrate(T[i], Asv[i], U0[i], 10.0, analytic_jac=eng.engine == 'wave')[0] for i in range(N)])) /
                            (1e-4 * np.abs(U) + 1e-8)))
