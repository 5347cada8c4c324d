"""Per-component GPU-vs-oracle differences on the parity-test inputs (tests/test_gpu_parity.py).
Usage: python scripts/diag_parity.py case N [rtol atol tf]"""
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
case, N = sys.argv[1], int(sys.argv[2])
rtol = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-6
atol = float(sys.argv[4]) if len(sys.argv) > 4 else 1e-10
tf = float(sys.argv[5]) if len(sys.argv) > 5 else 10.0
pm, om = _mechs(pkg, oracle, case)
eng = pkg.Engine(pm)
T, Asv, U0 = _ignition_inputs(pm, case, N, 5)
U, st = eng.integrate(T, Asv, U0, tf, rtol=rtol, atol=atol)
Ua, sa, _ = om.integrate_batch(T, Asv, U0, tf, rtol=rtol, atol=atol, analytic_jac=True, nthreads=8)
Ud, sd, _ = om.integrate_batch(T, Asv, U0, tf, rtol=rtol, atol=atol, analytic_jac=False, nthreads=8)
names = pm.gas_species + [f"s{i}" for i in range(pm.ns)]
Ut, stt, _ = om.integrate_batch(T, Asv, U0, tf, rtol=1e-10, atol=1e-14, analytic_jac=True, nthreads=8)
for i in range(N):
    fl = 1e-6 * np.abs(Ut[i]).max()
    eg = np.abs(U[i] - Ut[i]) / (np.abs(Ut[i]) + fl)
    ea = np.abs(Ua[i] - Ut[i]) / (np.abs(Ut[i]) + fl)
    k = int(np.argmax(eg))
    print(f"{i}: global err gpu {eg.max():.3e} ({names[k]}: gpu {U[i,k]:.6e} true {Ut[i,k]:.6e} orc {Ua[i,k]:.6e}) orc {ea.max():.3e}")
for i in range(N):
    e = np.abs(U[i] - Ua[i]) / (1e-4 * np.abs(Ua[i]) + 100 * atol)
    e2 = np.abs(Ud[i] - Ua[i]) / (1e-4 * np.abs(Ua[i]) + 100 * atol)
    k = int(np.argmax(e))
    print(f"{i}: gpu-vs-orc {e.max():8.3f} ({names[k]} gpu {U[i,k]:.6e} orc {Ua[i,k]:.6e} dq {Ud[i,k]:.6e}) "
          f"| dq-vs-an {e2.max():8.3f}  steps gpu {st['nsteps'][i]:.0f} an {sa[i]['nsteps']} dq {sd[i]['nsteps']}")
