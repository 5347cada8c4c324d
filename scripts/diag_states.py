"""RHS / Jacobian / LU-solve parity of the HIP kernels on states taken from an oracle trajectory
(late, near-equilibrium states included). Usage: python scripts/diag_states.py case index"""
import ctypes as C
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
case, idx = sys.argv[1], int(sys.argv[2])
gas = {"h2o2": "h2o2.dat", "gri": "grimech.dat"}[case]
pm = pkg.Mechanism.from_files(LIB, gas_mech=gas)
om = oracle.Mech(os.path.join(LIB, gas), os.path.join(LIB, "therm.dat"))
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, idx + 1)
T0, A0 = T[idx], Asv[idx]
uo, so, rows = om.integrate(T0, A0, U0[idx], 10.0, analytic_jac=True, record=True)
sel = list(range(1, len(rows), max(1, len(rows) // 40)))
U = np.stack([rows[s][1] for s in sel])
N = len(sel)
du = eng.rhs(np.full(N, T0), np.full(N, A0), U)
J = eng.jacobian(np.full(N, T0), np.full(N, A0), U)
n = pm.n
L = pkg._lib.lib()
for i, s in enumerate(sel):
    do, _, _ = om.rhs(T0, A0, U[i])
    Jo = om.jac(T0, A0, U[i])
    erhs = np.max(np.abs(du[i] - do) / (np.abs(do) + 1e-300 + np.abs(do).max() * 1e-14))
    ej = np.max(np.abs(J[i] - Jo) / (np.abs(Jo).max(1, keepdims=True) + 1e-300))
    h = rows[s + 1][0] - rows[s][0] if s + 1 < len(rows) else rows[s][0] - rows[s - 1][0]
    gam = np.array([h])
    b = np.random.default_rng(s).standard_normal((1, n))
    x = np.zeros((1, n))
    f = np.zeros(1, np.int32)
    Jc = np.ascontiguousarray(Jo[None])
    L.br_debug_lu_solve(1, n, pkg._lib.dptr(Jc), pkg._lib.dptr(gam), pkg._lib.dptr(b), pkg._lib.dptr(x),
                        f.ctypes.data_as(C.POINTER(C.c_int)))
    A = np.eye(n) - h * Jo
    xr = np.linalg.solve(A, b[0])
    ex = np.max(np.abs(x[0] - xr)) / np.max(np.abs(xr))
    print(f"step {s:5d} t={rows[s][0]:.4e} h={h:.3e} rhs_err {erhs:.2e} jac_err {ej:.2e} "
          f"solve_err {ex:.2e} cond {np.linalg.cond(A):.2e} minu {U[i].min():.2e}")
