"""How often does a factorization's pivot order differ from the previous factorization's? (oracle
diagnostic, orc_lu_diag). Sets the cost model of an LU that expects each step's pivot on its position
when the rows are loaded in the previous pivot order. Usage: python scripts/lu_order_stats.py CASE N"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import _pkgload  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import _mechs  # noqa: E402

case, N = sys.argv[1], int(sys.argv[2])
dq = len(sys.argv) > 3 and sys.argv[3] == "dq"
pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402
pm, om = _mechs(pkg, oracle, case)
L = C.CDLL(oracle.LIB)
L.orc_lu_diag.argtypes = [C.c_int]
out = (C.c_long * 8)()
T, Asv, U0 = ensemble.make_inputs(pm, case, 0, N)
tot = np.zeros(8)
for i in range(N):
    L.orc_lu_diag(1)
    om.integrate(T[i], Asv[i], U0[i], 10.0, analytic_jac=not dq)
    L.orc_lu_stats(out)
    tot += np.array(out[:])
print(f"{case} N={N} {'DQ' if dq else 'analytic'}: factorizations {tot[0]:.0f} ({tot[0]/N:.1f}/reactor), "
      f"deviating {tot[1]:.0f} ({tot[1]/tot[0]*100:.2f} %), steps {tot[2]:.0f}, interchanges {tot[3]:.0f} "
      f"({tot[3]/tot[2]*100:.3f} % of steps; {tot[3]/N:.1f}/reactor); first factorization {tot[6]/N:.1f}; "
      f"hi-word ties of the column max {tot[7]:.0f} ({tot[7]/tot[0]:.2f}/LU); restart cost in steps per reactor: whole LU "
      f"{tot[4]/N:.0f}, from the panel start {tot[5]/N:.0f} (steps per reactor {tot[2]/N:.0f})")
