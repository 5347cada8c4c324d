"""RHS / Jacobian sub-phase clocks from the profiling build (libbrhip_prof.so, a throwaway copy of
the kernel with clock64 probes; see git log). Prints clocks per call."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BRHIP_LIB", os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_prof.so"))
import _pkgload  # noqa: E402
pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402
LIB = os.path.join(ROOT, "tests", "golden", "lib")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
pm = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat")
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, "gri", 0, N)
U, st = eng.integrate(T, Asv, U0, 10.0)
nje_true = None
nfe = np.sum(st["nfe"]); nje = 21.08 * N   # nje slot is overwritten in this build; GRI mean from the product build
print("rhs total/call", np.sum(st["cyc_rhs"]) / nfe)
print("  conc+Ctot+third-body /call", np.sum(st["nsteps"]) / nfe)
print("  production /call", np.sum(st["nje"]) / nfe)
print("jac total/call", np.sum(st["cyc_jac"]) / nje, " column loop/call", np.sum(st["nsetups"]) / nje)
