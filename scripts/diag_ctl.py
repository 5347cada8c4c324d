"""Controller sub-phase clocks (profiling build libbrhip_prof.so, see git log): per-step costs."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BRHIP_LIB", os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_prof.so"))
import _pkgload  # noqa: E402
pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402
LIB = os.path.join(ROOT, "tests", "golden", "lib")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
pm = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat")
eng = pkg.Engine(pm)
T, Asv, U0 = ensemble.make_inputs(pm, "gri", 0, N)
U, st = eng.integrate(T, Asv, U0, 10.0)
nst = 965.0 * N
clk = np.sum(st["cyc_clk"])
print("clock/reactor", clk / N, "ctl share", np.sum(st["cyc_ctl"]) / clk)
for k, name in (("nsteps", "begin_step"), ("nje", "prepare_next(eta)"), ("nsetups", "cv_set"), ("nni", "cv_predict"), ("ncfn", "conv test")):
    print(f"  {name:20s} share {np.sum(st[k])/clk:.3f}  cycles/step {np.sum(st[k])/nst:.0f}")
