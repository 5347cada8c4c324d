"""Sub-phase clock split of the integrator (diagnostic build, BR_SUB_ADD slots in
brhip_device.hpp): cycles per call of each instrumented sub-phase next to the phase totals.
Usage: python scripts/diag_sub.py [config] [N]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BRHIP_LIB", os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_diag.so"))
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from bench import CONFIGS, ensemble_inputs, make_mech  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "gri"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
SLOTS = {0: ("LU panel 1", "nsetups"), 1: ("LU panel 2", "nsetups"), 2: ("LU gather", "nsetups"),
         6: ("J multipliers", "nje"), 3: ("ctl post_rhs", "nfe"), 4: ("J entries", "nje"), 5: ("J col write", "nje"),
         7: ("ctl begin_step", "nsteps"), 8: ("ctl conv+err test", "nni"), 9: ("ctl complete+prep", "nsteps"),
         10: ("ctl ign/unst/tstop", "nsteps"), 11: ("RHS setup", "nfe"), 12: ("RHS production", "nfe"),
         13: ("ctl post_solve (group engines)", "nni")}
mech = make_mech(pkg, cfg)
eng = pkg.Engine(mech)
lib = ctypes.CDLL(os.environ["BRHIP_LIB"])
out = (ctypes.c_double * 16)()
T, Asv, U0 = ensemble_inputs(pkg, mech, cfg, N)
lib.br_diag_sub(out)
U, st = eng.integrate(T, Asv, U0, CONFIGS[cfg]["tf"])
lib.br_diag_sub(out)
for ph, cnt in (("rhs", "nfe"), ("jac", "nje"), ("lu", "nsetups"), ("sol", "nni"), ("ctl", "nni")):
    print(f"{ph:4s} cycles/call {np.sum(st['cyc_' + ph]) / np.sum(st[cnt]):10.0f}")
for i, (name, cnt) in SLOTS.items():
    print(f"  {name:12s} cycles/call {out[i] / np.sum(st[cnt]):10.0f}")
