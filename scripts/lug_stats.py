"""Grid-LU event counts on a bench workload (diagnostic build libbrhip_lugstats.so, -DBR_LUG_STATS=1):
factorizations, steps run, pivot handler calls, ties, interchanges. Usage:
  BRHIP_LIB=batchreactor.jl_amd/libbrhip_lugstats.so python3 scripts/lug_stats.py gri 5000"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import _pkgload  # noqa: E402
import bench  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
pkg = _pkgload.load()
from batchreactor_amd import ensemble  # noqa: E402
L = pkg._lib.lib()
f = L.br_debug_lug_stats
f.argtypes = [C.POINTER(C.c_double)]
out = (C.c_double * 8)()
mech = bench.make_mech(pkg, cfg)
eng = pkg.Engine(mech, device=0)
T, Asv, U0 = ensemble.make_inputs(mech, cfg, 0, n)
f(out)
U, st = eng.integrate(T, Asv, U0, np.full(n, bench.CONFIGS[cfg]["tf"]))
f(out)
lu, steps, calls, ties, ich, ksum = out[:6]
print(f"{cfg} N={n}: factorizations {lu:.0f} ({lu / n:.1f}/reactor; nsetups {st['nsetups'].sum() / n:.1f}), "
      f"steps run {steps:.0f} ({steps / max(lu, 1):.1f}/LU, n = {mech.n}), handler calls {calls:.0f} "
      f"({calls / max(lu, 1):.3f}/LU), ties {ties:.0f}, interchanges {ich:.0f} ({ich / max(lu, 1):.3f}/LU, mean step "
      f"{ksum / max(ich, 1):.1f})")

if len(sys.argv) > 3:
    d = (C.c_ulonglong * 2048)()
    L.br_debug_lug_dump(d)
    import struct
    for e in range(min(int(sys.argv[3]), 256)):
        I, b0, b1, rm, a0, a1, h0, m = d[8 * e:8 * e + 8]
        rk = I & 3
        f = lambda u: struct.unpack("d", struct.pack("Q", u))[0]
        print(f"I={I:2d} row bits b0={(b0 >> (16 * rk)) & 0xffff:016b} b1={(b1 >> (16 * rk)) & 0xffff:016b} "
              f"rm={rm:08x} pivot-lane h0={h0:08x} m={m:08x} a0={f(a0):.6e} a1={f(a1):.6e}")
