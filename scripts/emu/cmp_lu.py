"""GPU lu_factor_mf (br_debug_lu_factor in the variant library libbrhip_lumf.so) against the lane-level emulation: first differing
column of the factor matrix, per matrix. Usage (GPU box): python3 scripts/emu/cmp_lu.py [n] [twice]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _pkgload  # noqa: E402
import lu_mf_emu as E  # noqa: E402

pkg = _pkgload.load()
L = C.CDLL(os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_lumf.so"))
f = L.br_debug_lu_factor
f.restype = C.c_int
n = int(sys.argv[1]) if len(sys.argv) > 1 else 53
twice = int(sys.argv[2]) if len(sys.argv) > 2 else 0
stop = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
PW = int(os.environ.get("PW", "8"))
NMAX = 56 if n <= 56 else 64
lw = NMAX * NMAX + 64
N = 3
rng = np.random.default_rng(n)
J = rng.standard_normal((N, n, n)) * np.exp(rng.uniform(-8, 8, (N, n, 1)))
g = np.exp(rng.uniform(-12, -2, N))
F = np.zeros((N, lw))
P = np.zeros((N, 64), np.int32)
dp = lambda a: a.ctypes.data_as(C.c_void_p)
rc = f(N, n, dp(J), dp(g), twice, stop, dp(F), dp(P))
assert rc == 0, rc
for i in range(N):
    Jt = np.zeros(NMAX * 64)
    for j in range(n):
        Jt[j * 64:j * 64 + n] = J[i][:, j]
    Fe = np.full(NMAX * NMAX, np.nan)
    De = np.zeros(64)
    fl, perm = E.lu_factor_mf(Jt, Fe, De, g[i], n, np.arange(64), NMAX, PW, stop)
    if twice:
        fl, perm = E.lu_factor_mf(Jt, Fe, De, g[i], n, perm, NMAX, PW)
    Mg = F[i, :NMAX * NMAX].reshape(NMAX, NMAX)
    Me = Fe.reshape(NMAX, NMAX)
    print(f"matrix {i}: perm equal {np.array_equal(P[i][:n], perm[:n])}")
    if stop < 100:
        for c in range(n):
            d = np.abs(Mg[c, :n] - Me[c, :n]) / (np.abs(Me[c, :n]) + 1e-300)
            nb = int(np.sum(~(d < 1e-8)))
            print(f"  col {c}: bad rows {nb}" + (f" e.g. {np.where(~(d < 1e-8))[0][:6].tolist()} gpu {Mg[c, np.where(~(d < 1e-8))[0][:3]]} emu {Me[c, np.where(~(d < 1e-8))[0][:3]]}" if nb else ""))
        continue
    for c in range(n):
        d = np.abs(Mg[c, :n] - Me[c, :n]) / (np.abs(Me[c, :n]) + 1e-300)
        if not np.all(d < 1e-8):
            bad = np.where(~(d < 1e-8))[0]
            print(f"  first bad column {c}: rows {bad[:12].tolist()} gpu {Mg[c, bad[:4]]} emu {Me[c, bad[:4]]}")
            break
    else:
        print("  factor matrix agrees")
    dd = np.abs(F[i, NMAX * NMAX:NMAX * NMAX + n] - De[:n])
    print("  D^-1 max diff", dd.max())
