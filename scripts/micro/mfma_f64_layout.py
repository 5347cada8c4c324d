"""Which lane map does v_mfma_f64_16x16x4f64 use? Feeds lane-tagged operands and prints the
accumulator map that reproduces D = C + A B (scripts/micro/mfma_f64_layout.hip)."""
import ctypes as C
import itertools
import os
import numpy as np

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_layout.so"))
rng = np.random.default_rng(1)
a = rng.integers(-8, 8, 64).astype(float)
b = rng.integers(-8, 8, 64).astype(float)
c = np.zeros((4, 64))
d = np.zeros((4, 64))
dp = lambda x: x.ctypes.data_as(C.c_void_p)
assert lib.mfma_f64_layout(dp(a), dp(b), dp(c), dp(d)) == 0
L = np.arange(64)
# candidate operand maps: A[m][k], B[k][n] from (m, k) = (l & 15, l >> 4) or (l >> 2, l & 3) ...
maps = {"lo4": (L & 15, L >> 4), "hi": (L >> 2, L & 3)}
cmaps = {"n=l&15,m=(l>>4)+4i": lambda i: ((L >> 4) + 4 * i, L & 15),
         "n=l&15,m=4(l>>4)+i": lambda i: (4 * (L >> 4) + i, L & 15),
         "m=l&15,n=(l>>4)+4i": lambda i: (L & 15, (L >> 4) + 4 * i),
         "m=l&15,n=4(l>>4)+i": lambda i: (L & 15, 4 * (L >> 4) + i)}
for (an, (am, ak)), (bn, (bn_, bk)) in itertools.product(maps.items(), maps.items()):
    A = np.zeros((16, 4)); B = np.zeros((4, 16))
    A[am, ak] = a
    B[bk, bn_] = b
    D = A @ B
    for cn, f in cmaps.items():
        ok = all(np.array_equal(D[f(i)[0], f(i)[1]], d[i]) for i in range(4))
        if ok:
            print("MATCH A", an, "B", bn, "C/D", cn)
print("done")
