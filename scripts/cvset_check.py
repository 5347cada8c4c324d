"""Bit-for-bit check of the 16-lane groups' lane-parallel cvSet and step-size ratios against the
generic forms on random controller states (scripts/micro/cvset_check.hip)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(3)
iin = np.zeros((N, 4), np.int32)
iin[:, 0] = rng.integers(1, 6, N)          # q
iin[:, 1] = rng.integers(0, 3, N)          # qwait
iin[:, 2] = rng.choice([0, 7], N)          # nst
din = np.zeros((N, 10))
h = 10.0 ** rng.uniform(-9, -2, N)
din[:, 0] = h
din[:, 1] = h * rng.uniform(0.2, 5.0, N) * 0.3      # gammap
for i in range(1, 7):
    din[:, 2 + i] = h * rng.uniform(0.3, 3.0, N)   # tau[1..6]
din[:, 9] = 10.0 ** rng.uniform(-3, 1, N)            # dsm
lib = C.CDLL(os.path.join(ROOT, "scripts", "micro", "libcvset_check.so"))
out = np.zeros((N, 16, 2, 16))
rc = lib.cvset_check(N, din.ctypes.data_as(C.c_void_p), iin.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
assert rc == 0, rc
names = ["l0", "l1", "l2", "l3", "l4", "l5", "tq1", "tq2", "tq3", "tq4", "tq5", "rl1", "gamma", "gamrat", "tq4_out", "eta_sum"]
a, b = out[:, :, 0, :], out[:, :, 1, :]
diff = a.view(np.int64) != b.view(np.int64)
res = {nm: int(diff[:, :, i].any(axis=1).sum()) for i, nm in enumerate(names)}
lanes = {nm: int((a[:, :, i].view(np.int64) != a[:, :1, i].view(np.int64)).any(axis=1).sum()) for i, nm in enumerate(names)}
print(json.dumps({"cases": N, "cases_differing_per_field": res, "generic_lane_spread_cases": lanes}))
bad = np.nonzero(diff.any(axis=(1, 2)))[0]
for c in bad[:5]:
    f = np.nonzero(diff[c, 0])[0]
    print("case", c, "q qwait nst", iin[c].tolist()[:3], [(names[i], a[c, 0, i], b[c, 0, i]) for i in f])
