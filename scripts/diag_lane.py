"""Lane-engine timing anatomy (H2/O2 C2 workload): kernel time, per-reactor wall ticks
(100 MHz) against step counts, and the straggler tail (reactors that hit max_steps)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkgload
pkg = _pkgload.load()
from batchreactor_amd import ensemble

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
ms = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "lib")
m = pkg.Mechanism.from_files(lib, gas_mech="h2o2.dat")
eng = pkg.Engine(m)
print("engine", eng.engine)
T, Asv, U0 = ensemble.make_inputs(m, "h2o2", 0, N)
t0 = time.time()
U, st = eng.integrate(T, Asv, U0, 10.0, max_steps=ms)
print(f"N={N} max_steps={ms} wall {time.time()-t0:.3f} s")
ns, tk, s = st["nsteps"], st["cyc_total"] / 1e8, st["status"]
print("status", {int(k): int(v) for k, v in zip(*np.unique(s, return_counts=True))})
print(f"steps mean {ns.mean():.1f} p50 {np.median(ns):.0f} p99 {np.percentile(ns, 99):.0f} max {ns.max():.0f}")
print(f"reactor wall s: mean {tk.mean():.4f} p50 {np.median(tk):.4f} p99 {np.percentile(tk, 99):.4f} max {tk.max():.4f}")
per = tk / np.maximum(ns, 1)
print(f"us per step (lane view): p50 {1e6*np.median(per):.2f} mean {1e6*per.mean():.2f}")
big = ns >= 0.5 * ms
print(f"reactors with >= max_steps/2 steps: {big.sum()}, their wall s {tk[big].round(3)[:10]}")
print("sum steps", ns.sum(), "frac in stragglers", ns[big].sum() / ns.sum())
if st["cyc_clk"].max() > 0:   # diagnostic build (BRHIP_LIB=.../libbrhip_diag.so): shader clocks per phase
    ok = s == 0
    tot = st["cyc_clk"][ok].sum()
    for k, lab in (("cyc_rhs", "rhs"), ("cyc_jac", "refill/init"), ("cyc_lu", "lu"), ("cyc_sol", "solve"), ("cyc_ctl", "controller")):
        print(f"{lab:12s} {st[k][ok].sum() / tot:6.3f}")
    it = (st["nfe"] + st["nje"] * m.n)[ok]
    print(f"clocks per iteration (wave view): {tot / it.sum():.0f}")
