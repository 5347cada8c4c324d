#!/usr/bin/env python3
"""A/B bit-identity check of libbrhip builds: integrates the first N reactors of a bench config
with each library (one child process per build, BRHIP_LIB), then compares the final states and
solver counters bitwise against the first build.

  python3 scripts/bitcmp.py --config gri --n 4000 head new1 new2   (names: libbrhip_<name>.so,
                                                                      "cur" = libbrhip.so)
"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(config, n, out):
    import _pkgload
    import bench
    pkg = _pkgload.load()
    from batchreactor_amd import ensemble
    mech = bench.make_mech(pkg, config)
    eng = pkg.Engine(mech, device=0)
    T, Asv, U0 = ensemble.make_inputs(mech, config, 0, n)
    tf = np.full(n, bench.CONFIGS[config]["tf"])
    U, st = eng.integrate(T, Asv, U0, tf)
    keys = ("nsteps", "nfe", "nje", "nsetups", "nni", "status")
    np.savez(out, U=U, **{k: st[k] for k in keys})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gri")
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--child", default=None)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.config, a.n, a.child)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res = {}
    for v in a.libs:
        lib = os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip.so" if v == "cur" else f"libbrhip_{v}.so")
        out = os.path.join(ROOT, "gpurun_out", f"bit_{a.config}_{v}.npz")
        env = dict(os.environ, BRHIP_LIB=lib)
        subprocess.run([sys.executable, __file__, "--config", a.config, "--n", str(a.n), "--child", out],
                       check=True, env=env, timeout=600)
        res[v] = np.load(out)
    ref = a.libs[0]
    for v in a.libs[1:]:
        same = np.array_equal(res[ref]["U"].view(np.int64), res[v]["U"].view(np.int64))
        diff = np.abs(res[ref]["U"] - res[v]["U"]) / (np.abs(res[ref]["U"]) * 1e-4 + 1e-8)
        cnt = {k: int(np.sum(res[ref][k] != res[v][k])) for k in ("nsteps", "nfe", "nje", "nsetups", "status")}
        print(f"{a.config} {v} vs {ref}: bit-identical={same} reactors_differing={int(np.sum(np.any(res[ref]['U'] != res[v]['U'], axis=1)))} "
              f"max_band={float(diff.max()):.3g} counters_differing={cnt} "
              f"steps {res[ref]['nsteps'].sum():.0f} -> {res[v]['nsteps'].sum():.0f}")


if __name__ == "__main__":
    main()
