"""Where a GPU trajectory leaves the oracle's: for given bench reactors, the per-step rows of the
wavefront engine's traced run (br_integrate_traced: t, h, q, accepted u) against the oracle's step
callback rows (same Jacobian kind), the first accepted step whose t or state differs beyond a
tolerance, and the solver counters of both runs. Diagnostic for scripts/parity_outliers.py's outliers.

  python3 scripts/dq_diverge.py CONFIG REACTOR [REACTOR ...] [--analytic] [--rtol R]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "scripts")]
import _pkgload  # noqa: E402
import bench  # noqa: E402
from parity_outliers import oracle_mech  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("reactors", type=int, nargs="+")
    ap.add_argument("--analytic", action="store_true")
    ap.add_argument("--rtol", type=float, default=1e-6)
    ap.add_argument("--tol", type=float, default=1e-9, help="relative state difference that counts as diverged")
    args = ap.parse_args()
    pkg = _pkgload.load()
    mech, om = oracle_mech(pkg, args.config)
    eng = pkg.Engine(mech)
    K = max(args.reactors) + 1
    T, A, U0 = bench.ensemble_inputs(pkg, mech, args.config, K)
    tf = bench.CONFIGS[args.config]["tf"]
    n = mech.n
    out = []
    for i in args.reactors:
        uo, so, rows = om.integrate(T[i], A[i], U0[i], tf, rtol=args.rtol, analytic_jac=args.analytic, record=True)
        cap = int(so["nsteps"]) + 200
        ug, sg, tr = eng.integrate(T[i:i + 1], A[i:i + 1], U0[i:i + 1], [tf], rtol=args.rtol, trace_cap=cap,
                                   dq_jacobian=not args.analytic)
        ng = int(sg["nsteps"][0])
        tg, hg, qg, Ug = tr[0, :ng + 1, 0], tr[0, :ng + 1, 1], tr[0, :ng + 1, 2], tr[0, :ng + 1, 4:4 + n]
        to = np.array([r[0] for r in rows])
        Uo = np.array([r[1] for r in rows])
        m = min(len(to), len(tg))
        first = None
        for k in range(m):
            dt = abs(tg[k] - to[k]) / max(abs(to[k]), 1e-300)
            du = float(np.max(np.abs(Ug[k] - Uo[k]) / (np.abs(Uo[k]) + 1e-20)))
            if dt > args.tol or du > args.tol:
                first = {"step": k, "t_gpu": float(tg[k]), "t_orc": float(to[k]), "rel_dt": float(dt),
                         "max_rel_du": du, "h_gpu": float(hg[k]), "q_gpu": int(qg[k]),
                         "prev_rel_du": float(np.max(np.abs(Ug[k - 1] - Uo[k - 1]) / (np.abs(Uo[k - 1]) + 1e-20)))
                         if k else 0.0}
                break
        rec = {"reactor": i, "T": float(T[i]), "steps": [ng, int(so["nsteps"])],
               "nfe": [int(sg["nfe"][0]), int(so["nfe"])], "nje": [int(sg["nje"][0]), int(so["nje"])],
               "nsetups": [int(sg["nsetups"][0]), int(so["nsetups"])], "netf": [int(sg["netf"][0]), int(so["netf"])],
               "ncfn": [int(sg["ncfn"][0]), int(so["ncfn"])],
               "t_ign": [float(sg["t_ign"][0]), float(so["t_ign"])], "first_divergence": first}
        # rows around the divergence
        if first:
            k0 = max(0, first["step"] - 3)
            rec["rows"] = [{"k": k, "t": [float(tg[k]), float(to[k])],
                            "rel_du": float(np.max(np.abs(Ug[k] - Uo[k]) / (np.abs(Uo[k]) + 1e-20)))}
                           for k in range(k0, min(m, first["step"] + 4))]
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
