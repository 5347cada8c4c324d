"""Bench-scale parity: the GPU's per-window deviations from the oracle (tests/parity_bands.py metric)
on the bench's parity samples, set against the oracle's OWN rounding spread on the same reactors, and
every reactor beyond a bound examined one by one. Writes profiles/r06_parity_outliers.json
(VERDICT r05 "Next round" item 1).

  python3 scripts/parity_outliers.py [--configs gri,gas_surf,h2o2,surf] [--out PATH] [--threads T]

Per config and Jacobian kind (analytic = the product default, DQ = CVODE's difference quotients,
the reference's own CVODE_BDF() setting, src/BatchReactor.jl:204-210):

1. sample = the first K reactors of the bench workload (bench.PARITY_SAMPLE, the sizes bench.py's
   parity_vs_oracle block scores), integrated with dense output at parity_bands.OUT_T on the GPU and
   on the oracle (same Jacobian kind, rtol 1e-6 / atol 1e-10).
2. RHS rounding calibration (calibrate()): at oracle states along the sample's trajectories, the
   GPU's RHS deviation from the oracle's, normalised per species by the random-rounding scale
   s_k = sqrt(sum_r (nu_kr q_r M_k)^2) (measured with the oracle's own rop jitter), gives the relative
   per-rate rounding sigma of the GPU's RHS; eps_cal = sigma is the oracle jitter (every rate of
   progress times 1 +- eps, orc_set_rop_jitter) that rounds as differently as the GPU does.
3. the oracle's self-spread on the same sample: R_U0 runs with u0 perturbed by 1e-15 relative and R_J
   runs with the calibrated rop jitter (deterministic per reactor and seed); per-window band errors of
   each against the unperturbed oracle. Proposed bound = 2 x the max over all runs (the rule of
   parity_bands.py, now on the bench-size sample; N stated).
4. every reactor whose GPU deviation exceeds the current bound (parity_bands.BOUNDS) or the proposed
   one: 32 more oracle realisations on that reactor alone (16 u0, 16 jitter seeds) give its own
   spread distribution, and the GPU's deviation is placed in it (rank); the rtol 1e-10 / atol 1e-16
   GPU-vs-oracle check on the same reactor (converged trajectories must agree to 1e-6).
The oracle is the checker here (test infrastructure), as in bench.py's cpu_baseline leg.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import _pkgload  # noqa: E402
import oracle as orc  # noqa: E402
import parity_bands as PB  # noqa: E402
import bench  # noqa: E402

LIB = os.path.join(ROOT, "tests", "golden", "lib")
R_U0, R_J, R_OUT = 2, 4, 16
JIT_UNIT = 4e-16


def band_matrix(Yg, Yo, sto, ok):
    """per reactor (ok ones) the three window maxima; NaN rows for excluded reactors"""
    W = np.full((len(ok), 3), np.nan)
    for i in np.nonzero(ok)[0]:
        W[i] = PB.band_errors(Yg[i], Yo[i], sto[i]["t_ign"])
    return W


def oracle_mech(pkg, config):
    cfg = bench.CONFIGS[config]
    mech = bench.make_mech(pkg, config)
    om = orc.Mech(os.path.join(LIB, cfg["gas"]) if cfg["gas"] else None, os.path.join(LIB, "therm.dat"),
                  os.path.join(LIB, cfg["surf"]) if cfg["surf"] else None,
                  gas_species=None if cfg["gas"] else mech.gas_species)
    return mech, om


def oracle_runs(om, T, A, U0, tf, aj, thr, jitter=0.0, seed=0, rtol=1e-6, atol=1e-10):
    L = orc.lib()
    L.orc_set_rop_jitter(jitter)
    L.orc_set_rop_jitter_seed(seed)
    try:
        _, st, _, Y = om.integrate_batch(T, A, U0, tf, rtol=rtol, atol=atol, analytic_jac=aj, nthreads=thr,
                                         tout=PB.OUT_T)
    finally:
        L.orc_set_rop_jitter(0.0)
        L.orc_set_rop_jitter_seed(0)
    return st, Y


def calibrate(eng, om, T, A, Y, nstate=400, R=8, rng=None):
    """eps_cal: the relative rate-of-progress jitter that rounds as differently as the GPU's RHS does.
    Model: an RHS whose every rate of progress q_r carries a random relative error of size sigma differs
    from the oracle's by f_k - f_orc,k ~ N(0, sigma^2 s_k^2), s_k^2 = sum_r (nu_kr q_r M_k)^2. The oracle's
    jitter at eps = 4e-16 has exactly that form (random signs), so R jittered evaluations per state give
    s_k = rms_R(f_jit,k - f_orc,k) / eps; the GPU's normalised deviation e_k = |f_gpu,k - f_orc,k| / s_k
    then estimates sigma = median(e) / 0.6745: eps_cal (the tails, p90(e) / 1.645 and p99(e), are
    reported beside it)."""
    rng = rng or np.random.default_rng(1)
    N, nt, n = Y.shape
    idx = rng.integers(0, N, nstate)
    tix = rng.integers(0, nt, nstate)
    U = Y[idx, tix]
    fg = eng.rhs(T[idx], A[idx], U)
    fo = np.array([om.rhs(T[i], A[i], U[k])[0] for k, i in enumerate(idx)])
    L = orc.lib()
    L.orc_set_rop_jitter(JIT_UNIT)
    try:
        dj = np.stack([np.array([om.rhs(T[i], A[i], U[k])[0] for k, i in enumerate(idx)]) - fo for _ in range(R)])
    finally:
        L.orc_set_rop_jitter(0.0)
    sk = np.sqrt(np.mean(dj ** 2, axis=0)) / JIT_UNIT
    m = sk > 0
    e = np.abs(fg - fo)[m] / sk[m]
    s50, s90 = float(np.median(e) / 0.6745), float(np.percentile(e, 90) / 1.645)
    return {"states": int(nstate), "jitter_evaluations_per_state": R, "pairs": int(m.sum()),
            "gpu_bitwise_equal_frac": float(np.mean(fg == fo)),
            "sigma_from_median": s50, "sigma_from_p90": s90, "e_p99": float(np.percentile(e, 99)),
            "eps_cal": max(s50, 1.1e-16)}


def summarize(W):
    W = W[np.all(np.isfinite(W), axis=1)]
    return {"reactors": int(len(W)), "max": W.max(0).tolist(), "p99": np.percentile(W, 99, axis=0).tolist(),
            "median": np.median(W, axis=0).tolist()}


def analyse(pkg, eng, mech, om, config, aj, K, thr, log):
    T, A, U0 = bench.ensemble_inputs(pkg, mech, config, K)
    tf = np.full(K, bench.CONFIGS[config]["tf"])
    t0 = time.time()
    sto, Yo = oracle_runs(om, T, A, U0, tf, aj, thr)
    _, stg = eng.integrate(T, A, U0, tf, tout=PB.OUT_T, dq_jacobian=not aj)
    oko = np.array([s["status"] == 0 for s in sto])
    ok = oko & (stg["status"] == 0)
    Wg = band_matrix(stg["yout"], Yo, sto, ok)
    cal = calibrate(eng, om, T, A, Yo)
    log(f"  {config} {'analytic' if aj else 'DQ'}: K={K} GPU max {np.nanmax(Wg, 0)} eps_cal {cal['eps_cal']:.3g} "
        f"({time.time() - t0:.1f} s)")
    # the oracle's own spread on the same sample
    series = []
    rng = np.random.default_rng(20250711)
    for r in range(R_U0):
        Up = U0 * (1 + 1e-15 * rng.standard_normal(U0.shape))
        st, Y = oracle_runs(om, T, A, Up, tf, aj, thr)
        okr = oko & np.array([s["status"] == 0 for s in st])
        series.append(("u0", r, band_matrix(Y, Yo, sto, okr)))
        log(f"    self-spread u0 #{r}: max {np.nanmax(series[-1][2], 0)}")
    for r in range(R_J):
        st, Y = oracle_runs(om, T, A, U0, tf, aj, thr, jitter=cal["eps_cal"], seed=1 + r)
        okr = oko & np.array([s["status"] == 0 for s in st])
        series.append(("jitter", r, band_matrix(Y, Yo, sto, okr)))
        log(f"    self-spread jitter #{r}: max {np.nanmax(series[-1][2], 0)}")
    Wself = np.nanmax(np.stack([w for _, _, w in series]), axis=0)     # per reactor, max over realisations
    self_max = np.nanmax(np.stack([np.nanmax(w, 0) for _, _, w in series]), axis=0)
    proposed = [float(2 * v) for v in self_max]
    cur = list(PB.BOUNDS[(config, not aj)][:3])
    # outliers: beyond the current or the proposed bound
    out_idx = [i for i in np.nonzero(ok)[0] if np.any(Wg[i] > np.minimum(cur, proposed))]
    outliers = []
    for i in out_idx[:16]:
        Ti, Ai, Ui = T[i:i + 1], A[i:i + 1], U0[i:i + 1]
        own = []
        rng_i = np.random.default_rng(1000 + i)
        Up = np.repeat(Ui, R_OUT, axis=0) * (1 + 1e-15 * rng_i.standard_normal((R_OUT, Ui.shape[1])))
        st, Y = oracle_runs(om, np.repeat(Ti, R_OUT), np.repeat(Ai, R_OUT), Up, np.full(R_OUT, tf[i]), aj, thr)
        own += [PB.band_errors(Y[k], Yo[i], sto[i]["t_ign"]) for k in range(R_OUT) if st[k]["status"] == 0]
        for s in range(R_OUT):
            st, Y = oracle_runs(om, Ti, Ai, Ui, tf[i:i + 1], aj, 1, jitter=cal["eps_cal"], seed=100 + s)
            if st[0]["status"] == 0:
                own.append(PB.band_errors(Y[0], Yo[i], sto[i]["t_ign"]))
        own = np.array(own)
        # converged check: rtol 1e-10 / atol 1e-16 on both sides
        stt, Yt = oracle_runs(om, Ti, Ai, Ui, tf[i:i + 1], aj, 1, rtol=1e-10, atol=1e-16)
        _, sgt = eng.integrate(Ti, Ai, Ui, tf[i:i + 1], rtol=1e-10, atol=1e-16, tout=PB.OUT_T, dq_jacobian=not aj)
        Yg_t, Yo_t = sgt["yout"][0], Yt[0]
        dev_t = np.abs(Yg_t - Yo_t) / (1e-6 * np.abs(Yo_t) + 1e-14)    # in 1e-6 bands, per output time
        tight = float(np.max(dev_t))
        tight_end = float(np.max(dev_t[-1]))                              # t = tf (the GPU test's check)
        gw = Wg[i].tolist()
        rank = [float(np.mean(own[:, w] >= gw[w])) if len(own) else None for w in range(3)]
        outliers.append({
            "reactor": int(i), "T": float(T[i]), "gpu_bands": gw, "self_spread_on_sample": Wself[i].tolist(),
            "own_realisations": int(len(own)), "own_spread_max": own.max(0).tolist() if len(own) else None,
            "own_spread_median": np.median(own, 0).tolist() if len(own) else None,
            "frac_own_ge_gpu": rank,
            "t_ign_orc": float(sto[i]["t_ign"]), "t_ign_gpu": float(stg["t_ign"][i]),
            "steps_orc": int(sto[i]["nsteps"]), "steps_gpu": int(stg["nsteps"][i]),
            "tight_rtol1e-10_max_dev_in_1e-6_bands": tight, "tight_rtol1e-10_end_dev_in_1e-6_bands": tight_end,
            "tight_status": [int(stt[0]["status"]), int(sgt["status"][0])],
            "verdict": ("inside the oracle's own spread" if len(own) and np.all(Wg[i] <= own.max(0))
                        else "inside 2x the oracle's own spread" if len(own) and np.all(Wg[i] <= 2 * own.max(0))
                        else "beyond 2x the oracle's own spread")
                       + ("; converged (rtol 1e-10) end states agree to 1e-6" if tight_end <= 1.0
                          else "; converged end states DIFFER beyond 1e-6"),
        })
        log(f"    reactor {i}: gpu {np.round(gw, 3)} own max {np.round(own.max(0), 3) if len(own) else None} "
            f"tight {tight:.3g}")
    # bound: 2x the largest oracle self-deviation seen on these reactors -- the sample's realisations
    # and the 32 per-reactor realisations of every examined reactor
    own_max = np.max([o["own_spread_max"] for o in outliers if o["own_spread_max"]], axis=0) if outliers else 0 * self_max
    bound = [float(2 * max(a, b)) for a, b in zip(self_max, own_max)]
    return {"jacobian": "analytic" if aj else "dq", "sample": int(K), "scored": int(ok.sum()),
            "bound_rule": "2 x max(oracle self-spread over the sample's realisations, per-outlier 32-realisation spread)",
            "bound": bound, "gpu_frac_within_bound": float(np.mean(np.all(Wg[ok] <= np.array(bound), axis=1))),
            "failed_either": int((~ok).sum()), "rhs_calibration": cal,
            "gpu_vs_oracle": summarize(Wg),
            "oracle_self_spread": {"realisations": {"u0_1e-15": R_U0, "rop_jitter_eps_cal": R_J},
                                   **summarize(Wself)},
            "current_bounds": cur, "proposed_bounds": proposed,
            "gpu_frac_within_current": float(np.mean(np.all(Wg[ok] <= np.array(cur), axis=1))),
            "gpu_frac_within_proposed": float(np.mean(np.all(Wg[ok] <= np.array(proposed), axis=1))),
            "outliers": outliers, "outliers_total": len(out_idx)}


class OracleAsGpu:
    """--cpu-dry-run: stands in for the engine with a jittered oracle (seed 999), to check this
    script's logic on a machine without a GPU; its numbers mean nothing"""
    def __init__(self, om, thr):
        self.om, self.thr = om, thr

    def integrate(self, T, A, U0, tf, rtol=1e-6, atol=1e-10, tout=None, dq_jacobian=False):
        st, Y = oracle_runs(self.om, T, A, U0, tf, not dq_jacobian, self.thr, jitter=1e-15, seed=999, rtol=rtol,
                            atol=atol)
        d = {k: np.array([s[k] for s in st]) for k in ("status", "t_ign", "nsteps")}
        d["yout"] = Y
        return None, d

    def rhs(self, T, A, U):
        orc.lib().orc_set_rop_jitter(1e-15)
        try:
            return np.array([self.om.rhs(T[k], A[k], U[k])[0] for k in range(len(T))])
        finally:
            orc.lib().orc_set_rop_jitter(0.0)

    def close(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="gri,gas_surf,h2o2,surf")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r06_parity_outliers.json"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--scale", type=float, default=1.0, help="sample-size factor (quick runs)")
    ap.add_argument("--cpu-dry-run", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    pkg = _pkgload.load()
    res = {"metric": "per reactor, max over the 28 output times of tests/test_gpu_parity.py in each window of "
                     "t/t_ign (pre < 0.5, front 0.5..2, post >= 2) of max_k |Y_a - Y_b| / (1e-4 |Y_b| + 100 atol)",
           "configs": {}}
    log = lambda s: print(s, flush=True)  # noqa: E731
    for config in args.configs.split(","):
        mech, om = oracle_mech(pkg, config)
        eng = OracleAsGpu(om, args.threads) if args.cpu_dry_run else pkg.Engine(mech)
        ka, kd = bench.PARITY_SAMPLE[config]
        res["configs"][config] = {}
        for aj, K in ((True, ka), (False, kd)):
            K = max(8, int(K * args.scale))
            res["configs"][config]["analytic" if aj else "dq"] = analyse(pkg, eng, mech, om, config, aj, K,
                                                                        args.threads, log)
            with open(args.out, "w") as fh:
                json.dump(res, fh, indent=1)
        eng.close()
    print("wrote", args.out)


if __name__ == "__main__":
    main()
