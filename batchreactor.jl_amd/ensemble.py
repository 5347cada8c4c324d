"""Synthetic ensembles and the algorithmic FLOP model used for roofline
accounting.

Inputs are drawn i.i.d. from splitmix64 (seed 20250711), stream index 4*i + j for reactor i,
draw j, so every rank can generate exactly its own contiguous shard.
"""
import numpy as np

SEED = 20250711
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_uniform(idx: np.ndarray, seed: int = SEED) -> np.ndarray:
    """U[0,1) from splitmix64 evaluated at counter `idx` (vectorised, stateless)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * _G
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _draws(start, count):
    i = np.arange(start, start + count, dtype=np.uint64)
    return [splitmix64_uniform(4 * i + j) for j in range(4)]


def make_inputs(mech, config: str, start: int, count: int):
    """Returns T[count], Asv[count], U0[count, n] for reactors [start, start+count)."""
    u0, u1, u2, u3 = _draws(start, count)
    ng = mech.ng
    X = np.zeros((count, ng))
    idx = mech.gas_species.index
    Asv = np.ones(count)
    if config == "h2o2":            # C2
        T = 1000.0 + 400.0 * u0
        p = np.exp(np.log(0.5e5) + (np.log(1e6) - np.log(0.5e5)) * u1)
        phi = np.exp(np.log(0.5) + (np.log(2.0) - np.log(0.5)) * u2)
        X[:, idx("H2")] = 0.5 * 2 * phi / (2 * phi + 1)
        X[:, idx("O2")] = 0.5 / (2 * phi + 1)
        X[:, idx("N2")] = 0.5
    elif config in ("gri", "gas_surf"):   # C3 / C5
        if config == "gri":
            T = 1100.0 + 200.0 * u0
            p = np.exp(np.log(1e5) + (np.log(1e6) - np.log(1e5)) * u1)
        else:
            T = 1100.0 + 150.0 * u0
            p = np.full(count, 1e5)
        phi = 0.5 + u2
        X[:, idx("CH4")] = 0.75 * phi / (phi + 2)
        X[:, idx("O2")] = 1.5 / (phi + 2)
        X[:, idx("N2")] = 0.25
    elif config == "surf":          # C4
        T = 973.0 + 200.0 * u0
        p = np.full(count, 1e5)
        sc = 1.0 + 2.0 * u2
        X[:, idx("CH4")] = 0.5 / (1 + sc)
        X[:, idx("H2O")] = 0.5 * sc / (1 + sc)
        X[:, idx("N2")] = 0.5
        Asv = np.exp(np.log(100.0) * u3)
    else:
        raise ValueError(config)
    Mb = X @ mech.molwt
    rho = p * Mb / (8.31446261815324 * T)
    U0 = np.empty((count, mech.n))
    U0[:, :ng] = X * mech.molwt / Mb[:, None] * rho[:, None]
    U0[:, ng:] = mech.theta0[None, :]
    return T, Asv, U0


def flop_model(mech) -> dict:
    """Algorithmic fp64 FLOPs per operation, counted from the mechanism tables
    (T-only terms hoisted; a transcendental counts as 1 FLOP). SURVEY.md section 8(d)."""
    t = mech.tables
    ng, n = mech.ng, mech.n
    F = 0
    F += 8 * ng                               # rho, Y, x, Mbar, p, c (composition, :326-353)
    tb = t["g_tb"]
    F += int((tb > 0).sum()) + 2 * sum(sum(1 for e in r.efficiencies.values() if e != 1.0) for r in mech.gas_rxns)
    for r in range(mech.nrg):
        F += max(t["g_nf"][r] - 1, 0) + max(t["g_nr"][r] - 1, 0) + 3
        if tb[r] == 1:
            F += 1
        elif tb[r] == 2:
            F += 6 + (16 if t["g_troe_n"][r] else 0)
        F += 2 * (t["g_nf"][r] + t["g_nr"][r])      # stoichiometric scatter
    for r in range(mech.nrs):
        F += 2 * t["s_ncov"][r] + (3 if t["s_ncov"][r] else 0) + t["s_nf"][r] + 1
        F += 2 * (t["s_nf"][r] + t["s_np"][r])
    F += 3 * n                                  # du assembly
    # analytic Jacobian: partial products + scatter; dense third-body columns; unit scaling
    J = 0
    for r in range(mech.nrg):
        e = t["g_nf"][r] + t["g_nr"][r]
        touched = len(set(t["g_f"][r, :t["g_nf"][r]]) | set(t["g_r"][r, :t["g_nr"][r]]))
        J += e * max(e - 2, 1) + 2 * touched * e + 6
        if tb[r]:
            J += 2 * touched * ng + 2
    for r in range(mech.nrs):
        e = t["s_nf"][r]
        touched = len(set(t["s_f"][r, :e]) | set(t["s_p"][r, :t["s_np"][r]]))
        J += e * max(e - 1, 1) + 2 * touched * (e + t["s_ncov"][r])
    J += 2 * n * n
    return dict(rhs=F, jac=J, lu=2.0 * n ** 3 / 3.0, sol=2.0 * n * n, step=26.0 * n)


def algorithmic_flops(mech, stats: dict) -> float:
    f = flop_model(mech)
    return float(np.sum(stats["nfe"]) * f["rhs"] + np.sum(stats["nje"]) * f["jac"] + np.sum(stats["nsetups"]) * f["lu"]
                 + np.sum(stats["nni"]) * f["sol"] + np.sum(stats["nsteps"]) * f["step"])
