"""Per-case parity bands for GPU-vs-oracle trajectories (test infrastructure; also read by bench.py's
cpu_baseline leg for its parity_vs_oracle block).

Metric: per reactor and output time, max_k |Y_gpu - Y_orc| / (1e-4 |Y_orc| + 100 atol) -- "bands"
of the north_star's 1e-4 relative bar -- maximised over three windows of t / t_ign: before 0.5
(pre-ignition), [0.5, 2) (the ignition front), >= 2 (post-ignition). The oracle runs the same
algorithm with the same Jacobian kind, so every difference is rounding; how far rounding alone moves
a CVODE trajectory was measured on the oracle itself (profiles/r04_parity_spread.json,
scripts/diag_spread.py: a second oracle run with u0 perturbed by 1e-15 relative; DQ runs also with
the increments jittered by 1e-15; 128-512 reactors of the bench workload per case):

                      pre-ignition   front    post-ignition     reactors
  GRI   analytic J       1.4e-10      1.23        2.51            256
  GRI   DQ J             1.28        34.6         2.83            256
  gas+surf analytic      1.01       572           8.25            256 (1 failed pair excluded)
  gas+surf DQ            0.93       144           4.56            128 (1 failed pair excluded)
  surface analytic       0.22         -            -              256 (no ignition)
  H2/O2 analytic         1.0e-10      0.37        1.28            512
  H2/O2 DQ               5.84       163           2.75            512

Bounds: front and post-ignition at 2x the measured spread; pre-ignition the north_star's 1e-4 bar
(1 band) where the spread is below it -- tightened to 1e-6 bands for the analytic gas-phase cases,
whose spread is ~1e-10 -- and 2x the spread where CVODE's DQ Jacobian alone exceeds it.
"""
import numpy as np

ATOL = 1e-10
OUT_T = np.concatenate([[1e-6, 1e-5, 1e-4], np.logspace(-3, 1, 25)])
WINDOWS = ((0.0, 0.5), (0.5, 2.0), (2.0, np.inf))

# (case, dq_jacobian) -> (pre-ignition, front, post-ignition) bounds in bands
BOUNDS = {
    ("gri", False): (1e-6, 2.5, 5.0),
    ("gri", True): (2.6, 70.0, 5.7),
    ("gas_surf", False): (1.0, 1150.0, 16.5),
    ("gas_surf", True): (1.9, 290.0, 9.2),
    ("surf", False): (0.45, 0.45, 0.45),
    ("h2o2", False): (1e-6, 0.75, 2.6),
    ("h2o2", True): (11.7, 330.0, 5.5),
}


def band_errors(Yg, Yo, tign, tout=OUT_T):
    """max error per ignition window (pre, front, post) for one reactor; no ignition: all pre"""
    e = (np.abs(Yg - Yo) / (1e-4 * np.abs(Yo) + 100 * ATOL)).max(axis=1)
    r = tout / tign if tign == tign else np.zeros_like(tout)
    return [float(e[(r >= lo) & (r < hi)].max(initial=0.0)) for lo, hi in WINDOWS]
