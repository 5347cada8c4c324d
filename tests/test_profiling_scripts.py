"""CPU tests of the counter-summary scripts behind bench.py's memory roofline (scripts/pmc_dram.py,
scripts/pmc_traffic.py): synthetic rocprofv3 counter CSVs in, bytes per reactor and the HBM bound out."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, rows):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_dram_summary(tmp_path):
    n = 1000
    k = "void (anonymous namespace)::k_integrate<56>(brhip::DevMech, ...)"
    other = "void at::native::elementwise_kernel<...>"
    # 2 dispatches of the integrator plus an unrelated kernel that must be ignored
    _csv(tmp_path / "f.csv", [{"Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 500.0},
                              {"Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 500.0},
                              {"Kernel_Name": other, "Counter_Name": "FETCH_SIZE", "Counter_Value": 1e9}])
    _csv(tmp_path / "w.csv", [{"Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": 250.0},
                              {"Kernel_Name": k, "Counter_Name": "TCC_HIT_sum", "Counter_Value": 30.0},
                              {"Kernel_Name": k, "Counter_Name": "TCC_MISS_sum", "Counter_Value": 70.0}])
    _csv(tmp_path / "d.csv", [{"Kernel_Name": k, "Counter_Name": "TCC_EA0_RDREQ_DRAM_32B_sum", "Counter_Value": 64000.0},
                              {"Kernel_Name": k, "Counter_Name": "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum", "Counter_Value": 8000.0},
                              {"Kernel_Name": k, "Counter_Name": "TCC_EA0_RDREQ_DRAM_sum", "Counter_Value": 16000.0},
                              {"Kernel_Name": k, "Counter_Name": "TCC_EA0_WRREQ_DRAM_sum", "Counter_Value": 4000.0}])
    bench = {"metric": "m", "value": 5000.0, "config": {"reactors_rank0": n},
             "roofline": {"kernel_ms": 0.2, "kernel": "k_integrate<56>"}}
    (tmp_path / "t.log").write_text("warming up\n" + json.dumps(bench) + "\n")
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_dram.py"), "gri", str(n), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), str(tmp_path / "d.csv"), str(tmp_path / "t.log"), str(out)],
                   check=True, capture_output=True)
    d = json.loads(out.read_text())
    fab_rd = 2.0 * 1000.0 * 1024.0          # FETCH_SIZE KiB x2 (gfx950 correction)
    fab_wr = 250.0 * 1024.0
    assert abs(d["l2_fabric"]["read_bytes_per_reactor"] - fab_rd / n) < 1e-9
    assert abs(d["l2_fabric"]["bytes_per_reactor"] - (fab_rd + fab_wr) / n) < 1e-9
    assert abs(d["l2_fabric"]["l2_hit_rate"] - 0.3) < 1e-12
    assert abs(d["dram_destined"]["bytes_per_reactor"] - 32.0 * 72000.0 / n) < 1e-9
    # rate = bytes per reactor x reactors / kernel time
    assert abs(d["l2_fabric"]["GBs"] - (fab_rd + fab_wr) / 0.2e-3 / 1e9) < 1e-9
    # HBM bound: at most 6.3 TB/s x 0.2 ms could come from HBM
    hbm_max = 6300e9 * 0.2e-3 / n
    assert abs(d["hbm_bound"]["max_hbm_bytes_per_reactor"] - hbm_max) < 1e-6
    share = max(0.0, 1.0 - hbm_max / ((fab_rd + fab_wr) / n))
    assert abs(d["hbm_bound"]["min_infinity_cache_share_of_fabric_bytes"] - share) < 1e-12


def test_pmc_traffic_summary(tmp_path):
    k = "void (anonymous namespace)::k_group<16, 9>(brhip::DevMech, ...)"
    _csv(tmp_path / "f.csv", [{"Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 10.0}])
    _csv(tmp_path / "w.csv", [{"Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": 4.0}])
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), "8", str(out)], check=True, capture_output=True)
    d = json.loads(out.read_text())
    assert abs(d["bytes_per_reactor"] - (2 * 10.0 * 1024 + 4.0 * 1024) / 8) < 1e-9


def test_parity_bounds_follow_the_committed_analysis():
    """tests/parity_bands.py's bounds are the ones profiles/r06_parity_outliers.json derived (2x the
    oracle's own spread on the bench samples, rounded up to 3 digits; analytic pre-ignition floors of
    1e-6 bands and the surface bar of 1.0 as documented there), for every bench config and Jacobian,
    and the GPU was inside them on every scored reactor of that analysis."""
    import json
    import math
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    import parity_bands as PB
    d = json.load(open(os.path.join(root, "profiles", "r06_parity_outliers.json")))
    for config, (ka, kd) in bench.PARITY_SAMPLE.items():
        for jac, dq, k in (("analytic", False, ka), ("dq", True, kd)):
            r = d["configs"][config][jac]
            assert r["sample"] == k and r["gpu_frac_within_bound"] == 1.0
            for w, (b, derived) in enumerate(zip(PB.BOUNDS[(config, dq)][:3], r["bound"])):
                if config == "surf" and w > 0:
                    continue                      # no ignition: only the pre-ignition window exists
                if config == "surf" and not dq:
                    assert b == 1.0 and max(r["gpu_vs_oracle"]["max"]) <= b
                    continue
                if w == 0 and not dq and config in ("gri", "h2o2"):
                    assert b == 1e-6 and derived < b
                    continue
                assert derived <= b <= derived * (1 + 1e-2) + 1e-12, (config, jac, w, b, derived)
                assert math.isfinite(b)
