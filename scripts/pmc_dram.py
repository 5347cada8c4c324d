"""Summarise scripts/pmc_dram.sh's counter passes into bytes per reactor and per-launch rates.

  python scripts/pmc_dram.py cfg N fetch.csv write.csv dram.csv timing.log out.json

Two views of the integrator's memory traffic (k_integrate / k_lane / k_quad / k_group dispatches):
  l2_fabric: FETCH_SIZE x 2 (the gfx950 correction of MI355X_MICROARCH.md, HBM section) + WRITE_SIZE,
             i.e. everything the L2 sends to the data fabric. The guide notes Infinity-Cache (MALL)
             hits are counted here, so this is NOT HBM traffic.
  dram:      TCC_EA0_RDREQ_DRAM_32B / TCC_EA0_WRREQ_WRITE_DRAM_32B x 32 B, the requests whose address
             maps to DRAM (as opposed to GMI peers or IO). The MALL sits in the fabric behind the L2,
             so these counters see the request before the MALL does: no counter in
             rocprofiler-sdk's gfx950 list separates MALL hits. The script therefore also reports the
             physical bound: at most HBM_ACHIEVABLE_GBS x kernel time can have come from HBM, the
             rest of the fabric-side bytes must have been Infinity-Cache hits.
"""
import csv
import json
import sys

HBM_PEAK_GBS = 8000.0
HBM_ACHIEVABLE_GBS = 6300.0   # MI355X_MICROARCH.md, HBM section
KERNELS = ("k_integrate", "k_lane", "k_quad", "k_group")


def total(path, name):
    s = 0.0
    for r in csv.DictReader(open(path)):
        if any(k in r["Kernel_Name"] for k in KERNELS) and r["Counter_Name"] == name:
            s += float(r["Counter_Value"])
    return s


def bench_line(path):
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            return json.loads(ln)
    raise SystemExit(f"no bench line in {path}")


def main():
    cfg, n = sys.argv[1], int(sys.argv[2])
    fetch_csv, write_csv, dram_csv, tlog, out = sys.argv[3:8]
    rd_fab = 2.0 * total(fetch_csv, "FETCH_SIZE") * 1024.0
    wr_fab = total(write_csv, "WRITE_SIZE") * 1024.0
    hit, miss = total(write_csv, "TCC_HIT_sum"), total(write_csv, "TCC_MISS_sum")
    rd_dram = 32.0 * total(dram_csv, "TCC_EA0_RDREQ_DRAM_32B_sum")
    wr_dram = 32.0 * total(dram_csv, "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
    rdreq_dram = total(dram_csv, "TCC_EA0_RDREQ_DRAM_sum")
    wrreq_dram = total(dram_csv, "TCC_EA0_WRREQ_DRAM_sum")
    b = bench_line(tlog)
    kms = b["roofline"]["kernel_ms"]
    n_bench = b["config"]["reactors_rank0"]
    ks = kms * 1e-3
    per = lambda x: x / n
    fab = per(rd_fab + wr_fab)
    dram = per(rd_dram + wr_dram)
    # rates at the timed kernel: bytes per reactor x reactors of one launch / kernel time
    rate = lambda bpr: bpr * n_bench / ks / 1e9
    hbm_max = HBM_ACHIEVABLE_GBS * ks * 1e9 / n_bench   # most bytes per reactor HBM could have moved
    res = {
        "config": cfg, "reactors_counted": n, "reactors_timed": n_bench, "kernel_ms": kms,
        "kernel": b["roofline"].get("kernel"),
        "reactors_per_s": b["value"],
        "l2_fabric": {"read_bytes_per_reactor": per(rd_fab), "write_bytes_per_reactor": per(wr_fab),
                      "bytes_per_reactor": fab, "GBs": rate(fab), "frac_of_hbm_peak": rate(fab) / HBM_PEAK_GBS,
                      "l2_hit_rate": hit / max(hit + miss, 1.0),
                      "counters": "FETCH_SIZE x2 + WRITE_SIZE (KiB -> B)"},
        "dram_destined": {"read_bytes_per_reactor": per(rd_dram), "write_bytes_per_reactor": per(wr_dram),
                          "bytes_per_reactor": dram, "GBs": rate(dram), "frac_of_hbm_peak": rate(dram) / HBM_PEAK_GBS,
                          "read_requests_per_reactor": per(rdreq_dram), "write_requests_per_reactor": per(wrreq_dram),
                          "counters": "TCC_EA0_RDREQ_DRAM_32B_sum, TCC_EA0_WRREQ_WRITE_DRAM_32B_sum (x 32 B); "
                                      "TCC_EA0_RDREQ_DRAM_sum, TCC_EA0_WRREQ_DRAM_sum (requests)"},
        "hbm_bound": {"achievable_GBs": HBM_ACHIEVABLE_GBS,
                      "max_hbm_bytes_per_reactor": hbm_max,
                      "min_infinity_cache_share_of_fabric_bytes": max(0.0, 1.0 - hbm_max / fab) if fab else None},
        "note": "dram_destined counts requests addressed to DRAM before the Infinity Cache (MALL) "
                "serves or forwards them; no gfx950 counter in rocprofiler-sdk separates MALL hits. "
                "hbm_bound: HBM cannot have delivered more than achievable_GBs x kernel time, so at least "
                "min_infinity_cache_share_of_fabric_bytes of the fabric-side bytes were Infinity-Cache hits.",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
