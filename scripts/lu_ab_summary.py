"""profiles/r05_lu_ab.json: the lane-grid LU (BR_LU_GRID=1, brhip_lug.hpp) against the row-per-lane LU
at HEAD in k_integrate<56> (GRI), from one gpurun call's outputs:
  gpurun_out/ab_<lib>.log              bench lines (driver-style reactors/s, N = 1e5) per library
  gpurun_out/pmcab_gri.json            PMC passes per library (scripts/pmc_ab.sh -> pmc_ab_sum.py)
  gpurun_out/diagperf_<name>.txt       scripts/diag_perf.py with the diagnostic builds (LU clocks per call)
  gpurun_out/bitcmp_gri.log            scripts/bitcmp.py (bit identity of the two builds)
  python3 scripts/lu_ab_summary.py out.json
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
VARIANTS = {"head (row-per-lane LU)": ("libbrhip.so", "diag"), "grid (BR_LU_GRID=1)": ("libbrhip_lug.so", "diaglug")}
KEYS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VALU_FMA_F64",
        "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD",
        "SQ_INSTS_VMEM_WR", "SQC_ICACHE_MISSES", "FETCH_SIZE", "WRITE_SIZE")


def bench(lib, cfg):
    p = os.path.join(G, f"ab_{cfg}_{lib}.log")
    if not os.path.exists(p):
        return None
    for ln in open(p).read().strip().splitlines()[::-1]:
        if ln.startswith("{"):
            d = json.loads(ln)
            return {"reactors_per_s": d["value"], "kernel_ms": d["roofline"]["kernel_ms"],
                    "mean_steps": d["solver"]["mean_steps"]}
    return None


def diag(name):
    p = os.path.join(G, f"diagperf_{name}.txt")
    if not os.path.exists(p):
        return None
    out = {}
    for ln in open(p):
        m = re.match(r"\s+(rhs|jac|lu|sol|ctl)\s+cycles/call\s+([\d.]+)\s+share of clock ([\d.]+)", ln)
        if m:
            out[m.group(1)] = {"cycles_per_call": float(m.group(2)), "share": float(m.group(3))}
    return out


def main():
    out = sys.argv[1]
    pmc = json.load(open(os.path.join(G, "pmcab_gri.json")))["variants"]
    res = {"kernel": "k_integrate<56> (GRI-Mech 3.0, n = 53)", "variants": {}}
    for name, (lib, dname) in VARIANTS.items():
        p = pmc.get(lib, {})
        v = {"bench_gri_1e5": bench(lib, "gri"), "bench_surf_1e5": bench(lib, "surf"),
             "pmc_per_reactor_gri_2e4": {k: p.get(k) for k in KEYS},
             "fetch_write_bytes_per_reactor": (2.0 * p["FETCH_SIZE"] * 1024 + p["WRITE_SIZE"] * 1024)
             if "FETCH_SIZE" in p and "WRITE_SIZE" in p else None,
             "phase_clocks_gri": diag(dname)}
        res["variants"][name] = v
    bc = os.path.join(G, "bitcmp_gri.log")
    if os.path.exists(bc):
        res["bit_identity"] = open(bc).read().strip().splitlines()[-1]
    h, g = res["variants"]["head (row-per-lane LU)"], res["variants"]["grid (BR_LU_GRID=1)"]
    try:
        res["lu_clocks_ratio"] = g["phase_clocks_gri"]["lu"]["cycles_per_call"] / h["phase_clocks_gri"]["lu"]["cycles_per_call"]
    except (TypeError, KeyError):
        res["lu_clocks_ratio"] = None
    try:
        res["gri_speed_ratio"] = g["bench_gri_1e5"]["reactors_per_s"] / h["bench_gri_1e5"]["reactors_per_s"]
        res["surf_speed_ratio"] = g["bench_surf_1e5"]["reactors_per_s"] / h["bench_surf_1e5"]["reactors_per_s"]
    except (TypeError, KeyError):
        pass
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in res if k != "variants"}))


if __name__ == "__main__":
    main()
