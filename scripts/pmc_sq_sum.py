"""Sum the SQ counters of the integrator kernel from scripts/pmc_sq.sh's passes; per reactor and ratios."""
import csv
import glob
import json
import sys

cfg, n = sys.argv[1], int(sys.argv[2])
tot = {}
for f in glob.glob(f"gpurun_out/pmc_sq[12]_{cfg}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("k_integrate", "k_lane", "k_quad", "k_group")):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {"config": cfg, "reactors": n, "totals": tot, "per_reactor": {k: v / n for k, v in tot.items()}}
if "SQ_INSTS_VALU" in tot and "SQ_ACTIVE_INST_VALU" in tot:
    out["valu_cycles_per_valu_inst"] = tot["SQ_ACTIVE_INST_VALU"] / tot["SQ_INSTS_VALU"]
json.dump(out, open(f"gpurun_out/sq_{cfg}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
