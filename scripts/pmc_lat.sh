#!/bin/bash
# Memory-side latency and back-pressure of the integrator kernel (two counter passes, no tracing):
# average EA read latency = TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ (cycles), DRAM credit stalls, TCC busy.
#   bash scripts/pmc_lat.sh [config] [N]  -> gpurun_out/pmc_lat_<config>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${1:-gri}; N=${2:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_lat1_$C -o run -- python3 bench.py $A > gpurun_out/pmc_lat1_$C.log 2>&1 || { echo "pass 1 failed"; tail -5 gpurun_out/pmc_lat1_$C.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum TCC_CYCLE_sum --output-format csv -d gpurun_out/pmc_lat2_$C -o run -- python3 bench.py $A > gpurun_out/pmc_lat2_$C.log 2>&1 || { echo "pass 2 failed"; tail -5 gpurun_out/pmc_lat2_$C.log; exit 1; }
python3 - "$C" <<'PY'
import csv, glob, json, sys
c = sys.argv[1]
tot = {}
for f in glob.glob(f"gpurun_out/pmc_lat[12]_{c}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_integrate" in r["Kernel_Name"] or "k_lane" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {"config": c, "totals": tot}
if tot.get("TCC_EA0_RDREQ_sum"):
    out["avg_ea_read_latency_cycles"] = tot["TCC_EA0_RDREQ_LEVEL_sum"] / tot["TCC_EA0_RDREQ_sum"]
if tot.get("TCC_CYCLE_sum"):
    out["tcc_busy_frac"] = tot.get("TCC_BUSY_sum", 0) / tot["TCC_CYCLE_sum"]
    out["dram_credit_stall_frac"] = tot.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", 0) / tot["TCC_CYCLE_sum"]
json.dump(out, open(f"gpurun_out/pmc_lat_{c}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
