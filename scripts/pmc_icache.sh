#!/bin/bash
# Instruction-cache behaviour of the integrator kernel (counter passes, no tracing):
# SQC_ICACHE_{REQ,HITS,MISSES,MISSES_DUPLICATE}, SQ_IFETCH(_LEVEL), SQ_WAIT_ANY, SQ_WAVE_CYCLES.
#   bash scripts/pmc_icache.sh [config] [N]  -> gpurun_out/pmc_icache_<config>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${1:-gri}; N=${2:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/pmc_ic1_$C -o run -- python3 bench.py $A > gpurun_out/pmc_ic1_$C.log 2>&1 || { echo "pass 1 failed"; tail -5 gpurun_out/pmc_ic1_$C.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc_ic2_$C -o run -- python3 bench.py $A > gpurun_out/pmc_ic2_$C.log 2>&1 || { echo "pass 2 failed"; tail -5 gpurun_out/pmc_ic2_$C.log; exit 1; }
python3 - "$C" "$N" <<'PY'
import csv, glob, json, sys
c, n = sys.argv[1], int(sys.argv[2])
tot = {}
for f in glob.glob(f"gpurun_out/pmc_ic[12]_{c}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("k_integrate", "k_lane", "k_group")):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {"config": c, "reactors": n, "per_reactor": {k: v / n for k, v in tot.items()}}
if tot.get("SQC_ICACHE_REQ"):
    out["icache_hit_rate"] = tot.get("SQC_ICACHE_HITS", 0) / tot["SQC_ICACHE_REQ"]
if tot.get("SQ_IFETCH"):
    out["avg_ifetch_level"] = tot.get("SQ_IFETCH_LEVEL", 0) / tot["SQ_IFETCH"]
json.dump(out, open(f"gpurun_out/pmc_icache_{c}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
