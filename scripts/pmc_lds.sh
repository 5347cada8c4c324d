#!/bin/bash
# LDS behaviour of the integrator kernel (one SQ counter pass, no tracing): instructions by kind,
# bank / address conflicts (cycles), LDS-active cycles.
#   bash scripts/pmc_lds.sh [config] [N]  -> gpurun_out/pmc_lds_<config>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${1:-gri}; N=${2:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_lds_$C -o run -- python3 bench.py $A > gpurun_out/pmc_lds_$C.log 2>&1 || { echo "pass failed"; tail -5 gpurun_out/pmc_lds_$C.log; exit 1; }
python3 - "$C" "$N" <<'PY'
import csv, glob, json, sys
c, n = sys.argv[1], int(sys.argv[2])
tot = {}
for f in glob.glob(f"gpurun_out/pmc_lds_{c}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_integrate" in r["Kernel_Name"] or "k_lane" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {"config": c, "reactors": n, "per_reactor": {k: v / n for k, v in tot.items()}}
json.dump(out, open(f"gpurun_out/pmc_lds_{c}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
