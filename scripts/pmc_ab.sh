#!/bin/bash
# SQ counters of the integrator kernel for several builds (one counter pass each, no tracing):
#   bash scripts/pmc_ab.sh name1 name2 ...   (libbrhip_<name>.so; "cur" = libbrhip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${CFG:-gri}; N=${PMC_N:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
for v in "$@"; do
  lib=$PWD/batchreactor.jl_amd/libbrhip_$v.so; [ "$v" = cur ] && lib=$PWD/batchreactor.jl_amd/libbrhip.so
  rm -rf gpurun_out/pab_$v
  BRHIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pab_$v -o run -- python3 bench.py $A > gpurun_out/pab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/pab_$v.log; exit 1; }
  python3 - "$v" "$N" <<'PY'
import csv, glob, sys
v, n = sys.argv[1], int(sys.argv[2])
tot = {}
for f in glob.glob(f"gpurun_out/pab_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_integrate" in r["Kernel_Name"] or "k_lane" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
pr = {k.replace("SQ_", ""): round(x / n / 1e3, 1) for k, x in tot.items() if k != "SQ_WAVES"}
print(v, "k/reactor:", pr)
PY
done
