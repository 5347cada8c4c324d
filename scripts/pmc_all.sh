#!/bin/bash
# HBM traffic of the integrator kernel for every config at this HEAD: one rocprofv3 counter pass
# per counter group (FETCH_SIZE; WRITE_SIZE; TCC hit/miss), no tracing in the same run, on a
# sample of each config's workload; summaries -> gpurun_out/${TAG}_traffic_<config>.json.
# Usage: bash scripts/pmc_all.sh [configs...]   (N per config: PMC_N, default 20000)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PN=${PMC_N:-20000}
CONFIGS=${*:-gri h2o2 surf gas_surf}
for C in $CONFIGS; do
  N=$PN
  [ "$C" = "h2o2" ] && N=$((PN * 10))
  A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${C}_f -o run -- python3 bench.py $A > gpurun_out/pmc_${C}_f.log 2>&1 || { echo "fetch pass $C failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${C}_w -o run -- python3 bench.py $A > gpurun_out/pmc_${C}_w.log 2>&1 || { echo "write pass $C failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_${C}_t -o run -- python3 bench.py $A > gpurun_out/pmc_${C}_t.log 2>&1 || { echo "tcc pass $C failed"; exit 1; }
  python3 scripts/pmc_traffic.py $(ls gpurun_out/pmc_${C}_f/*counter_collection.csv) $(ls gpurun_out/pmc_${C}_w/*counter_collection.csv) $N gpurun_out/${TAG:-r04}_traffic_${C}.json $(ls gpurun_out/pmc_${C}_t/*counter_collection.csv) || exit 1
done
echo pmc done
