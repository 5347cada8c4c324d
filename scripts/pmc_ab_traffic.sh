#!/bin/bash
# Memory-side traffic of the integrator kernel for several builds: two counter passes each
# ([FETCH_SIZE], [WRITE_SIZE TCC_HIT_sum TCC_MISS_sum]), no tracing; summary per build.
#   bash scripts/pmc_ab_traffic.sh name1 name2 ...   (libbrhip_<name>.so; "cur" = libbrhip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${CFG:-gri}; N=${PMC_N:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
for v in "$@"; do
  lib=$PWD/batchreactor.jl_amd/libbrhip_$v.so; [ "$v" = cur ] && lib=$PWD/batchreactor.jl_amd/libbrhip.so
  rm -rf gpurun_out/ptf_$v gpurun_out/ptw_$v
  BRHIP_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ptf_$v -o run -- python3 bench.py $A > gpurun_out/ptf_$v.log 2>&1 || { echo "$v fetch failed"; exit 1; }
  BRHIP_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/ptw_$v -o run -- python3 bench.py $A > gpurun_out/ptw_$v.log 2>&1 || { echo "$v write failed"; exit 1; }
  python3 scripts/pmc_traffic.py $(ls gpurun_out/ptf_$v/*counter_collection.csv) $(ls gpurun_out/ptw_$v/*counter_collection.csv) $N gpurun_out/traffic_${C}_$v.json $(ls gpurun_out/ptw_$v/*counter_collection.csv) > /dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'MB/reactor', round(d['bytes_per_reactor']/1e6,2), 'rd', round(d['read_bytes_corrected']/d['reactors']/1e6,2), 'wr', round(d['write_bytes']/d['reactors']/1e6,2), 'L2 hit', round(d['tcc_hit_rate'],3))" gpurun_out/traffic_${C}_$v.json $v
done
