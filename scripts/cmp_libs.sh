#!/bin/bash
# bench several builds of libbrhip back to back: bash scripts/cmp_libs.sh name1 name2 ...
# (batchreactor.jl_amd/libbrhip_<name>.so; "cur" = the in-tree libbrhip.so)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  lib=$PWD/batchreactor.jl_amd/libbrhip_$v.so; [ "$v" = cur ] && lib=$PWD/batchreactor.jl_amd/libbrhip.so
  BRHIP_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --no-pcie --steps 2 ${BENCH_ARGS:-} > gpurun_out/b_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/b_$v.log | cut -c60-120)"
done
