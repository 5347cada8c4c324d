#!/bin/bash
# Round-6 evidence session B: the bench line of every other config (C2 H2/O2, C4 surface, C5 gas+surface)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in ${CFGS:-h2o2 surf gas_surf}; do
  timeout -k 10 600 python3 bench.py --config $C > gpurun_out/b_bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 gpurun_out/b_bench_$C.log; exit 1; }
  echo "bench $C ok"
done
