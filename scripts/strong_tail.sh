#!/bin/bash
# Strong-scaling tail on one GPU: the per-rank shard sizes of 1/2/4/8 GPUs (BASELINE C3: 1e5 GRI
# reactors in total) run back to back; rate(N)/rate(1e5) is the scaling efficiency the tail allows.
#   bash scripts/strong_tail.sh [config]   (extra bench args in BENCH_ARGS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=${1:-gri}
for n in 100000 50000 25000 12500; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-phase --config $C --n $n --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/tail_${C}_$n.log 2>&1 || { echo "n=$n failed"; tail -3 gpurun_out/tail_${C}_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('tail', sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],1))" gpurun_out/tail_${C}_$n.log $C $n
done
