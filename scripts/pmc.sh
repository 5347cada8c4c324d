#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass) on a short GRI integration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
N=${N:-8192}
ARGS="--no-cpu --n $N --steps 1 --warmup 0"
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
