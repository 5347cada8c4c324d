#!/bin/bash
# Quick GPU iteration: GPU parity tests, then the GRI bench (no CPU leg); prints one summary line.
# Usage: bash scripts/quick.sh [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/b.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('BENCH', d['config']['workload'][:12], round(d['value']), round(d['roofline']['kernel_ms'],1), d['solver']['status_counts'], d['solver']['mean_steps'])"
