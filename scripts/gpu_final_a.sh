#!/bin/bash
# Round-6 evidence session A (GRI): smoke, the default bench line, a rocprofv3 kernel-trace summary
# of the same command, and the HBM / L2-fabric counter passes (scripts/pmc_dram.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/a_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke ok"
timeout -k 10 600 python3 bench.py > gpurun_out/a_bench_gri.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/a_bench_gri.log; exit 1; }
echo "bench ok"
rm -rf gpurun_out/a_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a_prof -o run -- python3 bench.py --no-cpu --no-phase --steps 3 --warmup 1 > gpurun_out/a_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
CFG=gri PMC_N=20000 bash scripts/pmc_dram.sh > gpurun_out/a_pmc.log 2>&1 || { echo "pmc failed"; cat gpurun_out/a_pmc.log; exit 1; }
echo "pmc ok"
