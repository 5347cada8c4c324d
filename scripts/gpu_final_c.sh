#!/bin/bash
# Round-6 final validation at HEAD: GPU suite, smoke, the default bench line, a rocprofv3 kernel-trace
# summary of the bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c_pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/c_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/c_pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/c_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/c_bench_gri.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/c_bench_gri.log; exit 1; }
echo "bench ok"
rm -rf gpurun_out/c_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof -o run -- python3 bench.py --no-cpu --no-phase --steps 3 --warmup 1 > gpurun_out/c_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
