#!/bin/bash
# Round-6 final evidence after the lane-parallel controller: smoke, the default bench line (GRI C3),
# a rocprofv3 kernel-trace summary of the same command, and the bench line of every other config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/d_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/d_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/d_bench_gri.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/d_bench_gri.log; exit 1; }
echo "bench gri ok"
rm -rf gpurun_out/d_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d_prof -o run -- python3 bench.py --no-cpu --no-phase --steps 3 --warmup 1 > gpurun_out/d_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
for C in h2o2 surf gas_surf; do
  timeout -k 10 600 python3 bench.py --config $C > gpurun_out/d_bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 gpurun_out/d_bench_$C.log; exit 1; }
  echo "bench $C ok"
done
