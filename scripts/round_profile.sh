#!/bin/bash
# Refresh the judged measurement files at this HEAD (one GPU session):
#  1. PMC traffic per config (scripts/pmc_all.sh) -> profiles/${TAG}_traffic_<cfg>.json (bench reads it)
#  2. one full bench line per config (CPU leg + phase split) -> profiles/${TAG}_bench_<cfg>.json
#  3. rocprofv3 --kernel-trace --stats of the default (GRI) bench -> profiles/${TAG}_gri1e5_kernel_stats.csv
# Stops at the first step that fails, times out or faults. Only gpurun_out/ comes back from a GPU box:
# everything destined for profiles/ is also written to gpurun_out/profiles/ (copy it over afterwards:
# cp gpurun_out/profiles/* profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
export TAG
mkdir -p gpurun_out/profiles profiles
CFGS=${CFGS:-gri h2o2 surf gas_surf}
if [ -z "$NO_PMC" ]; then
  bash scripts/pmc_all.sh $CFGS || exit $?
  for c in $CFGS; do cp gpurun_out/${TAG}_traffic_$c.json profiles/${TAG}_traffic_$c.json; cp gpurun_out/${TAG}_traffic_$c.json gpurun_out/profiles/; done
fi
for c in $CFGS; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log > gpurun_out/profiles/${TAG}_bench_$c.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']), round(r['kernel_ms'],1), 'frac', round(r['frac'],4), 'traffic/reactor', (r['traffic'] or 0)/d['config']['reactors_rank0'])" gpurun_out/profiles/${TAG}_bench_$c.json $c
done
if [[ " $CFGS " == *" gri "* ]]; then
  # SQ instruction mix / VALU-busy counters (two passes) -> profiles/${TAG}_pmc_sq_gri.json
  bash scripts/pmc_sq.sh gri 20000 > gpurun_out/pmc_sq_gri.log 2>&1 && cp gpurun_out/sq_gri.json gpurun_out/profiles/${TAG}_pmc_sq_gri.json || { echo "pmc_sq failed"; tail -5 gpurun_out/pmc_sq_gri.log; exit 1; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-phase --no-pcie > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
  cp "$(ls gpurun_out/prof/*kernel_stats.csv | head -1)" gpurun_out/profiles/${TAG}_gri1e5_kernel_stats.csv
  grep "^{\"metric\"" gpurun_out/prof.log | tail -1 > gpurun_out/profiles/${TAG}_gri1e5_rocprof_bench_line.json
  head -3 gpurun_out/profiles/${TAG}_gri1e5_kernel_stats.csv
fi
echo profile done
