#!/bin/bash
# One GPU session: smoke, GPU parity tests, a bench line and a rocprofv3 kernel-trace summary.
# Stops at the first step that times out, aborts or faults (exit >= 124); plain test failures
# (exit 1) are recorded and the session continues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
[[ $STEPS == *bench* ]] && run bench 900 python3 bench.py ${BENCH_ARGS:-}
[[ $STEPS == *parity* ]] && run parity 1200 python3 -u scripts/parity_outliers.py ${PARITY_ARGS:-}
[[ $STEPS == *prof* ]] && run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu ${PROF_ARGS:---steps 3 --warmup 1}
if [[ $STEPS == *pmc* ]]; then   # HBM traffic of k_integrate: separate counter passes (no tracing)
  PN=${PMC_N:-20000}
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 bench.py --no-cpu --no-phase --no-pcie --n $PN --steps 1 --warmup 0 ${PMC_ARGS:-}
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 bench.py --no-cpu --no-phase --no-pcie --n $PN --steps 1 --warmup 0 ${PMC_ARGS:-}
  run pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_t -o run -- python3 bench.py --no-cpu --no-phase --no-pcie --n $PN --steps 1 --warmup 0 ${PMC_ARGS:-}
  python3 scripts/pmc_traffic.py $(ls gpurun_out/pmc_f/*counter_collection.csv) $(ls gpurun_out/pmc_w/*counter_collection.csv) $PN gpurun_out/traffic_gri.json $(ls gpurun_out/pmc_t/*counter_collection.csv)
fi
echo done
