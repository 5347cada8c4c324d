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
[[ $STEPS == *prof* ]] && run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu ${PROF_ARGS:---n 20000 --steps 2 --warmup 1}
echo done
