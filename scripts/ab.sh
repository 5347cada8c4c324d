#!/bin/bash
# A/B of library variants on one GPU: for each lib in $LIBS, one bench line (no CPU leg, no phase
# split). Usage: LIBS="a.so b.so" CFG=gri bash scripts/ab.sh [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS}; do
  BRHIP_LIB=$PWD/batchreactor.jl_amd/$L timeout -k 10 300 python3 bench.py --no-cpu --no-phase --no-pcie --config ${CFG:-gri} "$@" > gpurun_out/ab_${CFG:-gri}_$L.log 2>&1 || { echo "FAIL $L rc=$?"; tail -5 gpurun_out/ab_${CFG:-gri}_$L.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${CFG:-gri}_$L.log').read().strip().splitlines()[-1]); print('AB', '$L', d['config']['workload'][:8], round(d['value']), round(d['roofline']['kernel_ms'],1), d['solver']['status_counts'], round(d['solver']['mean_steps'],2), (d.get('parity_vs_oracle') or {}).get('max'))"
done
