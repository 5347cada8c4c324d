#!/bin/bash
# bench library builds x configs back to back (no CPU leg, no phase split):
#   CFGS="gri surf" bash scripts/cmp_cfgs.sh name1 name2 ...   ("cur" = in-tree libbrhip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CFGS:-gri}; do
  for v in "$@"; do
    lib=$PWD/batchreactor.jl_amd/libbrhip_$v.so; [ "$v" = cur ] && lib=$PWD/batchreactor.jl_amd/libbrhip.so
    BRHIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --no-phase --no-pcie --config $c --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/b_${c}_$v.log 2>&1
    rc=$?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['roofline']['kernel_ms'],1), d['solver'].get('status_counts'))" gpurun_out/b_${c}_$v.log $c $v || { echo "$c $v rc=$rc"; tail -3 gpurun_out/b_${c}_$v.log; }
    [ $rc -ge 124 ] && exit $rc
  done
done
exit 0
