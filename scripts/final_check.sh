#!/bin/bash
# One GPU session at the end of a round: A/B bit-identity of the in-tree build against
# libbrhip_prev.so (if present), the GPU test suite, the round's profiles (scripts/round_profile.sh)
# and the driver's own bench command. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -f batchreactor.jl_amd/libbrhip_prev.so ]; then
  for c in ${BITCMP_CFGS:-gri gas_surf surf h2o2}; do
    timeout -k 10 300 python3 scripts/bitcmp.py --config $c --n 2000 prev cur > gpurun_out/fc_bit_$c.log 2>&1 || { echo "bitcmp $c failed"; tail -5 gpurun_out/fc_bit_$c.log; exit 1; }
    tail -1 gpurun_out/fc_bit_$c.log
  done
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
bash scripts/round_profile.sh > gpurun_out/round_profile.log 2>&1 || { echo "round profile failed"; tail -20 gpurun_out/round_profile.log; exit 1; }
tail -12 gpurun_out/round_profile.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_bench.log 2>&1 || { echo "driver bench failed"; tail -5 gpurun_out/driver_bench.log; exit 1; }
tail -1 gpurun_out/driver_bench.log | cut -c1-400
echo final check done
