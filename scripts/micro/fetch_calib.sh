#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/micro/fetch_calib.hip): per mode, a 1 GB stream (HBM:
# larger than the 256 MB Infinity Cache) and a 64 MB stream read 4x (Infinity-Cache resident after
# the first pass). Summary: scripts/micro/fetch_calib_sum.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for M in 0 1 2; do
  for S in 1073741824 67108864; do
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fc_${M}_${S} -o run -- python3 scripts/micro/fetch_calib.py $M $S 4 > gpurun_out/fc_${M}_${S}.log 2>&1 || { echo "mode $M size $S failed"; exit 1; }
  done
done
for S in 1073741824 67108864; do
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/fc_3_${S} -o run -- python3 scripts/micro/fetch_calib.py 3 $S 4 > gpurun_out/fc_3_${S}.log 2>&1 || { echo "store size $S failed"; exit 1; }
done
python3 scripts/micro/fetch_calib_sum.py
