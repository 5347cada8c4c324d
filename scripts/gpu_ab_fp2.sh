#!/bin/bash
# A/B of the LU pivot fast paths (CPL 1 and 2: libbrhip_fp2.so) against HEAD's library on C5 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bitcmp.py --config gas_surf --n 2000 cur fp2 > gpurun_out/fp2_bitcmp_gs.log 2>&1 || { echo "bitcmp gs failed"; tail -5 gpurun_out/fp2_bitcmp_gs.log; exit 1; }
tail -2 gpurun_out/fp2_bitcmp_gs.log
timeout -k 10 300 python3 scripts/bitcmp.py --config gri --n 4000 cur fp2 > gpurun_out/fp2_bitcmp_gri.log 2>&1 || { echo "bitcmp gri failed"; exit 1; }
tail -2 gpurun_out/fp2_bitcmp_gri.log
LIBS="libbrhip.so libbrhip_fp2.so libbrhip.so libbrhip_fp2.so" CFG=gas_surf bash scripts/ab.sh --steps 2 --warmup 1 > gpurun_out/fp2_ab_gs.txt 2>&1; cat gpurun_out/fp2_ab_gs.txt
LIBS="libbrhip.so libbrhip_fp2.so libbrhip.so libbrhip_fp2.so" CFG=gri bash scripts/ab.sh --steps 3 --warmup 1 > gpurun_out/fp2_ab_gri.txt 2>&1; cat gpurun_out/fp2_ab_gri.txt
