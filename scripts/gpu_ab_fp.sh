#!/bin/bash
# A/B of the LU pivot fast path (libbrhip_fp.so) against HEAD: bit identity, then timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bitcmp.py --config gri --n 4000 cur fp > gpurun_out/fp_bitcmp_gri.log 2>&1 || { echo "bitcmp gri failed"; tail -5 gpurun_out/fp_bitcmp_gri.log; exit 1; }
tail -3 gpurun_out/fp_bitcmp_gri.log
timeout -k 10 300 python3 scripts/bitcmp.py --config surf --n 8000 cur fp > gpurun_out/fp_bitcmp_surf.log 2>&1 || { echo "bitcmp surf failed"; tail -5 gpurun_out/fp_bitcmp_surf.log; exit 1; }
tail -3 gpurun_out/fp_bitcmp_surf.log
LIBS="libbrhip.so libbrhip_fp.so libbrhip.so libbrhip_fp.so" CFG=gri bash scripts/ab.sh --steps 3 --warmup 1 > gpurun_out/fp_ab_gri.txt 2>&1; cat gpurun_out/fp_ab_gri.txt
LIBS="libbrhip.so libbrhip_fp.so libbrhip.so libbrhip_fp.so" CFG=surf bash scripts/ab.sh --steps 3 --warmup 1 > gpurun_out/fp_ab_surf.txt 2>&1; cat gpurun_out/fp_ab_surf.txt
