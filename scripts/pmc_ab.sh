#!/bin/bash
# In-engine A/B of library variants with PMC counters (separate passes, no tracing):
#   LIBS="libbrhip_lu0.so libbrhip.so" CFG=gri N=20000 bash scripts/pmc_ab.sh
# -> gpurun_out/pmcab_<lib>_<pass>/ ; summary: python3 scripts/pmc_ab_sum.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${CFG:-gri}; N=${N:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
P3="SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
P6="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
P7="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_IFETCH"
# PASSES: which of the passes above to run (default 1..5)
for L in ${LIBS}; do
  for i in ${PASSES:-1 2 3 4 5}; do
    eval P=\$P$i
    BRHIP_LIB=$PWD/batchreactor.jl_amd/$L timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcab_${L}_$i -o run -- python3 bench.py $A > gpurun_out/pmcab_${L}_$i.log 2>&1 || { echo "pass $i of $L failed"; tail -3 gpurun_out/pmcab_${L}_$i.log; }
  done
done
python3 scripts/pmc_ab_sum.py $C $N ${LIBS}
