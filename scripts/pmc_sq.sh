#!/bin/bash
# SQ instruction-mix / busy counters of the integrator kernel (two counter passes, no tracing):
#   bash scripts/pmc_sq.sh [config] [N]   -> gpurun_out/pmc_sq1, pmc_sq2 ; summary via scripts/pmc_sq_sum.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${1:-gri}; N=${2:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sq1_$C -o run -- python3 bench.py $A > gpurun_out/pmc_sq1_$C.log 2>&1 || { echo "pass 1 failed"; tail -5 gpurun_out/pmc_sq1_$C.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_sq2_$C -o run -- python3 bench.py $A > gpurun_out/pmc_sq2_$C.log 2>&1 || { echo "pass 2 failed"; tail -5 gpurun_out/pmc_sq2_$C.log; exit 1; }
python3 scripts/pmc_sq_sum.py $C $N
