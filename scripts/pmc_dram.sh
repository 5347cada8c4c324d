#!/bin/bash
# DRAM-destined vs L2-fabric-side bytes of the integrator kernel: three counter
# passes over the same bench workload, each its own rocprofv3 run (no tracing):
#   1. FETCH_SIZE                                    (L2 memory-side reads, KiB, x2 on gfx950)
#   2. WRITE_SIZE TCC_HIT_sum TCC_MISS_sum           (L2 memory-side writes, L2 hit rate)
#   3. TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum
#      (requests the L2 sends towards DRAM, in 32-B units: a 64-B request counts 2, 128-B counts 4)
# then one plain bench run for the kernel time. Summary: scripts/pmc_dram.py -> gpurun_out/dram_<cfg>.json
#   CFG=gri PMC_N=20000 bash scripts/pmc_dram.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${CFG:-gri}; N=${PMC_N:-20000}
A="--no-cpu --no-phase --no-pcie --config $C --n $N --steps 1 --warmup 0"
rm -rf gpurun_out/pd_f_$C gpurun_out/pd_w_$C gpurun_out/pd_d_$C
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pd_f_$C -o run -- python3 bench.py $A > gpurun_out/pd_f_$C.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pd_w_$C -o run -- python3 bench.py $A > gpurun_out/pd_w_$C.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d gpurun_out/pd_d_$C -o run -- python3 bench.py $A > gpurun_out/pd_d_$C.log 2>&1 || { echo "dram pass failed"; exit 1; }
timeout -k 10 150 python3 bench.py --no-cpu --no-phase --no-pcie --config $C --n $N --steps 2 --warmup 1 > gpurun_out/pd_t_$C.log 2>&1 || { echo "timing run failed"; exit 1; }
python3 scripts/pmc_dram.py $C $N $(ls gpurun_out/pd_f_$C/*counter_collection.csv) $(ls gpurun_out/pd_w_$C/*counter_collection.csv) \
  $(ls gpurun_out/pd_d_$C/*counter_collection.csv) gpurun_out/pd_t_$C.log gpurun_out/dram_$C.json
python3 scripts/pmc_traffic.py $(ls gpurun_out/pd_f_$C/*counter_collection.csv) $(ls gpurun_out/pd_w_$C/*counter_collection.csv) $N \
  gpurun_out/traffic_$C.json $(ls gpurun_out/pd_w_$C/*counter_collection.csv) > /dev/null
