#!/bin/bash
# device-only compile of brhip.hip with extra -D flags; prints the register / occupancy summary of
# the kernels matching $KPAT (default k_quad). Usage: KPAT=k_quad scripts/micro/vgpr_probe.sh -DFOO=1
cd "$(dirname "$0")/../../batchreactor.jl_amd/csrc"
KPAT=${KPAT:-k_quad}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -mllvm -disable-machine-licm --cuda-device-only -c \
  -o /tmp/vp_$$.o brhip.hip -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -A7 "Function Name: .*${KPAT}" | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy" | sed 's/\[-Rpass.*//'
rm -f /tmp/vp_$$.o
