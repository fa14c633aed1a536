#!/bin/bash
# Per-kernel resource usage (VGPRs, spills, scratch, occupancy, LDS) of the product units, from
# the compiler's kernel-resource-usage remarks: tools/resource_usage.sh > profiles/rNN_resource_usage.txt
# Extra -D flags (a tuning variant) can be passed as arguments.
set -euo pipefail
cd "$(dirname "$0")/../chaum-pedersen-zkp_amd/csrc"
for u in kernels.hip rlc.hip part.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I . -I ../../include "$@" \
    --cuda-device-only -c "$u" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -E "remark: (Function Name|    (TotalSGPRs|VGPRs|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size))" || true
done
