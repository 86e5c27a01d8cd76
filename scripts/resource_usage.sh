#!/usr/bin/env bash
# Per-kernel resource usage (VGPRs, spills, occupancy, LDS) of a csrc/*.hip file for gfx950, from the
# compiler's kernel-resource-usage remarks (no GPU needed).  usage: scripts/resource_usage.sh FILE.hip [-DX=1 ...]
set -euo pipefail
cd "$(dirname "$0")/../cpuperformanceraytracer_amd/csrc"
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
    -fno-gpu-flush-denormals-to-zero -mllvm -amdgpu-atomic-optimizer-strategy=None -fno-slp-vectorize \
    -I../../include -I. --cuda-device-only -c "$f" -o /tmp/_ru.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep remark | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' |
  awk '/^Function Name/ {if (line) print line; cmd="c++filt " $3; cmd | getline n; close(cmd); line=n; next}
       /^(VGPRs|ScratchSize|Occupancy|VGPRs Spill|SGPRs Spill|LDS Size)/ {line=line " | " $0}
       END {print line}'
