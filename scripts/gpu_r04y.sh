#!/usr/bin/env bash
# Round 4 (y): rocprofv3 kernel traces + PMC passes of every bench workload on the final tree
# (continuous-tiles kernels), c4 / v4 with the L2 hit/miss pass, for profiles/r04z_*.
set -euo pipefail
export TMPDIR=/tmp
STEPS=10 bash scripts/round_profile.sh r04z c2_1080p c3_4k
TCC=1 STEPS=10 bash scripts/round_profile.sh r04z c4_env_1080p v4_1080p
