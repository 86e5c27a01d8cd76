#!/usr/bin/env bash
# Round 4 (b): rocprofv3 kernel traces + PMC passes of c2, c4 and v4 (v4 and c4 with the L2 hit /
# miss pass), for profiles/r04b_*.
set -euo pipefail
export TMPDIR=/tmp
STEPS=10 bash scripts/round_profile.sh r04b c2_1080p
TCC=1 STEPS=10 bash scripts/round_profile.sh r04b c4_env_1080p v4_1080p
