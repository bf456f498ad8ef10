#!/bin/bash
# Round 6 full GPU pass, part 1: every -m gpu test, smoke, the bench line
# (N = 1, default config, with its config1 legs), rocprofv3 kernel trace + PMC
# of the headline kernel and the bench line again with this build's traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=20 PROFILE=1 bash scripts/gpu_round.sh
