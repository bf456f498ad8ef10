#!/bin/bash
# Round 6: round 5's waiting fused launch (build_ab/libsf_r5.so) under calls
# that synchronise in between (the default pool then gives its freed blocks
# back) and calls queued back to back, alternating processes; spin bound
# 2^20 polls so a stuck chain gives up quickly.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s
for r in 1 2 3; do
  for sync in 1 0; do
    SYNC=$sync ITERS=200 SF_LIB=build_ab/libsf_r5.so SF_TEST_CHAIN_SPIN_LIMIT=1048576 timeout -k 10 200 python3 scripts/r5_fused_release_stress.py >> gpurun_out/s/r5_stress.log 2>&1 || exit $?
  done
done
