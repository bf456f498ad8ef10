#!/bin/bash
# Round 6 debug: scripts/sort_race_stress.py under each scratch pool and sort setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/o
for r in 1 2; do
  for v in "SF_STREAM_POOL=0" "SF_STREAM_POOL=1" "SF_STREAM_POOL=0 SF_TEST_TABLE_SORT=0"; do
    env $v SF_TEST_STREAM_STAGE_MIB=1 ITERS=60 timeout -k 10 200 python3 scripts/sort_race_stress.py >> gpurun_out/o/stress.log 2>&1 || exit $?
  done
done
