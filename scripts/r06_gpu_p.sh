#!/bin/bash
# Round 6 debug: scripts/sort_race_stress.py per scratch pool -- 0 the
# device's default pool (hipMallocAsync), 1 the library's own pool (shipped:
# reuse on the freeing stream only, 1 GiB kept), 2 own pool with cross-stream
# reuse on, 3 own pool releasing at every synchronisation -- and the default
# pool with the list sort off (no scratch at all); every setting in 4
# processes of 60 iterations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/p
for r in 1 2 3 4; do
  for v in "SF_TEST_STREAM_POOL=0" "SF_TEST_STREAM_POOL=1" "SF_TEST_STREAM_POOL=2" "SF_TEST_STREAM_POOL=3" "SF_TEST_STREAM_POOL=0 SF_TEST_TABLE_SORT=0"; do
    env $v SF_TEST_STREAM_STAGE_MIB=1 ITERS=60 timeout -k 10 200 python3 scripts/sort_race_stress.py >> gpurun_out/p/stress.log 2>&1 || exit $?
  done
done
