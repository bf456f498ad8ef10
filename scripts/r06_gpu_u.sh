#!/bin/bash
# Round 6: the scratch pool with no release threshold (and, rerun, lists sorted
# from 65 blocks) -- the list, file and
# robustness GPU tests, and the alternating-call stress.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/u
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_robustness.py tests/test_gpu_table_order.py tests/test_gpu_fds_blocks.py tests/test_c_consumer.py tests/test_wire.py tests/test_block_set.py -m gpu > gpurun_out/u/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  SF_TEST_STREAM_STAGE_MIB=1 ITERS=60 timeout -k 10 200 python3 scripts/sort_race_stress.py >> gpurun_out/u/stress.log 2>&1 || exit $?
done
