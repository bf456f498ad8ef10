#!/bin/bash
# Round 6: flakiness check of the final build -- the whole GPU suite twice
# more in fresh processes, then the alternating-call stress and the C
# consumer's many-file command at the default settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r
for r in 1 2; do
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r/pytest_gpu_$r.log 2>&1 || exit $?
done
for r in 1 2 3 4 5 6; do
  SF_TEST_STREAM_STAGE_MIB=1 ITERS=60 timeout -k 10 200 python3 scripts/sort_race_stress.py >> gpurun_out/r/stress.log 2>&1 || exit $?
done
