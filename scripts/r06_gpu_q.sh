#!/bin/bash
# Round 6: small explicit lists sorted (from 128 blocks) + the library's own
# scratch pool -- the whole GPU suite, the alternating-call stress and the C
# consumer repro at the default settings, configs[0]'s fused call, the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/q/pytest_gpu.log 2>&1 || exit $?
for r in 1 2 3 4; do
  SF_TEST_STREAM_STAGE_MIB=1 ITERS=60 timeout -k 10 200 python3 scripts/sort_race_stress.py >> gpurun_out/q/stress.log 2>&1 || exit $?
done
ROUNDS=6 timeout -k 10 300 python3 scripts/sort_small_repro.py > gpurun_out/q/repro.log 2>&1 || exit $?
CALLS=12 SF_TRACE=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/q/tail.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/q/bench.log 2>&1 || exit $?
