#!/bin/bash
# Round 6: explicit lists sorted by length from two waves (128 blocks) on:
# the whole GPU suite, configs[0]'s fused call (phase times), and the bench
# line with its default-mode legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/m/pytest_gpu.log 2>&1 || exit $?
CALLS=12 SF_TRACE=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/m/tail.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/m/bench.log 2>&1 || exit $?
