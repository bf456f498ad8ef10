#!/bin/bash
# Round 6, first GPU pass: the fused wait's poll (robustness tests, the XCD
# litmus), the multi-device forms (gather streams, the bench's library path at
# N = 1), the windowed cut's fallback and the large-file walk.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06a
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_robustness.py tests/test_gpu_multi.py -s > $OUT/robust.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/xcd_litmus.py --trials 100 > $OUT/litmus.log 2>&1 || exit $?
timeout -k 10 400 $T tests/test_gpu_fds_blocks.py -k "fd_cut or large_file" > $OUT/cut.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_c_consumer.py -k "default_mode or parallel_cut" > $OUT/cconsumer.log 2>&1 || exit $?
