#!/bin/bash
# Round 6: the stream-ordered allocator probe and the two-stream fused-launch
# stress, then the fused cut's double-buffered windows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 120 ./scripts/mallocasync_probe > $OUT/mallocasync_probe.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/fused_two_stream_stress.py --launches 2000 > $OUT/fused_stress.log 2>&1
echo "stress rc=$?" >> $OUT/fused_stress.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fds_blocks.py -k "fd_cut or large_file or native_chunker" > $OUT/cut.log 2>&1 || exit $?
