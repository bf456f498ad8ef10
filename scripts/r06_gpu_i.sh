#!/bin/bash
# Round 6: the bench's library path with two receive tables per device --
# the multi-GPU GPU tests, a kernel trace at N = 1 with the RCCL self
# send/recv (do the RCCL kernels on the gather stream now overlap the next
# step's hashing?), and the N = 1 library lines with and without the exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/i
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/i/pytest_multi.log 2>&1 || exit $?
SF_TEST_MULTI_SELF_GATHER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i/libprof -o lib -- python3 bench.py --gpus 1 --multi-path library --config 4 --steps 10 --warmup 2 --e2e-multi-gib 0 > gpurun_out/i/libprof.log 2>&1 || exit $?
SF_TEST_MULTI_SELF_GATHER=1 timeout -k 10 400 python bench.py --gpus 1 --multi-path library --config 4 --steps 20 --warmup 3 --e2e-multi-gib 0 > gpurun_out/i/bench_lib_c4_selfgather.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --multi-path library --config 4 --steps 20 --warmup 3 > gpurun_out/i/bench_lib_c4.log 2>&1 || exit $?
