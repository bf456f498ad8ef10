#!/bin/bash
# Round 6, last pass on this build: the multi-GPU GPU tests (the bench's
# library path included, with its new watchdog), a kernel trace of the
# library path at N = 1 with the RCCL self send/recv (hash kernels on the hash
# stream, RCCL kernels on the gather stream), and three default bench runs
# back to back (the driver's command) for the headline's spread.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/h
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/h/pytest_multi.log 2>&1 || exit $?
SF_TEST_MULTI_SELF_GATHER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h/libprof -o lib -- python3 bench.py --gpus 1 --multi-path library --config 4 --steps 10 --warmup 2 --e2e-multi-gib 0 > gpurun_out/h/libprof.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 400 python bench.py > gpurun_out/h/bench_$i.log 2>&1 || exit $?
done
