#!/bin/bash
# Round-5 host A/B session: the GPU tests of the host routes, the default
# mode's batch ramp vs flat batches and the kept helper threads vs threads
# started per stage (build_ab/old = the library before the pool), the pool's
# per-call cost on the box's CPUs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/pool
g++ -O2 -std=c++17 -pthread -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ scripts/pool_probe.cpp syncfast_amd/csrc/sf_pool.cpp -o /tmp/pool_probe && timeout -k 5 60 /tmp/pool_probe > gpurun_out/pool/pool_probe.log 2>&1; cat gpurun_out/pool/pool_probe.log
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_gpu_fds_blocks.py tests/test_gpu_files.py tests/test_gpu_parity.py tests/test_gpu_fd_routes.py > gpurun_out/pool/tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/pool/tests.log; exit 1; }
tail -2 gpurun_out/pool/tests.log
FORMS=ramp,flat,ramp@build_ab/old,flat@build_ab/old timeout -k 10 500 python scripts/default_mode_sweep.py 16 16 256 2 > gpurun_out/pool/sweep.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/pool/sweep.log; exit 1; }
REPS=3 timeout -k 10 400 python scripts/pool_ab.py new=syncfast_amd/lib/libsyncfast_amd.so old=build_ab/old/libsyncfast_amd.so > gpurun_out/pool/ab.log 2>&1 || { echo ab failed; tail -5 gpurun_out/pool/ab.log; exit 1; }
cat gpurun_out/pool/ab.log
