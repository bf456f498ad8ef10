#!/bin/bash
# Round-5 A/B: sf_index_files on the non-waiting batch path (in-tree build) vs
# the fused launch with its bounded wait (build_ab/fused: the library built
# from commit b53f593, see scripts/gpu_pool_ab.sh for the recipe).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_gpu_robustness.py tests/test_gpu_files.py > gpurun_out/fused/tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/fused/tests.log; exit 1; }
tail -2 gpurun_out/fused/tests.log
REPS=6 timeout -k 10 600 python scripts/pool_ab.py nowait=syncfast_amd/lib/libsyncfast_amd.so fused=build_ab/fused/libsyncfast_amd.so > gpurun_out/fused/ab.log 2>&1 || { echo ab failed; tail -5 gpurun_out/fused/ab.log; exit 1; }
cat gpurun_out/fused/ab.log
