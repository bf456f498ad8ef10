#!/bin/bash
# Round 6: equal-size batches with blocks_hash as two column halves (no
# waits): tests, the config-3 full-size check, and the shapes A/B against
# blocks-then-chains (round 5's waiting launch: r06e/shapes_r5.log).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06f
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_robustness.py tests/test_gpu_parity.py tests/test_gpu_files.py tests/test_gpu_fuzz.py tests/test_gpu_launch_split.py tests/test_gpu_batch_stream.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_fullsize.py -k "config3" > $OUT/fullsize_c3.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/batch_shapes_ab.py > $OUT/shapes_r6.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/fused_two_stream_stress.py --launches 1000 > $OUT/two_stream_stress.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_staged_$r.log 2>&1 || exit $?
done
REPS=4 timeout -k 10 900 python -u scripts/pool_ab.py halves=syncfast_amd/lib/libsyncfast_amd.so,SF_BATCH_FUSED=1 unfused=syncfast_amd/lib/libsyncfast_amd.so,SF_BATCH_FUSED=0 > $OUT/files_ab.log 2>&1 || exit $?
