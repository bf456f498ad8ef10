#!/bin/bash
# Round 6: the no-wait fused many-file launch -- its tests, the config-3
# staged bench A/B (fused vs blocks-then-chains), and sf_index_files with
# each (pool_ab.py, SF_BATCH_FUSED=1 / 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06c
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_robustness.py tests/test_gpu_parity.py tests/test_gpu_files.py tests/test_gpu_fuzz.py tests/test_gpu_table_order.py tests/test_gpu_launch_split.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_fullsize.py -k "config3" > $OUT/fullsize_c3.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/fused_two_stream_stress.py --launches 2000 > $OUT/fused_stress.log 2>&1 || exit $?
for r in 1 2; do
  for f in 1 0; do
    SF_BATCH_FUSED=$f timeout -k 10 300 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_staged_fused${f}_$r.log 2>&1 || exit $?
  done
done
REPS=4 timeout -k 10 900 python -u scripts/pool_ab.py fused=syncfast_amd/lib/libsyncfast_amd.so,SF_BATCH_FUSED=1 unfused=syncfast_amd/lib/libsyncfast_amd.so,SF_BATCH_FUSED=0 > $OUT/files_ab.log 2>&1 || exit $?
