#!/bin/bash
# Round 6: the no-wait fused launch with LDS-staged chain slices: tests and
# the config-3 staged bench, fused vs blocks-then-chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06d
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_robustness.py tests/test_gpu_parity.py -k "batch or staged or wide or files or null" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_fullsize.py -k "config3" > $OUT/fullsize_c3.log 2>&1 || exit $?
for r in 1 2; do
  for f in 1 0; do
    SF_BATCH_FUSED=$f timeout -k 10 300 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_staged_fused${f}_$r.log 2>&1 || exit $?
  done
done
for st in 4 8 32; do
  SF_TEST_STAGES=$st timeout -k 10 300 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_staged_S${st}.log 2>&1 || exit $?
done
