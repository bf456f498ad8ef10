#!/bin/bash
# GPU session: full gpu test suite, then config 3 in both modes and config 2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu3.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu3.log; [ $rc -ne 0 ] && exit $rc
for m in stream staged; do
  timeout -k 10 300 python bench.py --config 3 --c3-mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_c3_$m.log
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log
