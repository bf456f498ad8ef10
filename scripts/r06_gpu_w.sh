#!/bin/bash
# Round 6, final build: the headline, config 3 (stream and self-contained
# batches) and config 5 back to back on ONE box, so their ratios are free of
# the box-to-box clock spread.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/x
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-cdc-list --no-default-mode > gpurun_out/x/c2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/x/c3.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/x/c3_staged.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/x/c5.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-cdc-list --no-default-mode > gpurun_out/x/c2_again.log 2>&1 || exit $?
