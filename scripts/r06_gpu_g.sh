#!/bin/bash
# Round 6: the other configs' lines on this build (config 3 batch stream and
# staged, config 5, the 2-rank gloo rehearsal of the per-process form), and
# the single-process library path at N = 1 on configs[3]'s 32 GiB shard, with
# the RCCL self send/recv of every step's table and without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=20 SKIP_BASE=1 EXTRA=1 bash scripts/gpu_round.sh || exit $?
timeout -k 10 400 python bench.py --config 3 --c3-mode staged --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3_staged.log 2>&1 || exit $?
SF_TEST_MULTI_SELF_GATHER=1 timeout -k 10 400 python bench.py --gpus 1 --multi-path library --config 4 --steps 20 --warmup 3 > gpurun_out/bench_lib_c4_selfgather.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --multi-path library --config 4 --steps 20 --warmup 3 --e2e-multi-gib 0 > gpurun_out/bench_lib_c4.log 2>&1 || exit $?
