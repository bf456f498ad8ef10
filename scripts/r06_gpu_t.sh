#!/bin/bash
# Round 6 debug: the alternating-call stress on a tracing build of the
# library (allocation addresses on stderr), scratch from the default pool.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
for r in 1 2 3; do
  SF_LIB=build_dbg/libsf_dbg.so SF_TEST_STREAM_POOL=0 SF_TRACE=2 SF_TEST_STREAM_STAGE_MIB=1 ITERS=30 timeout -k 10 200 python3 scripts/sort_race_stress.py > gpurun_out/t/out_$r.log 2> gpurun_out/t/trace_$r.log || exit $?
done
