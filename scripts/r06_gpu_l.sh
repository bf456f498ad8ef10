#!/bin/bash
# Round 6: which part of the fused call's issue section stalls now and then
# (SF_TRACE=1 splits it: buffers, list upload, launch, digests back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/l
for r in 1 2; do
  CALLS=16 SF_TRACE=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/l/default_$r.log 2>&1 || exit $?
  CALLS=16 SF_TRACE=1 SF_TEST_TABLE_SORT=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/l/sorted_$r.log 2>&1 || exit $?
done
