#!/bin/bash
# Round 6: configs[0]'s fused call -- host phases (SF_TRACE=1 with issue and
# last-harvest times) and the explicit-list kernel's time in its one launch,
# the list in file order (default below 2^17 blocks) against sorted by length
# class (SF_TEST_TABLE_SORT=1), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k
for r in 1 2; do
  CALLS=12 SF_TRACE=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/k/default_$r.log 2>&1 || exit $?
  CALLS=12 SF_TRACE=1 SF_TEST_TABLE_SORT=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/k/sorted_$r.log 2>&1 || exit $?
done
SF_TEST_TABLE_SORT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k/prof_sorted -o t -- python3 scripts/fdcut_tail_probe.py > gpurun_out/k/prof_sorted.log 2>&1 || exit $?
