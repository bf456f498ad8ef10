#!/bin/bash
# Round 6: configs[0]'s fused default-mode call, its device tail taken apart
# (scripts/fdcut_tail_probe.py under a kernel trace, SF_TRACE=1 phase times).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/j
SF_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j/prof -o tail -- python3 scripts/fdcut_tail_probe.py > gpurun_out/j/tail.log 2>&1 || exit $?
SF_TRACE=1 timeout -k 10 200 python3 scripts/fdcut_tail_probe.py > gpurun_out/j/tail_noprof.log 2>&1 || exit $?
