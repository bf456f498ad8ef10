#!/bin/bash
# bench.py config 3 under a kernel trace with --events region (no timing
# event between launches), to compare launch durations with c3_trace.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c3t
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c3_region" -o run -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --events region > "$OUT/c3_region.log" 2>&1
rc=$?; echo "== c3_region rc=$rc"; exit $rc
