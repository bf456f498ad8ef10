#!/bin/bash
# Kernel trace of scripts/c3_seq.py (config 3 launch durations, back to back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c3s}
mkdir -p $OUT
echo "== seq"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/seq" -o run -- python3 scripts/c3_seq.py "$@" > "$OUT/seq.log" 2>&1
rc=$?; echo "== seq rc=$rc"; tail -2 "$OUT/seq.log"; exit $rc
