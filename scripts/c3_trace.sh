#!/bin/bash
# Kernel trace of bench.py config 2 and config 3 (20 steps each), to split
# config 3's overhead into launch durations and gaps (scripts/c3_trace.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c3t
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  return $rc
}
step c2 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c2" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit $?
step c3 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c3" -o run -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
