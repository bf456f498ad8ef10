#!/bin/bash
# The explicit-list kernel's A/B session (round 5): the in-tree build's list
# tests, then an order-rotated interleaved A/B of library builds on the
# CDC-like 4 GiB list, the 4 KiB list and the fixed kernel (scripts/cdc_ab.py)
# under rocprofv3 --kernel-trace, attributed per launch by
# scripts/table_ktrace.py.  Every step under its own time limit; the first
# failure ends the session.
# usage: bash scripts/gpu_tab_ab.sh OUTDIR "lib1 lib2 ..." [ROUNDS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tab}
LIBS=$2
ROUNDS=${3:-8}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  return $rc
}
if [ -z "$NO_TESTS" ]; then
  step tests 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
    tests/test_gpu_table_order.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_buffer_blocks.py \
    tests/test_gpu_fds_blocks.py tests/test_gpu_launch_split.py || exit $?
fi
export CDC_ROUNDS=$ROUNDS CDC_REPS=3
NL=$(echo $LIBS | wc -w)
step ab 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o kt -- python3 scripts/cdc_ab.py $LIBS || exit $?
KT=$(ls "$OUT"/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -z "$KT" ] && KT=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -1)
python3 scripts/table_ktrace.py "$KT" cdc,list4k "$NL" 3 "$ROUNDS" rot > "$OUT/ktrace_summary.txt" 2>&1
cat "$OUT/ktrace_summary.txt"
exit 0
