#!/bin/bash
# Content-defined list through sha1_table_kernel, several library builds:
# interleaved timing at 4 GiB (with the 4 KiB list and the fixed kernel) and
# at 16 GiB (the grid's tail amortised 4x), then per library a rocprofv3
# kernel-stats pass and separate PMC passes (traffic; VALU, waits, clock).
# Every step under its own time limit; the first failure ends the script.
# usage: bash scripts/cdc_variants.sh OUTDIR lib1.so [lib2.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/cdcv}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  return $rc
}
step ab 400 python -u scripts/cdc_ab.py "$@" || exit $?
CDC_GIB=16 CDC_LISTS=cdc CDC_ROUNDS=3 step ab16 400 python -u scripts/cdc_ab.py "$@" || exit $?
[ -n "$NO_PROF" ] && exit 0
export CDC_ONLY=1 CDC_ROUNDS=1 CDC_REPS=5
for L in "$@"; do
  n=$(basename "$L" .so)
  step "stats_$n" 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$n" -o run -- python3 scripts/cdc_ab.py "$L" || exit $?
  step "fetch_$n" 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$n" -o pmc -- python3 scripts/cdc_ab.py "$L" || exit $?
  step "sq_$n" 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq_$n" -o pmc -- python3 scripts/cdc_ab.py "$L" || exit $?
done
exit 0
