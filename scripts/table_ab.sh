#!/bin/bash
# The explicit-list kernel's A/B session: interleaved
# timing of library builds on the CDC-like 4 GiB list, the 4 KiB list and the
# fixed kernel (scripts/cdc_ab.py), per-wave traces of the traced builds
# (scripts/table_trace.py), and a PMC pass (cycles, waves, VALU) of the
# in-tree build.  Every step under its own time limit; the first failure ends.
# usage: bash scripts/table_ab.sh OUTDIR "lib1 lib2 ..." "tracelib1 tracelib2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tab}
LIBS=$2
TRACES=$3
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
step ab 400 python -u scripts/cdc_ab.py $LIBS || exit $?
for t in $TRACES; do
  n=$(basename "$t" .so)
  step "trace_$n" 200 python -u scripts/table_trace.py "$t" "$OUT/trace_$n.npz" || exit $?
done
[ -n "$NO_PMC" ] && exit 0
export CDC_ROUNDS=1 CDC_REPS=3
step pmc_sq 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 scripts/cdc_ab.py || exit $?
exit 0
