#!/bin/bash
# PMC passes of the explicit-list kernel, one library and one list per run
# (so every dispatch of sha1_table_kernel in a CSV is that list's):
#   rocprofv3 --pmc GRBM_GUI_ACTIVE + SQ counters, then FETCH_SIZE,
# over scripts/cdc_ab.py (CDC_LISTS=<list>, 1 round of CDC_REPS launches);
# the fixed kernel on the same bytes from a cdc_ab.py pass without a list
# filter.  Summaries: scripts/pmc_summary.py.
# usage: bash scripts/table_pmc.sh OUTDIR lib1.so [lib2.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tpmc}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp CDC_ROUNDS=1 CDC_REPS=4
SQ="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
for L in "$@"; do
  n=$(basename "$L" .so)
  for list in cdc list4k; do
    CDC_LISTS=$list timeout -k 10 150 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/${n}_${list}_sq" -o pmc -- python3 scripts/cdc_ab.py "$L" > "$OUT/${n}_${list}_sq.log" 2>&1 || exit $?
    CDC_LISTS=$list timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/${n}_${list}_fetch" -o pmc -- python3 scripts/cdc_ab.py "$L" > "$OUT/${n}_${list}_fetch.log" 2>&1 || exit $?
    python3 scripts/pmc_summary.py sha1_table_kernel "${n}_${list}=$OUT/${n}_${list}_sq/pmc_counter_collection.csv" "${n}_${list}_fetch=$OUT/${n}_${list}_fetch/pmc_counter_collection.csv" | tee -a "$OUT/summary.txt"
  done
done
L=$1
timeout -k 10 150 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/fixed_sq" -o pmc -- python3 scripts/cdc_ab.py "$L" > "$OUT/fixed_sq.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py sha1_fixed_kernel "fixed=$OUT/fixed_sq/pmc_counter_collection.csv" | tee -a "$OUT/summary.txt"
