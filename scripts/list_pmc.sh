#!/bin/bash
# PMC passes of sha1_table_kernel over one list (CDC_LISTS) for each library
# given: SQ issue/wait counters, TA/TCP request counters, traffic.
# usage: CDC_LISTS=list4k bash scripts/list_pmc.sh OUTDIR lib1.so [lib2.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/list_pmc}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp CDC_ROUNDS=1 CDC_REPS=5
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "$OUT/$name.log"; return $rc; }
i=0
for lib in "$@"; do
  i=$((i+1))
  step sq$i 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq$i" -o pmc -- python3 scripts/cdc_ab.py "$lib" || exit $?
  step ta$i 120 rocprofv3 --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCC_EA0_RDREQ_sum TCC_HIT_sum --kernel-trace --output-format csv -d "$OUT/ta$i" -o pmc -- python3 scripts/cdc_ab.py "$lib" || exit $?
  step fetch$i 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch$i" -o pmc -- python3 scripts/cdc_ab.py "$lib" || exit $?
done
for j in $(seq 1 $i); do for p in sq ta fetch; do python3 scripts/pmc_summary.py sha1_table_kernel $p$j=$OUT/$p$j/pmc_counter_collection.csv; done; done | tee "$OUT/summary.txt"
