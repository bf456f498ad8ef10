#!/bin/bash
# L2 (TCC) request counters of the explicit-list kernel against the fixed
# kernel on the same bytes (pin the CDC-like list's
# FETCH_SIZE ratio).  One pass per list: TCC_HIT / TCC_MISS (L2 lookups that
# hit / went to the fabric), TCC_EA0_RDREQ (fabric read requests, what
# FETCH_SIZE is derived from) and TCC_REQ (all L2 requests), then the fabric
# reads by size (128 / 64 / 32 B) and those addressed to local DRAM (which
# the Infinity Cache sits in front of); cdc_ab.py's
# fixed-kernel launches of the same pass give the reference.  Also the
# box's counter list.
# usage: bash scripts/table_tcc.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tcc}
mkdir -p "$OUT"
export TMPDIR=/tmp CDC_ROUNDS=1 CDC_REPS=3
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1 || true
for list in cdc list4k; do
  CDC_LISTS=$list timeout -k 10 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum \
    --kernel-trace --output-format csv -d "$OUT/$list" -o pmc -- python3 scripts/cdc_ab.py > "$OUT/$list.log" 2>&1 || exit $?
  CDC_LISTS=$list timeout -k 10 150 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d "$OUT/${list}_sz" -o pmc -- python3 scripts/cdc_ab.py \
    > "$OUT/${list}_sz.log" 2>&1 || exit $?
  for d in $list ${list}_sz; do
    python3 scripts/pmc_summary.py sha1_table_kernel "table_$d=$OUT/$d/pmc_counter_collection.csv" | tee -a "$OUT/summary.txt"
    python3 scripts/pmc_summary.py sha1_fixed_kernel "fixed_$d=$OUT/$d/pmc_counter_collection.csv" | tee -a "$OUT/summary.txt"
  done
done
