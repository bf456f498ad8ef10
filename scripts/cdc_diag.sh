#!/bin/bash
# Diagnostics for the explicit-list kernel on content-defined lists: A/B of
# builds, the length-class width, and PMC passes of the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/cdc_diag}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"; return $rc; }
step ab 300 python -u scripts/cdc_ab.py "$@" || exit $?
for cb in ${CLASS_BITS:-4 5 6}; do
  SF_TABLE_CLASS_BITS=$cb CDC_ONLY=1 step class$cb 120 python -u scripts/cdc_ab.py || exit $?
done
[ -n "$NO_PMC" ] && exit 0
export CDC_ONLY=1 CDC_ROUNDS=1 CDC_REPS=5
step stats 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 scripts/cdc_ab.py || exit $?
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_mem 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/pmc_mem" -o pmc -- python3 scripts/cdc_ab.py || exit $?
exit 0
