#!/bin/bash
# Content-defined block list through sha1_table_kernel: timing, rocprofv3
# kernel stats and separate PMC passes (traffic, VALU, waits, LDS, TCP).
# Every step under its own time limit; the first failure ends the script.
# usage: bash scripts/cdc_prof.sh OUTDIR [libs for the A/B...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/cdc}; shift
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
step ab 300 python -u scripts/cdc_ab.py "$@" || exit $?
[ -n "$NO_PROF" ] && exit 0
export CDC_ONLY=1 CDC_ROUNDS=1 CDC_REPS=5
step stats 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 scripts/cdc_ab.py || exit $?
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o pmc -- python3 scripts/cdc_ab.py || exit $?
step pmc_mem 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_mem" -o pmc -- python3 scripts/cdc_ab.py || exit $?
exit 0
