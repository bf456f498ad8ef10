#!/bin/bash
# Config 5 (64 KiB blocks) vs config 2 (4 KiB): where does the 64 KiB launch
# lose its expected ~1% per-byte advantage?  SQ issue/wait counters and the
# TCP address-translation counters of both launches, one pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
step() {  # name cmd... ; stops the script on a timeout/kill/abort/segv
  local name=$1; shift
  echo "== $name"
  timeout -k 10 -s KILL 120 "$@" > "gpurun_out/c5/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/c5/$name.log"
  case $rc in 124|137|134|139) exit $rc ;; esac
  return 0
}
rocprofv3 --list-avail > gpurun_out/c5/avail.txt 2>&1 || true
B2="python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
B5="python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
for c in 2 5; do
  B=$B2; [ $c = 5 ] && B=$B5
  step sq_c$c rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/c5/sq_c$c -o pmc -- $B
  step tlb_c$c rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCP_LATENCY_sum --kernel-trace --output-format csv -d gpurun_out/c5/tlb_c$c -o pmc -- $B
  step ta_c$c rocprofv3 --pmc TA_BUSY_avr TA_BUFFER_LOAD_WAVEFRONTS_sum TCC_EA0_RDREQ_sum TCC_HIT_sum --kernel-trace --output-format csv -d gpurun_out/c5/ta_c$c -o pmc -- $B
done
exit 0
