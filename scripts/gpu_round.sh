#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Stops at the first step that crashes / times out (exit >= 2 from pytest
# means an internal error; 124/137/134/139 mean timeout/kill/abort/segv).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-10}"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
if [ -n "$PROBE" ]; then
  run valu_probe 300 ./scripts/valu_probe || exit $?
fi
rc=0
if [ -z "$SKIP_BASE" ]; then  # SKIP_BASE=1: only the optional steps below
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread
rc=$?; if [ $rc -ge 2 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py --steps "$STEPS" --warmup 2 --cpu-seconds 8 || exit $?
fi
if [ -n "$EXTRA" ]; then
  run bench_c3 600 python bench.py --config 3 --steps "$STEPS" --warmup 2 --no-cpu-baseline || exit $?
  run bench_c5 600 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline || exit $?
  # N>1 code path rehearsal on one GPU: bench.py starts its 2 ranks itself,
  # both share cuda:0, gloo gather
  run bench_rehearsal2 600 python bench.py --gpus 2 --steps 5 --warmup 1 --shard-gib 1 --dist-backend gloo --no-cpu-baseline || exit $?
fi
if [ -n "$ASAN" ]; then
  # host-side ASan + UBSan of the C-ABI's host pipelines (make -C examples asan first)
  run asan_host 600 bash scripts/asan_host.sh || exit $?
fi
if [ -n "$CDC" ]; then
  # the content-defined-like list through sha1_table_kernel: timing A/B
  # against the 4 KiB list and the fixed kernel, kernel stats, PMC passes
  run cdc_prof 900 bash scripts/cdc_prof.sh gpurun_out/cdc || exit $?
fi
if [ -n "$PROFILE" ]; then
  # --no-e2e --no-cdc-list --no-default-mode: only the timed kernel launches, so rocprof's average is the
  # bench line's kernel_ms (the end-to-end leg launches 256 MiB stages)
  B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-cdc-list --no-default-mode"
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- $B || exit $?
  run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o pmc -- $B || exit $?
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- $B || exit $?
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- $B || exit $?
  python scripts/pmc_traffic.py gpurun_out/pmc_fetch/pmc_counter_collection.csv gpurun_out/pmc_write/pmc_counter_collection.csv config2 8589934592 gpurun_out/traffic.json
  # the bench line again, now with this build's PMC traffic attached
  run bench_traffic 600 python bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline --traffic-file gpurun_out/traffic.json || exit $?
fi
exit $rc
