#!/bin/bash
# Critical-path priority of sha1_table_kernel: the
# CDC-like list's timing (interleaved) and FETCH_SIZE per library build.
# usage: bash scripts/prio_thr.sh OUTDIR lib1.so [lib2.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/pthr}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
python -c "import torch; p=torch.cuda.get_device_properties(0); print('device', p.name, 'CUs', p.multi_processor_count)" > "$OUT/device.log" 2>&1
CDC_LISTS=cdc CDC_ROUNDS=8 timeout -k 10 400 python -u scripts/cdc_ab.py "$@" > "$OUT/ab.log" 2>&1 || exit $?
tail -1 "$OUT/ab.log"
export CDC_ONLY=1 CDC_ROUNDS=1 CDC_REPS=5
for L in "$@"; do
  n=$(basename "$L" .so)
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$n" -o pmc -- python3 scripts/cdc_ab.py "$L" > "$OUT/fetch_$n.log" 2>&1 || exit $?
done
