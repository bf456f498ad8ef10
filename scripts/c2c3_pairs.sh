#!/bin/bash
# Config 2 and config 3 bench lines alternating on one box (the batch
# stream's overhead over the plain kernel): PAIRS pairs,
# 20 steps each, no CPU baseline / end-to-end / CDC legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/pairs}
mkdir -p "$OUT"
for i in $(seq 1 "${PAIRS:-3}"); do
  for c in 2 3; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-cdc-list \
      > "$OUT/c${c}_$i.json" 2> "$OUT/c${c}_$i.err" || exit $?
    tail -1 "$OUT/c${c}_$i.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$c', $i, d['value'], d['ms_per_step'])"
  done
done
