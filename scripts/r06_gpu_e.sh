#!/bin/bash
# Round 6: batch shapes A/B -- this round's no-wait fused launch (S = 32, 16),
# blocks-then-chains, and round 5's waiting fused launch (build_ab/libsf_r5.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 300 python -u scripts/batch_shapes_ab.py > $OUT/shapes_r6.log 2>&1 || exit $?
SF_AB_OLD=1 SF_LIB=build_ab/libsf_r5.so timeout -k 10 300 python -u scripts/batch_shapes_ab.py > $OUT/shapes_r5.log 2>&1 || exit $?
