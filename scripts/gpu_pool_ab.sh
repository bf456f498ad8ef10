#!/bin/bash
# Round-5 host A/B session: the default mode's stage size per call and the
# kept helper threads vs threads started per stage (build_ab/old = the
# library before the pool, built from an earlier commit), on the consumer's
# many-file route and on the library's file routes (scripts/pool_ab.py).
# build_ab/old (git-ignored, removed after the round-5 A/B):
#   git archive 239da2a syncfast_amd/csrc include | tar -x -C /tmp/o && \
#   mkdir -p /tmp/o/syncfast_amd/lib && make -C /tmp/o/syncfast_amd/csrc && \
#   mkdir -p build_ab/old && cp /tmp/o/syncfast_amd/lib/libsyncfast_amd.so build_ab/old/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
OUT=gpurun_out/${POOL_OUT:-pool}
mkdir -p $OUT
FORMS=${FORMS:-base,base+G64,base@build_ab/old} timeout -k 10 500 python scripts/default_mode_sweep.py 16 16 256 ${SWEEP_REPS:-2} > $OUT/sweep.log 2>&1 || { echo sweep failed; tail -5 $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
REPS=${AB_REPS:-6} timeout -k 10 500 python scripts/pool_ab.py new=syncfast_amd/lib/libsyncfast_amd.so old=build_ab/old/libsyncfast_amd.so > $OUT/ab.log 2>&1 || { echo ab failed; tail -5 $OUT/ab.log; exit 1; }
cat $OUT/ab.log
