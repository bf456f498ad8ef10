#!/bin/bash
# Round 6 full GPU pass, part 2: host ASan over every host route,
# sf_index_fd_cut's double-buffered windows against round 5's library
# (build_ab/libsf_r5.so), and the explicit-list kernel's traffic record
# (TCC request counters, FETCH_SIZE + SQ passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SKIP_BASE=1 ASAN=1 bash scripts/gpu_round.sh || exit $?
mkdir -p gpurun_out/cutab
REPS=3 timeout -k 10 400 python -u scripts/fd_cut_ab.py r6=syncfast_amd/lib/libsyncfast_amd.so r5=build_ab/libsf_r5.so > gpurun_out/cutab/fd_cut_ab.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/table_tcc.sh gpurun_out/tcc > gpurun_out/tcc.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/table_pmc.sh gpurun_out/tpmc syncfast_amd/lib/libsyncfast_amd.so > gpurun_out/tpmc.log 2>&1 || exit $?
