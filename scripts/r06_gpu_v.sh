#!/bin/bash
# Round 6, the final build (lists sorted from 65 blocks, scratch pool with no
# release threshold): the whole GPU suite, smoke and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/v/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/v/bench.log 2>&1 || exit $?
