cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu2.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu2.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench2.log 2>&1 || exit $?
tail -1 gpurun_out/bench2.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --weak > gpurun_out/bench2_weak.log 2>&1 || exit $?
tail -1 gpurun_out/bench2_weak.log
exit $rc
