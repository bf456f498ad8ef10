#!/bin/bash
# sf_index_fd_cut's phase times (SF_TRACE=1) on configs[0]'s 64 MiB file, four
# passes in one process, then the two-call route (-W) for comparison.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ftrace
python3 -c "
import sys; sys.path.insert(0,'.')
import oracle; oracle.splitmix_bytes(64<<20, 0x5EED0000).tofile('/tmp/f64m')"
SF_TRACE=1 timeout -k 10 60 ./examples/build/sf_index -Z -p 16 -T /tmp/f64m /tmp/f64m /tmp/f64m /tmp/f64m > /dev/null 2> gpurun_out/ftrace/trace.log
SF_TRACE=1 timeout -k 10 60 ./examples/build/sf_index -Z -p 16 -W -T /tmp/f64m /tmp/f64m /tmp/f64m /tmp/f64m > /dev/null 2>> gpurun_out/ftrace/trace.log
cat gpurun_out/ftrace/trace.log
