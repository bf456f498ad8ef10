#!/bin/bash
# Host-side AddressSanitizer run of the C-ABI's host pipelines on the GPU box:
# the plain-C consumer (examples/sf_index.c) linked against a library whose
# HOST code is ASan-instrumented (make -C examples asan; the GPU code is not),
# over regular files (pread pipeline, small stages so many stage edges),
# many files (sf_index_files), a FIFO and stdin (sf_index_fd).  Its output
# must equal the uninstrumented build's, and ASan must report nothing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for b in ./examples/build/sf_index ./examples/build/asan/sf_index; do
  [ -x "$b" ] || { echo "missing $b (make -C examples && make -C examples asan, in-tree)"; exit 1; }
done
W=$(mktemp -d /tmp/sf_asan.XXXXXX)
python3 - "$W" <<'EOF'
import os, sys
sys.path.insert(0, os.getcwd())
import oracle
w = sys.argv[1]
sizes = [0, 1, 55, 56, 4095, 4096, 4097, 100_000, (5 << 20) + 77, (9 << 20) + 4096]
for i, n in enumerate(sizes):
    oracle.splitmix_bytes(n, 4000 + i).tofile(os.path.join(w, f"f{i:02d}"))
for i in range(300):
    oracle.splitmix_bytes((i * 7919) % 200_000, 5000 + i).tofile(os.path.join(w, f"s{i:03d}"))
EOF
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:exitcode=99
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:exitcode=98
export SF_TEST_STREAM_STAGE_MIB=1
rc=0
run() {  # name cmd...  (both builds, same input, outputs compared)
  local name=$1; shift
  timeout -k 10 120 ./examples/build/sf_index "$@" > "$W/$name.plain" 2> "$W/$name.plain.err" < "$W/f07" || { echo "$name: plain build failed"; cat "$W/$name.plain.err"; return 1; }
  timeout -k 10 300 ./examples/build/asan/sf_index "$@" > "$W/$name.asan" 2> "gpurun_out/asan_$name.err" < "$W/f07"
  local r=$?
  if [ $r -ne 0 ]; then echo "$name: asan build rc=$r"; tail -30 "gpurun_out/asan_$name.err"; return 1; fi
  [ -s "$W/$name.asan" ] || { echo "$name: no output"; return 1; }
  cmp -s "$W/$name.plain" "$W/$name.asan" || { echo "$name: outputs differ"; return 1; }
  echo "$name: ok ($(wc -l < "$W/$name.asan") lines, asan clean)"
}
run files -b 4096 "$W"/f0* || rc=1
run files_bs1000 -b 1000 "$W"/f0* || rc=1
run many -m -b 4096 "$W"/s* "$W"/f0* || rc=1
run stdin -b 4096 - || rc=1
run buffer -B -b 4096 "$W"/f0* || rc=1
run buffer_small -B -b 64 "$W"/f0[0-7] || rc=1
run shards -s 3 -b 4096 "$W"/f0* || rc=1
SF_INPLACE_MIN_MIB=1 run inplace -B -b 4096 "$W"/f0* || rc=1
SF_INPLACE_MIN_MIB=1 SF_TEST_INPLACE_FAIL_AT=1 run inplace_bounce -B -b 4096 "$W"/f0* || rc=1
run wire -w 104857601 -b 4096 || rc=1
run wire_bs1000 -w 3000001 -b 1000 || rc=1
run lookup -L -b 4096 "$W"/f09 "$W"/f09 || rc=1
run cdc -C "$W"/f0* || rc=1
run zpaq -Z "$W"/f0* || rc=1  # default splice: stamp + stand-in chunker + sf_index_fd_blocks
# the default mode over many files: chunker threads + sf_index_fds_blocks, 1 MiB batches, two passes
run zpaq_par -Z -p 4 "$W"/f0* || rc=1  # the file cut on 4 threads, read once, hashed from HBM (sf_index_fd_cut)
run zpaq_par2 -Z -p 4 -W "$W"/f0* || rc=1  # sf_cut_fd, then sf_index_fd_blocks
run zpaq_many -Z -M -j 4 -S 1 -P 2 "$W"/f0* || rc=1
run zpaq_many_small -Z -M -j 4 -S 1 "$W"/s* || rc=1
run zpaq_many_large -Z -M -j 4 -S 1 -K 1 "$W"/f0* "$W"/s00* || rc=1  # files >= 1 MiB alone through sf_index_fd_cut, in walk order
SF_TEST_CUT_WINDOW_MIB=1 run zpaq_par_win -Z -p 4 "$W"/f0* || rc=1  # 1 MiB windows: double-buffered window seams
run multi -X 0 -b 4096 "$W"/f0* || rc=1  # one file on every visible device from one process
run wire_cdc -v 20000001 || rc=1
# every route over the same files gives the same rows and blocks_hash
same() { [ -s "$1" ] && cmp -s "$1" "$2"; }  # equal, and not two empty outputs
same "$W/zpaq.asan" "$W/zpaq_many.asan" && echo "zpaq_many == zpaq: ok" || { echo "zpaq_many differs from zpaq"; rc=1; }
same "$W/zpaq.asan" "$W/zpaq_par.asan" && echo "zpaq_par == zpaq: ok" || { echo "zpaq_par differs from zpaq"; rc=1; }
same "$W/zpaq.asan" "$W/zpaq_par2.asan" && echo "zpaq_par2 == zpaq: ok" || { echo "zpaq_par2 differs from zpaq"; rc=1; }
for m in buffer shards inplace inplace_bounce multi; do
  same "$W/files.asan" "$W/$m.asan" && echo "$m == files: ok" || { echo "$m differs from files"; rc=1; }
done
mkfifo "$W/pipe"
# the writer's open of the FIFO is inside its own time limit: if the reader
# never opens the other end, the writer still ends and `wait` returns
( sleep 1; timeout -k 5 100 sh -c 'cat "$1" > "$2"' sh "$W/f08" "$W/pipe" ) &
timeout -k 10 120 ./examples/build/asan/sf_index -b 4096 "$W/pipe" > "$W/fifo.asan" 2> gpurun_out/asan_fifo.err
r=$?; wait
if [ $r -ne 0 ]; then echo "fifo: asan build rc=$r"; tail -30 gpurun_out/asan_fifo.err; rc=1
else
  ./examples/build/sf_index -b 4096 "$W/f08" | sed "s|$W/f08|$W/pipe|" > "$W/fifo.plain"
  same "$W/fifo.plain" "$W/fifo.asan" && echo "fifo: ok (asan clean)" || { echo "fifo: outputs differ"; rc=1; }
fi
rm -rf "$W"
exit $rc
