#!/bin/bash
# Records what the GPU box's host offers for the reference CPU path
# (BASELINE.md:25 asks for a timed `syncfast index` run or a probe showing it
# cannot run): Rust toolchain, CPU model / SHA-NI, usable cores.
echo "date: $(date -u +%FT%TZ)"
echo "hostname: $(hostname)"
for t in cargo rustc rustup; do
  p=$(command -v "$t" 2>/dev/null)
  echo "which $t: ${p:-<absent>}"
done
echo "~/.cargo: $(ls -d "$HOME/.cargo" 2>/dev/null || echo '<absent>')"
echo "/usr/local/cargo: $(ls -d /usr/local/cargo 2>/dev/null || echo '<absent>')"
echo "cargo --version: $(cargo --version 2>&1)"
echo "cpu model: $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2-)"
echo "sha_ni: $(grep -m1 -o -w sha_ni /proc/cpuinfo || echo '<absent>')"
echo "nproc (machine): $(nproc --all)"
echo "affinity cpus: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
echo "OMP_NUM_THREADS: ${OMP_NUM_THREADS:-<unset>}"
