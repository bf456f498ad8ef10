#!/bin/bash
# Compile sf_capi.hip (device only) with extra flags and compare the hot loop
# of sha1_fixed_chained_kernel<128> with sha1_fixed_kernel<128,1,false>'s.
# usage: scripts/isa_loop_cmp.sh "<extra flags>"
set -e
D=$(mktemp -d /tmp/isa_cmp.XXXX)
cd "$(dirname "$0")/../syncfast_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-sched-strategy=max-ilp $1 \
  --cuda-device-only -S -o "$D/k.s" sf_capi.hip
python3 ../../scripts/isa_loop_cmp.py "$D/k.s"
rm -rf "$D"
