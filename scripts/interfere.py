"""Rank-0 interference rehearsal for the N>1 bench on one GPU (not a test).

At N GPUs, rank 0 receives (N-1) x 40 MiB of digest tables per step while its
next sha1_fixed_kernel runs (bench.py pipelines the gather one step behind).
This times the headline kernel alone, a D2D copy of that volume alone, and
both together on two streams, so the overlap the N=8 run depends on can be
checked without 8 GPUs.  Usage: python scripts/interfere.py [--peers 7]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd.device import fill_splitmix, index_device  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--peers", type=int, default=7)
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    dev = torch.device("cuda:0")
    n, bs = 1 << 33, 4096
    data = torch.empty(n, dtype=torch.uint8, device=dev)
    fill_splitmix(data, 0x5EED0000)
    dig = torch.empty((n // bs, 20), dtype=torch.uint8, device=dev)
    vol = a.peers * dig.numel()
    src = torch.empty(vol, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]

    def run(kernel, copy, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if kernel:
                index_device(data, bs, out=dig, stream=s1)
            if copy == "nocu":  # hipMemcpyDeviceToDeviceNoCU: SDMA engine, no CUs
                assert hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), vol, 1024, s2.cuda_stream) == 0
            elif copy:
                with torch.cuda.stream(s2):
                    dst.copy_(src)
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    t_end = time.perf_counter() + 0.5  # clock ramp, as bench.py's setup
    while time.perf_counter() < t_end:
        run(True, False, 1)
    out = {"copy_mib": vol / 2**20}
    for name, k, c in (("kernel", True, False), ("copy", False, True), ("both", True, True),
                       ("copy_nocu", False, "nocu"), ("both_nocu", True, "nocu"),
                       ("kernel_again", True, False)):
        out[name + "_ms"] = round(run(k, c, a.steps), 4)
    out["overhead_frac"] = round(out["both_ms"] / out["kernel_ms"] - 1.0, 4)
    out["overhead_frac_nocu"] = round(out["both_nocu_ms"] / out["kernel_ms"] - 1.0, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
