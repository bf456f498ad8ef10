"""Wave-quantisation probe for sha1_fixed_kernel (not a test).

The headline launch is 2^21 blocks = 32768 waves over 3072 wave slots
(256 CUs x 4 SIMDs x 3 waves): 10.67 slot rounds.  Timing launches of
30720 / 32768 / 33792 / 36864 waves (10, 10.67, 11, 12 rounds) shows how much
the partial last round costs.  Usage: python scripts/tail_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd.device import fill_splitmix, index_device  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    bs = 4096
    waves = [30720, 32768, 33792, 36864]
    n_max = max(waves) * 64 * bs
    data = torch.empty(n_max, dtype=torch.uint8, device=dev)
    fill_splitmix(data, 0x5EED0000)
    dig = torch.empty((n_max // bs, 20), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        index_device(data[: waves[1] * 64 * bs], bs, out=dig, stream=s)
        s.synchronize()
    out = {}
    for rep in range(2):
        for w in waves:
            view = data[: w * 64 * bs]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                index_device(view, bs, out=dig, stream=s)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 10
            out[f"{w}"] = {"ms": round(ms, 4), "us_per_wave_round": round(ms * 1e3 / (w / 3072), 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
