"""The bench line's default_mode_files leg alone (bench.default_mode_files):
the reference's content-defined mode over many files on disk, stand-in
chunker on 1 and N threads -> sf_index_fds_blocks, beside the per-file loop.

usage: python scripts/default_mode_probe.py [threads]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402
from syncfast_amd import device  # noqa: E402


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else max(1, min(16, len(os.sched_getaffinity(0))))
    data = torch.empty(8 << 30, dtype=torch.uint8, device="cuda:0")
    device.fill_splitmix(data, bench.SEED, 0)
    torch.cuda.synchronize()
    print(json.dumps(bench.default_mode_files(data, threads)), flush=True)


if __name__ == "__main__":
    main()
