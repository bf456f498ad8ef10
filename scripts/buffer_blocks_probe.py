"""End-to-end rate of sf_index_buffer_blocks (host buffer + explicit,
content-defined-like block list -> rows + blocks_hash) beside sf_index_buffer
(fixed 4 KiB tiling) on the same host bytes (not a test).

The list is what the reference's default chunker produces in shape
(src/index.rs:40-41: ZPAQ 13 bits = 8 KiB mean, 32 KiB cap): geometric sizes,
mean 8 KiB, capped at 32 KiB, tiling the buffer.  Best of REPS calls each;
a sample of digests is checked with hashlib.
Usage: python scripts/buffer_blocks_probe.py [GiB ...]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd import device, host  # noqa: E402

GiB = 1 << 30


def main():
    for arg in (sys.argv[1:] or ["4"]):
        one(float(arg))


def one(gib):
    reps = int(os.environ.get("REPS", "3"))
    n = int(gib * GiB)
    import torch
    data = device.splitmix_tensor(n, 0x5EED0000, torch.device("cuda:0")).cpu().numpy()  # host bytes
    rng = np.random.default_rng(1)
    sizes = np.minimum(rng.geometric(1.0 / 8192, size=n // 4096 + 64), 32768).astype(np.uint64)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    b = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    offs, szs = b[:-1], np.diff(b).astype(np.uint32)
    res = {"bytes": n, "blocks": int(offs.size), "mean_block": n / offs.size}
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "sf_bb_probe.bin")
    data.tofile(path)  # page-cache resident for the file forms
    for name, fn in (("fixed4k", lambda: host.index_buffer(data, 4096)),
                     ("cdc_list", lambda: host.index_buffer_blocks(data, offs, szs)),
                     ("file_fixed4k", lambda: host.index_file(path, 4096)),
                     ("file_cdc_list", lambda: host.index_file_blocks(path, offs, szs))):
        best = None
        out = None
        for _ in range(reps):
            t0 = time.perf_counter()
            out = fn()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        rows = out[0] if isinstance(out, tuple) else out
        for i in (0, rows.size // 2, rows.size - 1):
            o, s = int(rows["offset"][i]), int(rows["size"][i])
            assert bytes(rows["sha1"][i]) == hashlib.sha1(data[o:o + s].tobytes()).digest(), (name, i)
        res[name] = {"s": round(best, 4), "GB/s": round(n / best / 1e9, 2), "GiB/s": round(n / best / GiB, 2)}
        print(name, res[name], flush=True)
    os.unlink(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
