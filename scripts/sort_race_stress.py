#!/usr/bin/env python3
"""Debug (round 6): a high-rate form of the C consumer's intermittent wrong
digests.  One process alternates, ITERS times, a many-file batch through
sf_index_fds_blocks (small stages: SF_TEST_STREAM_STAGE_MIB=1, two streams)
and a 2 MiB file through sf_index_fd_cut, checking every digest against the
oracle's (computed once).  Settings from the environment (SF_TEST_STREAM_POOL,
SF_TEST_TABLE_SORT, ...); prints one JSON line: iterations with a wrong row,
per route."""
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import oracle
    from syncfast_amd import _lib, host
    Z = ctypes.CDLL(os.path.join(ROOT, "examples", "build", "libzpaq_standin.so"))
    Z.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    Z.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    ops = Z.sf_zpaq_standin_ops(13, 32768)
    tmp = tempfile.mkdtemp()
    rng = np.random.default_rng(4)
    files = []
    for k, n in enumerate([int(x) for x in rng.integers(0, 300_000, 40)]):
        p = os.path.join(tmp, f"s{k:03d}")
        d = oracle.splitmix_bytes(n, 900 + k)
        d.tofile(p)
        sizes = oracle.zpaq_standin_sizes(d).astype(np.uint32) if n else np.zeros(0, np.uint32)
        offs = np.concatenate([[0], np.cumsum(sizes, dtype=np.uint64)[:-1]]).astype(np.uint64) if n else \
            np.zeros(0, np.uint64)
        want = oracle.index_blocks(d, offs, sizes) if n else np.zeros((0, 20), np.uint8)
        files.append((p, offs, sizes, want))
    big = oracle.splitmix_bytes(2 << 20, 947)
    bp = os.path.join(tmp, "big")
    big.tofile(bp)
    bsz = oracle.zpaq_standin_sizes(big).astype(np.uint32)
    boff = np.concatenate([[0], np.cumsum(bsz, dtype=np.uint64)[:-1]]).astype(np.uint64)
    bwant = oracle.index_blocks(big, boff, bsz)
    iters = int(os.environ.get("ITERS", "100"))
    bad = {"fds": 0, "fd_cut": 0}
    t0 = time.perf_counter()
    for it in range(iters):
        fds = [os.open(p, os.O_RDONLY) for p, *_ in files]
        try:
            rows, first, _bh, st = host.index_fds_blocks(fds, [(o, z) for _p, o, z, _w in files])
        finally:
            for fd in fds:
                os.close(fd)
        ok = True
        for k, (_p, _o, _z, w) in enumerate(files):
            if int(st[k]) != 0 or not np.array_equal(rows["sha1"][first[k]:first[k + 1]].reshape(-1, 20), w):
                ok = False
        bad["fds"] += not ok
        fd = os.open(bp, os.O_RDONLY)
        try:
            r2, _ = host.index_fd_cut(fd, ops, 4)
        finally:
            os.close(fd)
        bad["fd_cut"] += not np.array_equal(r2["sha1"].reshape(-1, 20), bwant)
    print(json.dumps({"iters": iters, "bad_iterations": bad, "s": round(time.perf_counter() - t0, 2),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("SF_")}}), flush=True)


if __name__ == "__main__":
    main()
