#!/usr/bin/env python3
"""sf_index_fd_cut (one file, the default mode: the caller's chunker on 16
threads, the file read once, hashed on the GPU) across builds of the library:
round 6's double-buffered windows (a window's list upload, kernel and digests
run while the next window is read and cut) against round 5's one window at a
time.  Files of 64 MiB, 600 MiB and 2 GiB in the page cache, the stand-in
chunker (examples/build/libzpaq_standin.so); each library in its own process
(SF_LIB), interleaved, REPS rounds; per call the best of 3 after a warm-up.
Raw ctypes: round 5's library lacks this round's symbols.

usage: python scripts/fd_cut_ab.py NAME=LIB [NAME=LIB ...]
       python scripts/fd_cut_ab.py --child DIR"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
SIZES = {"64MiB": 64 << 20, "600MiB": (600 << 20) + 5, "2GiB": 2 << 30}


def child(d):
    L = ctypes.CDLL(os.environ["SF_LIB"])
    Z = ctypes.CDLL(os.path.join(ROOT, "examples", "build", "libzpaq_standin.so"))
    Z.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    Z.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    ops = Z.sf_zpaq_standin_ops(13, 32768)
    vp = ctypes.c_void_p
    L.sf_index_fd_cut.argtypes = [ctypes.c_int, vp, vp, ctypes.c_uint32, vp, vp, vp]
    L.sf_free_rows.argtypes = [vp]
    res = {}
    for name in SIZES:
        p = os.path.join(d, name)
        fd = os.open(p, os.O_RDONLY)
        try:
            def call():
                rows, n, bh = vp(), ctypes.c_uint64(), (ctypes.c_uint8 * 20)()
                t0 = time.perf_counter()
                rc = L.sf_index_fd_cut(fd, None, ops, 16, ctypes.byref(rows), ctypes.byref(n), bh)
                dt = time.perf_counter() - t0
                assert rc == 0, rc
                L.sf_free_rows(rows)
                return dt, n.value, bytes(bh).hex()
            call()
            best = min(call() for _ in range(3))
            res[name] = {"GB/s": round(os.path.getsize(p) / best[0] / 1e9, 3), "blocks": best[1], "bh": best[2][:16]}
        finally:
            os.close(fd)
    print(json.dumps(res), flush=True)


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    libs = [a.split("=", 1) for a in sys.argv[1:]]
    reps = int(os.environ.get("REPS", "3"))
    d = tempfile.mkdtemp(prefix="sf_cutab_")
    try:
        import numpy as np
        rng = np.random.default_rng(5)
        src = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
        for name, n in SIZES.items():
            with open(os.path.join(d, name), "wb") as f:
                left = n
                while left:
                    k = min(left, src.size)
                    src[:k].tofile(f)
                    left -= k
        for r in range(reps):
            order = libs[r % len(libs):] + libs[:r % len(libs)]
            for name, lib in order:
                out = subprocess.run([sys.executable, __file__, "--child", d], capture_output=True, text=True,
                                     env=dict(os.environ, SF_LIB=os.path.abspath(lib)), timeout=300)
                line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-300:]
                print(json.dumps({"round": r, "lib": name, "result": line}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
