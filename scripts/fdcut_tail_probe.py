#!/usr/bin/env python3
"""Where configs[0]'s fused default-mode call spends its device tail: one
process, a 64 MiB random file in the page cache, sf_index_fd_cut with the
stand-in chunker on 16 threads, 8 calls (SF_TRACE=1 prints each call's
cut+join and total), meant to run under `rocprofv3 --kernel-trace --stats`
so the sort and sha1_table_kernel durations of each call's one launch can
be set against the call's time after its cut.  Prints one JSON line per call."""
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    import numpy as np
    L = ctypes.CDLL(os.path.join(ROOT, "syncfast_amd", "lib", "libsyncfast_amd.so"))
    Z = ctypes.CDLL(os.path.join(ROOT, "examples", "build", "libzpaq_standin.so"))
    Z.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    Z.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    ops = Z.sf_zpaq_standin_ops(13, 32768)
    vp = ctypes.c_void_p
    L.sf_index_fd_cut.argtypes = [ctypes.c_int, vp, vp, ctypes.c_uint32, vp, vp, vp]
    L.sf_free_rows.argtypes = [vp]
    d = tempfile.mkdtemp(prefix="sf_tail_")
    p = os.path.join(d, "f64")
    np.random.default_rng(5).integers(0, 256, 64 << 20, dtype=np.uint8).tofile(p)
    fd = os.open(p, os.O_RDONLY)
    try:
        for i in range(int(os.environ.get("CALLS", "8"))):
            rows, n, bh = vp(), ctypes.c_uint64(), (ctypes.c_uint8 * 20)()
            t0 = time.perf_counter()
            rc = L.sf_index_fd_cut(fd, None, ops, 16, ctypes.byref(rows), ctypes.byref(n), bh)
            dt = time.perf_counter() - t0
            assert rc == 0, rc
            L.sf_free_rows(rows)
            print(json.dumps({"call": i, "ms": round(dt * 1e3, 3), "blocks": n.value,
                              "GB/s": round((64 << 20) / dt / 1e9, 2)}), flush=True)
            time.sleep(0.05)
    finally:
        os.close(fd)
        os.unlink(p)
        os.rmdir(d)


if __name__ == "__main__":
    sys.exit(main())
