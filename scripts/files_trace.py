"""Where sf_index_files spends its time: the many-small-files tree and the
config-3 shape (8 MiB files) from the page cache, each call run with
SF_TRACE=1 (per-phase times on stderr: stat, read, issue = H2D + batch launch
+ D2H enqueue incl. the ragged block table, wait, harvest = rows +
blocks_hash on the host).

usage: python scripts/files_trace.py   (E2E_GIB, default 2; E2E_DIR, default /tmp)"""
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

GiB = 1 << 30


def tree(root, data, sizes):
    paths, off = [], 0
    for i, k in enumerate(sizes):
        p = os.path.join(root, f"f{i:06d}")
        with open(p, "wb") as f:
            f.write(data[off:off + k].tobytes())
        paths.append(p)
        off += k
    return paths, off


def main():
    n = int(float(os.environ.get("E2E_GIB", "2")) * GiB)
    data = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
    rng = np.random.default_rng(1)
    small, left = [], n
    while left > 200 << 10:
        k = int(rng.integers(0, 200 << 10))
        small.append(k)
        left -= k
    cases = [("0-200 KiB files", small), ("8 MiB files", [8 << 20] * (n // (8 << 20)))]
    set_knob("SF_TRACE", 1)
    for name, sizes in cases:
        root = tempfile.mkdtemp(dir=os.environ.get("E2E_DIR", "/tmp"))
        try:
            paths, total = tree(root, data, sizes)
            host.index_files(paths[:8], 4096)  # warm up
            for rep in range(3):
                t0 = time.perf_counter()
                host.index_files(paths, 4096)
                t = time.perf_counter() - t0
                print(f"{len(paths)} {name} ({total / GiB:.2f} GiB) rep {rep}: {t * 1e3:.1f} ms, "
                      f"{total / t / 1e9:.2f} GB/s", flush=True)
        finally:
            shutil.rmtree(root)


if __name__ == "__main__":
    main()
