"""sf_index_files over 0-200 KiB files and 8 MiB files with 8/12/16/24 reader
threads (SF_IO_THREADS), files in the page cache."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

rng = np.random.default_rng(1)
blob = rng.integers(0, 256, 1 << 30, dtype=np.uint8).tobytes()
with tempfile.TemporaryDirectory(dir=os.environ.get("E2E_DIR", "/tmp")) as td:
    small, off, i = [], 0, 0
    while off < (1 << 30) - (200 << 10):
        n = int(rng.integers(0, 200 << 10))
        p = os.path.join(td, f"s{i:06d}")
        with open(p, "wb") as f:
            f.write(blob[off:off + n])
        small.append(p)
        off += n
        i += 1
    big = []
    for j in range(128):
        p = os.path.join(td, f"b{j:04d}")
        with open(p, "wb") as f:
            f.write(blob[j * (8 << 20):(j + 1) * (8 << 20)])
        big.append(p)
    for name, paths, nbytes in (("0-200 KiB", small, off), ("8 MiB", big, 1 << 30)):
        host.index_files(paths, 4096)
        for th in ("8", "12", "16", "24", "8", "12", "16", "24"):
            set_knob("SF_IO_THREADS", int(th))
            t0 = time.perf_counter()
            host.index_files(paths, 4096)
            t = time.perf_counter() - t0
            print(f"sf_index_files {len(paths)} files of {name}, {th:>2} threads: {nbytes / t / 1e9:6.2f} GB/s", flush=True)
