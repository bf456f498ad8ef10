"""sf_index_buffer / sf_index_file rate vs size: exposes the per-call fixed
cost (allocations, stream setup) of the host entry points."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

MiB = 1 << 20
b = np.random.default_rng(0).integers(0, 256, 4096 * MiB, dtype=np.uint8)
host.index_buffer(b[:256 * MiB], 4096)
for mib in (64, 128, 256, 1024, 4096):
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        host.index_buffer(b[:mib * MiB], 4096)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(f"sf_index_buffer {mib:5d} MiB: {t * 1e3:8.2f} ms  {mib * MiB / t / 1e9:6.2f} GB/s", flush=True)
d = os.environ.get("E2E_DIR", "/tmp")
for mib in (64, 256, 1024):
    with tempfile.NamedTemporaryFile(dir=d, delete=False) as f:
        f.write(b[:mib * MiB].tobytes())
        path = f.name
    try:
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            host.index_file(path, 4096)
            ts.append(time.perf_counter() - t0)
    finally:
        os.unlink(path)
    t = min(ts)
    print(f"sf_index_file   {mib:5d} MiB: {t * 1e3:8.2f} ms  {mib * MiB / t / 1e9:6.2f} GB/s", flush=True)
# many files through one sf_index_files call: 8 MiB files, trees of 8..512
with tempfile.TemporaryDirectory(dir=d) as td:
    paths = []
    for i in range(512):
        p = os.path.join(td, f"f{i:04d}")
        with open(p, "wb") as f:
            f.write(b[i * 8 * MiB:(i + 1) * 8 * MiB].tobytes())
        paths.append(p)
    for nf in (8, 32, 128, 512):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            host.index_files(paths[:nf], 4096)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        print(f"sf_index_files {nf:4d} x 8 MiB: {t * 1e3:8.2f} ms  {nf * 8 * MiB / t / 1e9:6.2f} GB/s", flush=True)
