"""sf_index_buffer / sf_index_file per call at 1-32 MiB: staged (pread /
memcpy into pinned stages) vs in place (page-locked), SF_INPLACE_MIN_MIB."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

MiB = 1 << 20
b = np.random.default_rng(0).integers(0, 256, 64 * MiB, dtype=np.uint8)
host.index_buffer(b, 4096)
d = os.environ.get("E2E_DIR", "/tmp")
with tempfile.NamedTemporaryFile(dir=d, delete=False) as f:
    f.write(b.tobytes())
    path = f.name
try:
    for mib in (1, 4, 8, 32):
        paths = []
        for k in range(16):
            p = f"{path}.{mib}.{k}"
            with open(p, "wb") as f:
                f.write(b[k * MiB:k * MiB + mib * MiB].tobytes() if k + mib <= 64 else b[:mib * MiB].tobytes())
            paths.append(p)
        for knob in ("1024", "0", "1024", "0"):
            set_knob("SF_INPLACE_MIN_MIB", int(knob))
            name = "staged " if knob != "0" else "in place"
            t0 = time.perf_counter()
            for k in range(16):
                host.index_buffer(b[k * MiB:k * MiB + mib * MiB] if k + mib <= 64 else b[:mib * MiB], 4096)
            tb = (time.perf_counter() - t0) / 16
            t0 = time.perf_counter()
            for p in paths:
                host.index_file(p, 4096)
            tf = (time.perf_counter() - t0) / 16
            print(f"{mib:3d} MiB {name}: index_buffer {tb * 1e3:7.3f} ms ({mib * MiB / tb / 1e9:5.1f} GB/s)  "
                  f"index_file {tf * 1e3:7.3f} ms ({mib * MiB / tf / 1e9:5.1f} GB/s)", flush=True)
        for p in paths:
            os.unlink(p)
finally:
    os.unlink(path)
