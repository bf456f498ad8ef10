"""sf_index_files over 16 and 32 MiB files (page cache): pread stages vs
files DMA'd from their page-locked mappings (SF_MAP_MIN_MIB)."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

MiB = 1 << 20
blob = np.random.default_rng(2).integers(0, 256, 2048 * MiB, dtype=np.uint8).tobytes()
with tempfile.TemporaryDirectory(dir=os.environ.get("E2E_DIR", "/tmp")) as td:
    for fm in tuple(int(x) for x in os.environ.get("MAP_FILE_MIB", "16,32").split(",")):
        paths = []
        for j in range(2048 // fm):
            p = os.path.join(td, f"f{fm}_{j:04d}")
            with open(p, "wb") as f:
                f.write(blob[j * fm * MiB:(j + 1) * fm * MiB])
            paths.append(p)
        host.index_files(paths, 4096)
        for knob in (os.environ.get("MAP_HI", "64"), os.environ.get("MAP_LO", "8")) * 2:
            os.environ["SF_MAP_MIN_MIB"] = knob
            t0 = time.perf_counter()
            host.index_files(paths, 4096)
            t = time.perf_counter() - t0
            route = "pread " if int(knob) > fm else "mapped"
            print(f"sf_index_files {len(paths)} x {fm} MiB, {route}: {2048 * MiB / t / 1e9:6.2f} GB/s", flush=True)
