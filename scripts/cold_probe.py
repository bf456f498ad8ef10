"""sf_index_file on a file that is NOT in the page cache: write, fsync,
posix_fadvise(DONTNEED) (drops the file's clean pages without root), check
residency with mincore via a mapping, then index it (pread route).  Also
the same file warm (page cache) for comparison."""
import mmap
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)
import numpy as np  # noqa: E402

from syncfast_amd import host  # noqa: E402

GiB = 1 << 30


def resident_frac(path):
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    n = os.path.getsize(path)
    with open(path, "rb") as f:
        m = mmap.mmap(f.fileno(), n, prot=mmap.PROT_READ)
        pg = mmap.PAGESIZE
        vec = (ctypes.c_ubyte * ((n + pg - 1) // pg))()
        # mincore needs the mapping address: use numpy's view of the mmap
        arr = np.frombuffer(m, dtype=np.uint8)
        rc = libc.mincore(ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(n), vec)
        frac = (np.frombuffer(vec, np.uint8) & 1).mean() if rc == 0 else -1.0
        del arr
        m.close()
    return frac


def main():
    n = int(float(os.environ.get("COLD_GIB", "4")) * GiB)
    d = os.environ.get("E2E_DIR", "/tmp")
    data = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
    with tempfile.NamedTemporaryFile(dir=d, delete=False) as f:
        f.write(data.tobytes())
        f.flush()
        os.fsync(f.fileno())
        path = f.name
    del data
    try:
        # A/B interleaved: SF_FADVISE=1 (default: sequential + WILLNEED of the
        # next stage) vs 0 (plain pread)
        for rep in range(2):
          for adv in ("1", "0"):
            set_knob("SF_FADVISE", int(adv))
            fd = os.open(path, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.close(fd)
            fr = resident_frac(path)
            t0 = time.perf_counter()
            rows, bh = host.index_file(path, 4096)
            t = time.perf_counter() - t0
            print(f"sf_index_file {n / GiB:.0f} GiB cold (resident before: {fr:.3f}), SF_FADVISE={adv}, "
                  f"incl. blocks_hash: {n / t / 1e9:.2f} GB/s", flush=True)
            t0 = time.perf_counter()
            host.index_file(path, 4096)
            t = time.perf_counter() - t0
            print(f"sf_index_file {n / GiB:.0f} GiB warm (resident: {resident_frac(path):.3f}): {n / t / 1e9:.2f} GB/s",
                  flush=True)
        print("filesystem:", os.popen(f"df -T {d} | tail -1").read().strip(), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
