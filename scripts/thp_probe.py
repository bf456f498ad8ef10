"""A/B: pinned staging buffers from hipHostMalloc (default) vs anonymous
memory on transparent huge pages, page-locked with hipHostRegister
(SF_PIN_THP=1).  The knob is read once per process, so each setting runs in
its own child process, alternating: the page-cache copy into the stages
(pread) and the DMA out of them are what changes.  Result
(profiles/r02/e2e/thp_pinned_ab.log): no gain, so the knob was removed from
the library after the run (commit "Remove the THP staging knob"); run as is,
both settings now measure the default.

usage: python scripts/thp_probe.py            (parent: writes inputs, runs children)
       python scripts/thp_probe.py child DIR  (one measurement set)"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)


def child(d):
    import numpy as np
    from syncfast_amd import host
    big = os.path.join(d, "big")
    files8 = sorted(os.path.join(d, "m", f) for f in os.listdir(os.path.join(d, "m")))
    small = sorted(os.path.join(d, "s", f) for f in os.listdir(os.path.join(d, "s")))
    n_big = os.path.getsize(big)
    buf = np.fromfile(big, np.uint8)
    host.index_file(big, 4096)  # warm: stages allocated, pages resident
    host.index_files(files8[:4], 4096)
    out = {}
    for name, fn, nbytes in (
            ("sf_index_file 4 GiB", lambda: host.index_file(big, 4096), n_big),
            ("sf_index_files 512 x 8 MiB", lambda: host.index_files(files8, 4096), 512 << 23),
            ("sf_index_files small", lambda: host.index_files(small, 4096), sum(map(os.path.getsize, small))),
            ("sf_index_buffer staged 4 GiB", lambda: host.index_buffer(buf, 4096), n_big)):
        if name.startswith("sf_index_buffer"):
            set_knob("SF_NO_HOSTREG", 1)
        best = min(_t(fn) for _ in range(3))
        set_knob("SF_NO_HOSTREG", 0)
        out[name] = nbytes / best / 1e9
    print(" | ".join(f"{k}: {v:.2f} GB/s" for k, v in out.items()), flush=True)


def _t(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def main():
    import numpy as np
    with tempfile.TemporaryDirectory(dir=os.environ.get("E2E_DIR", "/tmp")) as d:
        rng = np.random.default_rng(0)
        blob = rng.integers(0, 256, 4 << 30, dtype=np.uint8)
        blob.tofile(os.path.join(d, "big"))
        os.mkdir(os.path.join(d, "m"))
        for i in range(512):
            blob[i << 23:(i + 1) << 23].tofile(os.path.join(d, "m", f"m{i:04d}"))
        os.mkdir(os.path.join(d, "s"))
        off = 0
        for i in range(8000):
            k = int(rng.integers(0, 200 << 10))
            blob[off:off + k].tofile(os.path.join(d, "s", f"s{i:05d}"))
            off += k
        del blob
        for rep in range(2):
            for thp in ("0", "1"):
                env = dict(os.environ, SF_PIN_THP=thp)
                r = subprocess.run([sys.executable, __file__, "child", d], env=env, capture_output=True, text=True,
                                   timeout=300)
                line = (r.stdout.strip().splitlines() or ["<no output>"])[-1]
                print(f"rep {rep} SF_PIN_THP={thp}: {line}" + ("" if r.returncode == 0 else f" rc={r.returncode} "
                                                               f"{r.stderr[-500:]}"), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
    else:
        main()
