"""A/B of two builds of the library on the host pipelines (round 5: helper
threads kept between stages vs started per stage).  The kernels are the
same; what differs is the host side, so the routes timed are the file ones,
files in the page cache:
  files8m  sf_index_files over 256 x 8 MiB (fixed 4 KiB blocks)
  small    sf_index_files over ~4,000 files of 0-200 KiB
  file     sf_index_file over one 2 GiB file
  fds      sf_index_fds_blocks over the small tree, CDC-like lists
Each library runs in its own process (SF_LIB), interleaved, REPS rounds.

usage: python scripts/pool_ab.py NAME=LIB[,KNOB=VALUE...] [NAME=LIB ...]
       (round 6: the same library with SF_BATCH_FUSED=1 / 0, the fused
       many-file launch against blocks-then-chains inside sf_index_files)
       python scripts/pool_ab.py --child DIR   (one library, one JSON line)"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def write_tree(d):
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    out = {"files8m": [], "small": [], "file": []}
    for k in range(256):
        p = os.path.join(d, f"m{k:04d}")
        a = int(rng.integers(0, src.size - (8 << 20)))
        src[a:a + (8 << 20)].tofile(p)
        out["files8m"].append(p)
    tot = 0
    while tot < (400 << 20):
        n = int(rng.integers(0, 200 << 10))
        p = os.path.join(d, f"s{len(out['small']):05d}")
        a = int(rng.integers(0, src.size - n))
        src[a:a + n].tofile(p)
        out["small"].append(p)
        tot += n
    p = os.path.join(d, "big")
    with open(p, "wb") as f:
        for _ in range(32):
            f.write(src.tobytes())
    out["file"] = [p]
    return out


def cdc_like(n, seed):
    rng = np.random.default_rng(seed)
    sizes = []
    while sum(sizes) < n:
        sizes.append(int(min(32768, 2048 + rng.exponential(6000))))
    over = sum(sizes) - n
    sizes[-1] -= over
    if sizes[-1] <= 0:
        sizes.pop()
    offs = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64) if sizes else np.zeros(0, np.uint64)
    return offs, np.asarray(sizes, np.uint32)


def child(d):
    sys.path.insert(0, ROOT)
    from syncfast_amd import host
    tree = json.load(open(os.path.join(d, "tree.json")))
    lists = [cdc_like(os.path.getsize(p), k) for k, p in enumerate(tree["small"])]
    res = {}

    def timed(name, nbytes, fn, reps=3):
        fn()  # warm: stage buffers, first launches
        best = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            best.append(time.perf_counter() - t0)
        res[name] = round(nbytes / min(best) / 1e9, 3)

    size = lambda ps: sum(os.path.getsize(p) for p in ps)  # noqa: E731
    timed("files8m", size(tree["files8m"]), lambda: host.index_files(tree["files8m"], 4096))
    timed("small", size(tree["small"]), lambda: host.index_files(tree["small"], 4096))
    timed("file", size(tree["file"]), lambda: host.index_file(tree["file"][0], 4096))

    def fds():
        fs = [open(p, "rb") for p in tree["small"]]
        try:
            host.index_fds_blocks([f.fileno() for f in fs], lists)
        finally:
            for f in fs:
                f.close()
    timed("fds", size(tree["small"]), fds)
    print(json.dumps(res), flush=True)


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    libs = [a.split("=", 1) for a in sys.argv[1:]]
    reps = int(os.environ.get("REPS", "3"))
    d = tempfile.mkdtemp(prefix="sf_poolab_")
    try:
        json.dump(write_tree(d), open(os.path.join(d, "tree.json"), "w"))
        for r in range(reps):
            order = libs[r % len(libs):] + libs[:r % len(libs)]
            for name, spec in order:
                lib, *kv = spec.split(",")
                env = dict(os.environ, SF_LIB=os.path.abspath(lib), **dict(x.split("=", 1) for x in kv))
                out = subprocess.run([sys.executable, __file__, "--child", d], capture_output=True, text=True,
                                     env=env, timeout=300)
                line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-300:]
                print(json.dumps({"round": r, "lib": name, "GB/s": line}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
