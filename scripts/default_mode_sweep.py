"""Sweep of the default-mode many-file route (examples/build/sf_index -Z -M):
chunker threads x the library's reader threads (SF_IO_THREADS) x batch size,
on config 3's shape (1024 x 8 MiB) and a 0-200 KiB tree, files in the page
cache.  One line per run: tree, -j, SF_IO_THREADS, -S, wall, hash call, wait.

usage: python scripts/default_mode_sweep.py [j,j,...] [io,io,...] [S,S,...] [reps]
FORMS=base,base+G64,...: forms interleaved within each setting; +G64 passes
-G 64 (stages of 64 MiB inside each sf_index_fds_blocks call), +S64 -S 64
(64 MiB batches, after the S of the setting); FORM@DIR runs
the consumer against DIR/libsyncfast_amd.so (LD_LIBRARY_PATH before its
RUNPATH).  (Round 5 also measured a batch plan that ramped the first and
last batches down, with no gain: removed)
(round 5 also swept a read-once form, every file read once into pinned
batch buffers and hashed from there: slower, removed)"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
EXE = os.path.join(ROOT, "examples", "build", "sf_index")


def write_tree(d, lens, seed):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    paths = []
    for k, n in enumerate(lens):
        p = os.path.join(d, f"f{k:05d}")
        a = int(rng.integers(0, src.size - n)) if n < src.size else 0
        src[a:a + n].tofile(p)
        paths.append(p)
    return paths


def main():
    js = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,12,16").split(",")]
    ios = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,8,16").split(",")]
    ss = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "256").split(",")]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    forms = os.environ.get("FORMS", "base").split(",")
    rng = np.random.default_rng(3)
    small, tot = [], 0
    while tot < (1 << 30):
        small.append(int(rng.integers(0, 200 << 10)))
        tot += small[-1]
    for name, lens in (("c3_1024x8MiB", [8 << 20] * 1024), ("small_0_200KiB", small)):
        d = tempfile.mkdtemp(prefix="sf_sw_")
        try:
            paths = write_tree(d, lens, 5)
            for S, io, j, form, rep in [(S, io, j, f, r) for S in ss for io in ios for j in js
                                        for r in range(reps) for f in forms]:
                env = dict(os.environ, SF_IO_THREADS=str(io))
                if "@" in form:
                    env["LD_LIBRARY_PATH"] = os.path.abspath(form.split("@", 1)[1])
                if os.environ.get("TRACE") == "1":
                    env["SF_TRACE"] = "1"
                plan = form.split("@")[0].split("+")  # "base+G64": 64 MiB stages per call; "+S64": 64 MiB batches
                flags = [a for g in plan[1:] for a in (("-S" if g[0] == "S" else "-G"), g[1:])]
                r = subprocess.run([EXE, "-Z", "-M", "-q", "-T", "-P", "2", "-j", str(j), "-S", str(S)] + flags + paths,
                                   capture_output=True, text=True, env=env, timeout=300)
                if r.returncode:
                    print(json.dumps({"tree": name, "error": r.stderr[-300:]}), flush=True)
                    return 1
                t = [json.loads(ln) for ln in r.stderr.splitlines() if ln.startswith("{")][-1]
                print(json.dumps({"tree": name, "form": form, "rep": rep, "j": j, "io": io, "S": S,
                                  "batches": t["batches"],
                                  "GB/s": round(t["bytes"] / t["wall_s"] / 1e9, 3),
                                  "wall": round(t["wall_s"], 3), "hash": round(t["hash_call_s"], 3),
                                  "wait": round(t["wait_cut_s"], 3), "chunk_cpu": round(t["chunk_cpu_s"], 2),
                                  "open": round(t["open_s"], 2), "read": round(t["read_s"], 2)}),
                      flush=True)
                if os.environ.get("TRACE") == "1":
                    tr = [ln for ln in r.stderr.splitlines() if "trace:" in ln]
                    for ln in tr[:3] + tr[-2:]:
                        print("   ", ln, flush=True)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
