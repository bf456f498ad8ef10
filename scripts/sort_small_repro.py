#!/usr/bin/env python3
"""Debug (round 6): the C consumer's default mode over many files
(tests/test_c_consumer.py::test_c_consumer_default_mode_many_files[4-2])
gave one wrong digest once explicit lists were sorted from 128 blocks.  The
same files and command, repeated with the library's scratch from the
device's default pool (SF_TEST_STREAM_POOL=0, hipMallocAsync) and from its own
pool without cross-stream reuse (1), alternating; per run, the files whose
rows differ from the oracle and their first wrong blocks."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import oracle
    exe = os.path.join(ROOT, "examples", "build", "sf_index")
    rng = np.random.default_rng(4)
    tmp = tempfile.mkdtemp()
    paths, want = [], {}
    for k, n in enumerate([0, 1, 100_000, 32768, 3 << 20, 777, (9 << 20) + 3] +
                          [int(x) for x in rng.integers(0, 300_000, 40)] + [2 << 20]):
        p = os.path.join(tmp, f"f{k:03d}")
        d = oracle.splitmix_bytes(n, 900 + k)
        d.tofile(p)
        paths.append(p)
        sizes = oracle.zpaq_standin_sizes(d) if d.size else np.zeros(0, np.uint32)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) if sizes.size else sizes
        dig = oracle.index_blocks(d, offs, sizes) if sizes.size else np.zeros((0, 20), np.uint8)
        want[p] = [(int(o), int(s), bytes(h).hex()) for o, s, h in zip(offs, sizes, dig)]
    runs = []
    for i in range(int(os.environ.get("ROUNDS", "6"))):
        args = ["-P", "1" if i % 2 else "2", "-K", "2", "-j", "4" if i % 3 else "1"]
        pair = [("pool0", {"SF_TEST_STREAM_POOL": "0"}, args), ("pool1", {"SF_TEST_STREAM_POOL": "1"}, args)]
        runs += pair if i % 2 == 0 else pair[::-1]
    for name, env, args in runs:
        r = subprocess.run([exe, "-Z", "-M", "-S", "1"] + args + paths, capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, **env))
        files, cur = {}, None
        for ln in r.stdout.splitlines():
            f = ln.split()
            if f[0] == "file":
                cur = files.setdefault(f[1], [])
            elif f[0] != "blocks_hash":
                cur.append((int(f[0]), int(f[1]), f[2]))
        bad = {}
        for p in paths:
            g, w = files.get(p, []), want[p]
            if g != w:
                idx = [i for i in range(min(len(g), len(w))) if g[i] != w[i]]
                bad[os.path.basename(p)] = {"n": len(w), "got_n": len(g), "wrong": len(idx), "first": idx[:6]}
        print(json.dumps({"run": name, "args": " ".join(args), "rc": r.returncode, "bad_files": bad}), flush=True)


if __name__ == "__main__":
    main()
