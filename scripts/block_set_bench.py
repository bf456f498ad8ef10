"""Rate of the receiving side's block lookup (sf_block_set_*): config 2's
signature table (2^21 digests of the 8 GiB stream) as the destination index,
looked up with 2^22 digests (half hits in shuffled order, half fresh).  HIP
events around the build and the lookup launches; beside it the same question
asked the reference's way, Index.get_block (one SQL query per FILE_BLOCK) on a
smaller index, and the numpy oracle.

usage: python scripts/block_set_bench.py"""
import os
import sys
import time
from pathlib import PurePath

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from syncfast_amd import device  # noqa: E402
from syncfast_amd.device import BlockSet  # noqa: E402


def events(fn, reps):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    data = device.splitmix_tensor(8 << 30, 0x5EED0000)
    dig = device.index_device(data, 4096)
    del data
    n = dig.shape[0]
    q = torch.cat([dig[torch.randperm(n, device="cuda")], torch.randint(0, 256, (n, 20), dtype=torch.uint8,
                                                                           device="cuda")])
    m = q.shape[0]
    holder = {}

    def build():
        if "s" in holder:
            holder["s"].close()
        holder["s"] = BlockSet(dig)
    t_build = events(build, 10)
    bset = holder["s"]
    out = torch.empty(m, dtype=torch.int64, device="cuda")

    def look():
        out.copy_(bset.lookup(q))
    t_look = events(lambda: bset.lookup(q), 20)
    got = bset.lookup(q).cpu().numpy()
    assert np.array_equal(got, oracle.block_lookup(dig.cpu().numpy(), None, q.cpu().numpy()))
    # algorithmic bytes per lookup: the query (20), the result (8), one slot (8)
    # and, for a hit, one table row (20)
    alg = m * (20 + 8 + 8) + (m // 2) * 20
    print(f"build: {n} rows in {t_build:.3f} ms ({n / t_build / 1e6:.2f} G rows/s)", flush=True)
    print(f"lookup: {m} digests ({m // 2} hits) in {t_look:.3f} ms = {m / t_look / 1e6:.2f} G lookups/s, "
          f"{alg / t_look / 1e6:.1f} GB/s of algorithmic bytes", flush=True)
    # beyond the caches: 2^25 rows (640 MiB of digests, 512 MiB of slots),
    # uniform random digests (SHA-1 output is uniform), 2^25 lookups, half hits
    big_n = 1 << 25
    big = torch.randint(0, 256, (big_n, 20), dtype=torch.uint8, device="cuda")
    bq = torch.cat([big[torch.randint(0, big_n, (big_n // 2,), device="cuda")],
                    torch.randint(0, 256, (big_n // 2, 20), dtype=torch.uint8, device="cuda")])
    hb = {}

    def build_big():
        if "s" in hb:
            hb["s"].close()
        hb["s"] = BlockSet(big)
    tb = events(build_big, 3)
    tl = events(lambda: hb["s"].lookup(bq), 5)
    algb = big_n * (20 + 8 + 8) + (big_n // 2) * 20
    print(f"2^25-row table: build {tb:.2f} ms ({big_n / tb / 1e6:.2f} G rows/s), 2^25 lookups {tl:.2f} ms = "
          f"{big_n / tl / 1e6:.2f} G lookups/s, {algb / tl / 1e6:.1f} GB/s of algorithmic bytes", flush=True)
    gb = hb["s"].lookup(bq)  # property check: hits find their own digest, fresh digests miss
    half = big_n // 2
    assert bool((gb[:half] >= 0).all()) and torch.equal(big[gb[:half]], bq[:half]) and bool((gb[half:] == -1).all())
    hb["s"].close()
    del big, bq
    # numpy oracle (sort-based), the same question on the host cores
    tq = q.cpu().numpy()
    tt = dig.cpu().numpy()
    t0 = time.perf_counter()
    oracle.block_lookup(tt, None, tq)
    t = time.perf_counter() - t0
    print(f"numpy oracle (sort + searchsorted, 1 core): {m / t / 1e6:.3f} M lookups/s", flush=True)
    # the reference's way: one SQL query per FILE_BLOCK (Index.get_block) on a
    # 2^18-row index built from the first rows of the same table
    from syncfast_amd.digest import HashDigest
    from syncfast_amd.index import Index
    from syncfast_amd.timestamp import DateTimeUtc
    k = 1 << 18
    idx = Index.open_in_memory()
    fid, _ = idx.add_file(PurePath("big"), DateTimeUtc.from_ns(0))
    hx = tt[:k].tobytes().hex()
    idx.db.executemany("INSERT INTO blocks(hash, file_id, offset, size, present) VALUES(?, ?, ?, ?, 1);",
                       ((hx[40 * i:40 * i + 40], fid, i * 4096, 4096) for i in range(k)))
    idx.commit()
    sample = [HashDigest(bytes(tt[i])) for i in np.random.default_rng(0).integers(0, k, 20000)]
    t0 = time.perf_counter()
    for h in sample:
        idx.get_block(h)
    t = time.perf_counter() - t0
    print(f"Index.get_block (SQLite, one query per block, 2^18-row index): {len(sample) / t / 1e3:.1f} K lookups/s",
          flush=True)
    bset.close()


if __name__ == "__main__":
    main()
