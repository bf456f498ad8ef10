"""The receiving side's block lookup (sf_block_set_*, device.BlockSet,
Index.get_blocks): for each incoming digest, the row Index::get_block
(src/index.rs:77-103) returns -- first present row with that hash, rowid
order -- or none.

The oracle (oracle.block_lookup) is pinned on CPU against the reference's
own SQL, run by the Index mirror on randomized indexes with repeated digests,
missing blocks and temporary files; the GPU tests compare the device lookup
with the oracle and with Index.get_block."""
from pathlib import PurePath

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd.digest import HashDigest
from syncfast_amd.index import Index
from syncfast_amd.timestamp import DateTimeUtc


def _random_index(seed, n_files=6, per_file=40):
    """An in-memory index: files (one temporary) with blocks drawn from a small
    pool of digests (so digests repeat within and across files), some rows
    recorded as missing (present = 0)."""
    rng = np.random.default_rng(seed)
    pool = [HashDigest(rng.integers(0, 256, 20, dtype=np.uint8).tobytes()) for _ in range(60)]
    idx = Index.open_in_memory()
    for f in range(n_files):
        if f == n_files - 1:
            fid = idx.add_temp_file(PurePath(f"dir/t{f}"))
        else:
            fid, _ = idx.add_file(PurePath(f"dir/f{f}"), DateTimeUtc.from_ns(f))
        for b in range(per_file):
            h = pool[int(rng.integers(0, len(pool)))]
            if rng.random() < 0.3:
                idx.add_missing_block(h, fid, b * 4096, 4096)
            else:
                idx.add_block(h, fid, b * 4096, 4096)
    idx.commit()
    return idx, pool


def _rows(idx):
    rows = idx.db.execute("SELECT blocks.hash, blocks.present = 1 AND files.file_id IS NOT NULL, files.name, "
                          "blocks.offset, blocks.size FROM blocks LEFT JOIN files ON blocks.file_id = files.file_id "
                          "ORDER BY blocks.rowid;").fetchall()
    table = np.frombuffer(bytes.fromhex("".join(r[0] for r in rows)), np.uint8).reshape(-1, 20)
    present = np.array([bool(r[1]) for r in rows])
    return rows, table, present


@pytest.mark.parametrize("seed", range(8))
def test_oracle_is_get_block(seed):
    # the reference's SQL (Index.get_block) and the oracle agree on every
    # digest of the pool and on digests absent from the index
    idx, pool = _random_index(seed)
    rows, table, present = _rows(idx)
    extra = [HashDigest(bytes([seed] * 20))]
    q = pool + extra
    got = oracle.block_lookup(table, present, np.frombuffer(b"".join(h.bytes for h in q), np.uint8).reshape(-1, 20))
    for h, r in zip(q, got):
        want = idx.get_block(h)
        assert (None if r < 0 else (PurePath(rows[r][2]), int(rows[r][3]), int(rows[r][4]))) == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_index_get_blocks_on_device_is_get_block(gpu, seed):
    idx, pool = _random_index(100 + seed, n_files=12, per_file=300)
    q = pool + [HashDigest(bytes([7] * 20))] + pool[::-1]
    assert idx.get_blocks(q, device=gpu) == [idx.get_block(h) for h in q]


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,dup,with_present", [(0, 10, 0, False), (1, 5, 0, True), (1000, 3000, 50, True),
                                                   (100_000, 200_000, 5000, True), (100_000, 50_000, 0, False)])
def test_block_set_matches_oracle(gpu, n, m, dup, with_present):
    from syncfast_amd.device import BlockSet
    rng = np.random.default_rng(n + m)
    table = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    if dup and n:  # repeated digests at random later rows
        src = rng.integers(0, n, dup)
        dst = rng.integers(0, n, dup)
        table[dst] = table[src]
    present = rng.random(n) < 0.7 if with_present else None
    # queries: rows of the table (hits, or misses when not present), fresh digests
    picks = table[rng.integers(0, max(n, 1), m // 2)] if n else np.zeros((0, 20), np.uint8)
    fresh = rng.integers(0, 256, (m - picks.shape[0], 20), dtype=np.uint8)
    queries = np.concatenate([picks, fresh])
    rng.shuffle(queries)
    t = torch.from_numpy(table).to(gpu)
    with BlockSet(t, torch.from_numpy(present).to(gpu) if present is not None else None) as bset:
        got = bset.lookup(torch.from_numpy(queries).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.block_lookup(table, present, queries))


@pytest.mark.gpu
def test_block_set_colliding_slots(gpu):
    # digests that share their slot bits (bytes 0-7) and fingerprint (8-10)
    # but differ later: the probe must compare whole digests
    from syncfast_amd.device import BlockSet
    base = np.zeros((64, 20), np.uint8)
    base[:, 19] = np.arange(64)  # same first 19 bytes, different last byte
    table = np.concatenate([base, base[::2]])  # repeats: the first row wins
    present = np.ones(table.shape[0], bool)
    present[:8] = False  # the first copies of rows 0..7 are missing: rows 0,2,4,6 resolve to the repeats
    q = np.concatenate([base, np.full((1, 20), 255, np.uint8)])
    t = torch.from_numpy(table).to(gpu)
    with BlockSet(t, torch.from_numpy(present).to(gpu)) as bset:
        got = bset.lookup(torch.from_numpy(q).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.block_lookup(table, present, q))
    assert got[0] == 64 and got[1] == -1 and got[8] == 8 and got[-1] == -1


@pytest.mark.gpu
def test_block_set_config2_table(gpu):
    # config 2's whole signature table (2^21 digests of the 8 GiB stream) as a
    # destination index, looked up with the same table shuffled plus as many
    # fresh digests: every answer vs the oracle
    from syncfast_amd import device
    from syncfast_amd.device import BlockSet
    data = device.splitmix_tensor(8 << 30, 0x5EED0000, device=gpu)
    dig = device.index_device(data, 4096)
    del data
    n = dig.shape[0]
    perm = torch.randperm(n, device=gpu)
    fresh = torch.randint(0, 256, (n, 20), dtype=torch.uint8, device=gpu)
    q = torch.cat([dig[perm], fresh])
    with BlockSet(dig) as bset:
        got = bset.lookup(q)
    torch.cuda.synchronize()
    g = got.cpu().numpy()
    assert np.array_equal(g[:n], perm.cpu().numpy())  # the splitmix blocks are all distinct
    assert np.array_equal(g, oracle.block_lookup(dig.cpu().numpy(), None, q.cpu().numpy()))
