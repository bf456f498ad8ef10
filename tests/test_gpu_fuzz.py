"""GPU: seeded randomized cross-entry-point parity against the oracle.

Each case draws a shape (lengths, block size, alignment, file mix) from a
fixed-seed generator and runs it through one C-ABI entry point; every digest,
row and blocks_hash is compared with the oracle on the same bytes
(src/index.rs:621-682 restated).  The draws favour the edges the reference
tests care about in this domain: empty and 1-byte inputs, lengths at SHA-1
padding edges (len % 64 in {55, 56, 63, 0}), block sizes that are not
multiples of 16 or 64, misaligned device pointers, zero-length files inside
batches, ragged last blocks.  Sizes stay small (<= 3 MiB per case) so the
whole file runs in well under a minute."""
import os

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, host

pytestmark = pytest.mark.gpu

BLOCK_SIZES = [1, 3, 16, 55, 56, 63, 64, 65, 100, 1000, 4095, 4096, 4097, 8192, 65536, 100_000]


def _len(rng, bs):
    kind = rng.integers(0, 6)
    if kind == 0:
        return int(rng.integers(0, 3))
    if kind == 1:  # a multiple of the block size, +-1
        return max(0, int(rng.integers(1, 40)) * bs + int(rng.integers(-1, 2)))
    if kind == 2:  # SHA-1 padding edges inside the last block
        return int(rng.integers(0, 30)) * bs + int(rng.choice([55, 56, 63, 64, 119, 120]) % max(bs, 1))
    return int(rng.integers(0, min(3 << 20, 300 * bs + 1)))


def _bs(rng):
    return int(rng.choice(BLOCK_SIZES))


def _dev(data, gpu, shift):
    """data on the device starting `shift` bytes into an allocation."""
    t = torch.empty(data.size + shift, dtype=torch.uint8, device=gpu)
    if data.size:
        t[shift:] = torch.from_numpy(data).to(gpu)
    return t[shift:]


@pytest.mark.parametrize("case", range(160))
def test_fuzz_fixed_device(gpu, case):
    rng = np.random.default_rng(10_000 + case)
    bs = _bs(rng)
    n = _len(rng, bs)
    data = oracle.splitmix_bytes(n, 20_000 + case)
    t = _dev(data, gpu, int(rng.integers(0, 16)))
    got = device.index_device(t, bs).cpu().numpy()
    want = oracle.index_fixed(data, bs)[2]
    assert got.shape == want.shape and np.array_equal(got, want), (n, bs)


@pytest.mark.parametrize("case", range(100))
def test_fuzz_explicit_blocks(gpu, case):
    rng = np.random.default_rng(11_000 + case)
    n = int(rng.integers(0, 2 << 20))
    data = oracle.splitmix_bytes(n, 21_000 + case)
    m = int(rng.integers(0, 300))
    sizes = rng.integers(0, 70_000, m).astype(np.int64)
    sizes = np.minimum(sizes, n)
    offs = np.array([int(rng.integers(0, n - s + 1)) for s in sizes], np.int64)
    t = _dev(data, gpu, int(rng.integers(0, 16)))
    got = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes)), (n, m)


@pytest.mark.parametrize("case", range(100))
def test_fuzz_batch(gpu, case):
    # many files in one buffer: equal and ragged mixes, zero-length files,
    # files at 16-B aligned and unaligned offsets
    rng = np.random.default_rng(12_000 + case)
    bs = _bs(rng)
    nf = int(rng.integers(1, 80))
    if rng.integers(0, 2):
        ln = int(rng.integers(0, 40)) * bs
        lens = [ln] * nf
    else:
        lens = [_len(rng, bs) // 4 for _ in range(nf)]
    align = int(rng.choice([1, 16]))
    files, off = [], 0
    for ln in lens:
        files.append((off, ln))
        off += (ln + align - 1) // align * align
    data = oracle.splitmix_bytes(off, 22_000 + case)
    t = _dev(data, gpu, 0)
    dig, first, fh = device.index_device_batch(t, files, bs)
    dig, fh = dig.cpu().numpy(), fh.cpu().numpy()
    for k, (o, ln) in enumerate(files):
        want = oracle.index_fixed(data[o:o + ln], bs)[2]
        assert np.array_equal(dig[first[k]:first[k + 1]], want), (k, ln, bs)
        assert bytes(fh[k]) == oracle.blocks_hash(want), (k, ln, bs)


@pytest.mark.parametrize("case", range(60))
def test_fuzz_host_routes(gpu, case, tmp_path, knobs):
    # one input through the buffer, file, fd and file-range entry points,
    # with small pipeline stages so stage edges land anywhere
    rng = np.random.default_rng(13_000 + case)
    bs = _bs(rng)
    n = _len(rng, bs)
    knobs.set("SF_TEST_STREAM_STAGE_MIB", int(rng.integers(1, 4)))
    data = oracle.splitmix_bytes(n, 23_000 + case)
    offs, sizes, want = oracle.index_fixed(data, bs)
    bh_want = oracle.blocks_hash(want)

    def same(rows):
        assert rows.shape[0] == want.shape[0], (n, bs)
        if want.shape[0]:
            assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
            assert np.array_equal(rows["sha1"], want)

    same(host.index_buffer(data, bs))
    p = tmp_path / "f"
    data.tofile(p)
    rows, bh = host.index_file(p, bs)
    same(rows)
    assert bh == bh_want
    fd = os.open(p, os.O_RDONLY)
    try:
        rows, bh = host.index_fd(fd, bs)
    finally:
        os.close(fd)
    same(rows)
    assert bh == bh_want
    from syncfast_amd.shard import shard_range
    world = int(rng.integers(1, 5))
    parts = [host.index_file_range(p, *shard_range(n, bs, world, r), bs) for r in range(world)]
    same(np.concatenate(parts))


@pytest.mark.parametrize("case", range(30))
def test_fuzz_index_files(gpu, case, tmp_path):
    rng = np.random.default_rng(14_000 + case)
    bs = _bs(rng)
    nf = int(rng.integers(1, 60))
    paths, datas = [], []
    for i in range(nf):
        d = oracle.splitmix_bytes(_len(rng, bs) // 3, 24_000 + 100 * case + i)
        p = tmp_path / f"f{i}"
        d.tofile(p)
        paths.append(p)
        datas.append(d)
    stage = int(rng.choice([0, 1 << 20, 3 << 20]))
    rows, first, fh = host.index_files(paths, bs, stage_bytes=stage)
    for k, d in enumerate(datas):
        offs, sizes, want = oracle.index_fixed(d, bs)
        r = rows[int(first[k]):int(first[k + 1])]
        assert r.shape[0] == want.shape[0]
        if want.shape[0]:
            assert np.array_equal(r["sha1"], want) and np.array_equal(r["offset"], offs)
        assert bytes(fh[k]) == oracle.blocks_hash(want)


@pytest.mark.parametrize("case", range(40))
def test_fuzz_block_set(gpu, case):
    # destination tables drawn from a small digest pool (many repeats), random
    # present flags; queries from the pool and fresh: vs the first-row oracle
    from syncfast_amd.device import BlockSet
    rng = np.random.default_rng(15_000 + case)
    pool = rng.integers(0, 256, (int(rng.integers(1, 400)), 20), dtype=np.uint8)
    if rng.integers(0, 2):  # pool digests that share slot bits and fingerprint
        pool[:, :11] = pool[0, :11]
    n = int(rng.integers(0, 5000))
    table = pool[rng.integers(0, pool.shape[0], n)] if n else np.zeros((0, 20), np.uint8)
    present = rng.random(n) < rng.random() if rng.integers(0, 2) else None
    q = np.concatenate([pool, rng.integers(0, 256, (int(rng.integers(0, 50)), 20), dtype=np.uint8)])
    t = torch.from_numpy(np.ascontiguousarray(table)).to(gpu)
    pres = torch.from_numpy(present).to(gpu) if present is not None else None
    with BlockSet(t, pres) as bset:
        got = bset.lookup(torch.from_numpy(q).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.block_lookup(table, present, q)), (n, pool.shape[0])


@pytest.mark.parametrize("case", range(60))
def test_fuzz_explicit_list_host_routes(gpu, case, tmp_path, knobs):
    """A host chunker's list over host memory or a file (sf_index_buffer_blocks
    / sf_index_file_blocks): random block-size mixes (1-byte to 40 KiB blocks,
    gaps, overlaps on odd cases, empty blocks), odd buffer starts, random stage
    sizes, in place or staged, against the oracle's rows and blocks_hash."""
    rng = np.random.default_rng(50_000 + case)
    n = int(rng.choice([0, 1, 63, 64, 4097, int(rng.integers(1, 3 << 20))]))
    raw = oracle.splitmix_bytes(n + 16, 60_000 + case)
    shift = int(rng.integers(0, 16))
    data = raw[shift:shift + n]
    mean = float(rng.choice([1.5, 64, 3000, 8192, 20000]))
    sizes, offs, pos = [], [], 0
    while pos < n:
        s = int(min(rng.geometric(1.0 / mean), 40_000, n - pos))
        if case % 2 and rng.random() < 0.1:  # overlap or skip on odd cases
            start = max(0, pos - int(rng.integers(0, 200)))
            s = min(s, n - start)
        else:
            start = pos
        if rng.random() < 0.03:
            s = 0
        offs.append(start)
        sizes.append(s)
        pos = max(pos, start + max(s, 1))
    offs = np.asarray(offs, np.uint64)
    sizes = np.asarray(sizes, np.uint32)
    order = np.argsort(offs, kind="stable")  # non-decreasing offsets, as a chunker gives
    offs, sizes = offs[order], sizes[order]
    knobs.set("SF_TEST_STREAM_STAGE_MIB", int(rng.choice([1, 2, 256])))
    if rng.random() < 0.3:
        knobs.set("SF_NO_HOSTREG", 1)
    want = oracle.index_blocks(data, offs, sizes)
    rows, bh = host.index_buffer_blocks(data, offs, sizes)
    assert np.array_equal(rows["sha1"], want) and bh == oracle.blocks_hash(want), (n, mean)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    if case % 3 == 0:
        p = tmp_path / "f"
        data.tofile(p)
        rows2, bh2 = host.index_file_blocks(p, offs, sizes)
        assert np.array_equal(rows2, rows) and bh2 == bh
