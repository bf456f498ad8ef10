"""GPU: inputs with more blocks than one launch takes.

HIP caps a launch at 2^32 - 1 work-items; the kernels run one lane per block,
so a table of more than ~2^32 blocks (only reachable with tiny blocks, e.g.
1-B blocks over 4 GiB or 16-B blocks over 64 GiB) is hashed as several
launches over consecutive block ranges (sf_capi.hip, launch_max_blocks).
SF_TEST_LAUNCH_MAX_BLOCKS lowers the piece size so the split runs at small sizes
through every launcher; one test crosses the real limit."""
import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, wire
from syncfast_amd._lib import SfError

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_pieces(knobs):
    knobs.set("SF_TEST_LAUNCH_MAX_BLOCKS", 48)


@pytest.mark.parametrize("n,bs,shift", [(100_000, 64, 0), (77_777, 100, 3), (4096 * 300 + 5, 4096, 0),
                                        (5000, 1, 0), (48 * 4096, 4096, 0), (49 * 4096, 4096, 8)])
def test_fixed_in_pieces(gpu, small_pieces, n, bs, shift):
    data = oracle.splitmix_bytes(n, n + bs)
    t = torch.empty(n + shift, dtype=torch.uint8, device=gpu)
    t[shift:] = torch.from_numpy(data).to(gpu)
    got = device.index_device(t[shift:], bs).cpu().numpy()
    assert np.array_equal(got, oracle.index_fixed(data, bs)[2])


def test_fixed_weak_in_pieces(gpu, small_pieces):
    n, bs = 4096 * 123 + 17, 4096
    data = oracle.splitmix_bytes(n, 5)
    dig, weak = device.index_device_weak(torch.from_numpy(data).to(gpu), bs)
    assert np.array_equal(dig.cpu().numpy(), oracle.index_fixed(data, bs)[2])
    assert np.array_equal(weak.cpu().numpy().view(np.uint32), oracle.adler_fixed(data, bs))


def test_table_in_pieces(gpu, small_pieces):
    rng = np.random.default_rng(3)
    n = 1 << 20
    data = oracle.splitmix_bytes(n, 9)
    sizes = rng.integers(0, 9000, 500).astype(np.int64)
    offs = np.array([int(rng.integers(0, n - s + 1)) for s in sizes], np.int64)
    t = torch.from_numpy(data).to(gpu)
    got = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes))
    # a block out of range in a later piece is still reported
    offs[400] = n
    sizes[400] = 1
    with pytest.raises(SfError):
        device.index_device_blocks(t, torch.from_numpy(offs).to(gpu), torch.from_numpy(sizes.astype(np.int32)).to(gpu))


@pytest.mark.parametrize("ragged", [False, True])
def test_batch_in_pieces(gpu, small_pieces, ragged):
    bs = 4096
    lens = [bs * 40] * 16 if not ragged else [bs * 40 + 3 * i for i in range(16)]
    files, off = [], 0
    for ln in lens:
        files.append((off, ln))
        off += (ln + 15) // 16 * 16
    data = oracle.splitmix_bytes(off, 11)
    dig, first, fh = device.index_device_batch(torch.from_numpy(data).to(gpu), files, bs)
    dig, fh = dig.cpu().numpy(), fh.cpu().numpy()
    for k, (o, ln) in enumerate(files):
        want = oracle.index_fixed(data[o:o + ln], bs)[2]
        assert np.array_equal(dig[first[k]:first[k + 1]], want)
        assert bytes(fh[k]) == oracle.blocks_hash(want)


def test_wire_in_pieces(gpu, small_pieces):
    n, bs = 100 * 1000 + 7, 1000
    data = oracle.splitmix_bytes(n, 13)
    dig = device.index_device(torch.from_numpy(data).to(gpu), bs)
    got = wire.file_blocks_device(dig, bs, n).cpu().numpy().tobytes()
    _, sizes, want_d = oracle.index_fixed(data, bs)
    assert got == b"".join(wire.write_message("FileBlock", bytes(d), int(s)) for d, s in zip(want_d, sizes))


def test_chained_batch_over_the_limit_is_refused(gpu, small_pieces):
    # the batch stream is one launch per batch: a batch over the limit is an
    # argument error, not a silent partial launch
    bs = 4096
    data = torch.zeros(64 * bs, dtype=torch.uint8, device=gpu)
    s = device.BatchStream(1, 64 * bs, bs)
    with pytest.raises(SfError):
        s.push(data, torch.empty((64, 20), dtype=torch.uint8, device=gpu))


def test_more_blocks_than_one_launch_holds(gpu):
    # 1-B blocks over 4 GiB + 77 B: 2^32 + 77 blocks, more work-items than
    # one HIP launch allows; block i's digest is SHA-1 of the single byte i
    n = (1 << 32) + 77
    data = device.splitmix_tensor(n, 0x5EED0000, device=gpu)
    dig = device.index_device(data, 1)
    assert dig.shape == (n, 20)
    table = torch.from_numpy(np.stack([np.frombuffer(oracle.sha1(bytes([b])), np.uint8) for b in range(256)])).to(gpu)
    step = 1 << 28
    for a in range(0, n, step):
        b = min(n, a + step)
        want = table[data[a:b].long()]
        assert torch.equal(dig[a:b], want), a
        del want
