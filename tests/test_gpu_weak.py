"""GPU: the opt-in weak sum (zlib Adler-32 per block) fused into the SHA-1
pass, through the C-ABI (sf_index_device_fixed_weak / _blocks_weak).

Not a reference path: syncfast computes no weak sum;
north_star names one.  Checked against the C oracle (itself checked against
zlib.adler32 in test_oracle.py) and, for small cases, zlib directly; the
SHA-1 digests of the weak build must equal the plain build's."""
import zlib

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import SfError, device

pytestmark = pytest.mark.gpu


def to_dev(b, dev):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) if len(b) else torch.empty(0, dtype=torch.uint8, device=dev)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("bs", [1, 16, 63, 64, 65, 100, 4096, 4097, 65536, 1 << 20])
def test_fixed_weak_random_lengths(gpu, bs):
    rng = np.random.default_rng(bs + 5)
    for _ in range(3):
        nblk = int(rng.integers(1, 200)) if bs < 65536 else int(rng.integers(1, 30))
        n = max(0, nblk * bs + int(rng.integers(-bs + 1, bs)))
        data = oracle.splitmix_bytes(n, int(rng.integers(0, 1 << 62)))
        t = to_dev(data.tobytes(), gpu)
        d, w = device.index_device_weak(t, bs)
        _, _, want = oracle.index_fixed(data, bs)
        assert np.array_equal(d.cpu().numpy(), want), (bs, n)
        assert np.array_equal(u32(w), oracle.adler_fixed(data, bs)), (bs, n)
        assert torch.equal(d, device.index_device(t, bs))


def test_fixed_weak_small_vs_zlib(gpu):
    data = oracle.splitmix_bytes(4096 * 5 + 77, 3).tobytes()
    _, w = device.index_device_weak(to_dev(data, gpu), 4096)
    assert u32(w).tolist() == [zlib.adler32(data[i:i + 4096]) for i in range(0, len(data), 4096)]


@pytest.mark.parametrize("bs", [4096, 65536, 32 << 20])
def test_weak_worst_case_bytes(gpu, bs):
    # all-0xFF blocks give the largest A/B sums: partial-reduction overflow guard
    n = max(3 * bs, 8 << 20) + 5
    t = torch.full((n,), 255, dtype=torch.uint8, device=gpu)
    _, w = device.index_device_weak(t, bs)
    host = t.cpu().numpy()
    assert np.array_equal(u32(w), oracle.adler_fixed(host, bs))


@pytest.mark.parametrize("shift", [1, 3, 8, 15])
def test_weak_misaligned_pointer(gpu, shift):
    n = 4096 * 70 + 333
    raw = oracle.splitmix_bytes(n + shift, 9)
    t = to_dev(raw.tobytes(), gpu)[shift:]
    d, w = device.index_device_weak(t, 4096)
    data = raw[shift:]
    assert np.array_equal(d.cpu().numpy(), oracle.index_fixed(data, 4096)[2])
    assert np.array_equal(u32(w), oracle.adler_fixed(data, 4096))


def test_blocks_weak_ragged_and_range(gpu):
    rng = np.random.default_rng(21)
    n = 600_000
    data = oracle.splitmix_bytes(n, 12)
    t = to_dev(data.tobytes(), gpu)
    sizes = rng.integers(0, 70_000, 300)
    offs = np.array([int(rng.integers(0, n - s)) for s in sizes], np.int64)
    offs[::4] = offs[::4] // 16 * 16
    d, w = device.index_device_blocks_weak(t, torch.from_numpy(offs).to(gpu),
                                           torch.from_numpy(sizes.astype(np.int32)).to(gpu))
    assert np.array_equal(d.cpu().numpy(), oracle.index_blocks(data, offs, sizes))
    assert np.array_equal(u32(w), oracle.adler_blocks(data, offs, sizes))
    bad_o = torch.tensor([0, n - 10], dtype=torch.int64, device=gpu)
    bad_s = torch.tensor([10, 11], dtype=torch.int32, device=gpu)
    with pytest.raises(SfError):
        device.index_device_blocks_weak(t, bad_o, bad_s)
    d2, w2 = device.index_device_blocks_weak(t, bad_o, bad_s, check_range=False)
    assert u32(w2).tolist() == [zlib.adler32(data[:10].tobytes()), 0]
    assert bytes(d2.cpu().numpy()[1]) == bytes(20)


def test_weak_empty(gpu):
    d, w = device.index_device_weak(torch.empty(0, dtype=torch.uint8, device=gpu), 4096)
    assert d.shape == (0, 20) and w.numel() == 0
