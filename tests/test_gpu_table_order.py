"""GPU: explicit block lists hashed in order of length (sha1_table_kernel's
`order`, launch_table's rocprim sort).

The launcher sorts a list of more than 64 blocks (two waves or more; until
round 6 from 2^17) by compression count, largest first, so each wave's 64 blocks are
about the same length; every digest must
still land at its block's own index, bit-identical to the oracle
(src/index.rs:621-647 restated) and to the list-order launch.
SF_TEST_TABLE_SORT=1 forces the sorted launch on small lists, SF_TEST_TABLE_SORT=0 the
list order."""
import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device
from syncfast_amd._lib import SfError

pytestmark = pytest.mark.gpu


def _dev(data, gpu, shift=0):
    t = torch.empty(data.size + shift, dtype=torch.uint8, device=gpu)
    if data.size:
        t[shift:] = torch.from_numpy(data).to(gpu)
    return t[shift:]


def _cdc_like(rng, n, mean=8192, cap=32768):
    """Content-defined-like boundaries: geometric sizes (mean 8 KiB), capped
    at 32 KiB (ZPAQ 13 bits + max_size, src/index.rs:40-41), tiling [0, n)."""
    sizes = np.minimum(cap, np.maximum(1, rng.geometric(1 / mean, size=n // 64 + 16))).astype(np.int64)
    ends = np.cumsum(sizes)
    k = int(np.searchsorted(ends, n))
    sizes = sizes[:k + 1]
    sizes[-1] = n - (int(ends[k - 1]) if k else 0)
    sizes = sizes[sizes > 0]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    return offs, sizes


@pytest.mark.parametrize("case", range(60))
def test_sorted_explicit_blocks_fuzz(gpu, case, knobs):
    # random, overlapping, unsorted, empty and tiny-to-70 KB blocks, any
    # alignment of the data pointer: forced sort, then list order
    rng = np.random.default_rng(31_000 + case)
    n = int(rng.integers(0, 2 << 20))
    data = oracle.splitmix_bytes(n, 41_000 + case)
    m = int(rng.integers(0, 700))
    sizes = np.minimum(rng.integers(0, 70_000, m).astype(np.int64), n)
    offs = np.array([int(rng.integers(0, n - s + 1)) for s in sizes], np.int64)
    t = _dev(data, gpu, int(rng.integers(0, 16)))
    to, tz = torch.from_numpy(offs).to(gpu), torch.from_numpy(sizes.astype(np.int32)).to(gpu)
    want = oracle.index_blocks(data, offs, sizes)
    for mode in ("1", "0"):
        knobs.set("SF_TEST_TABLE_SORT", int(mode))
        got = device.index_device_blocks(t, to, tz).cpu().numpy()
        assert np.array_equal(got, want), (mode, n, m)


@pytest.mark.parametrize("case", range(12))
def test_sorted_cdc_like_lists(gpu, case, knobs):
    rng = np.random.default_rng(32_000 + case)
    n = int(rng.integers(1, 24 << 20))
    data = oracle.splitmix_bytes(n, 42_000 + case)
    offs, sizes = _cdc_like(rng, n)
    assert offs[-1] + sizes[-1] == n
    t = _dev(data, gpu, int(rng.integers(0, 16)))
    knobs.set("SF_TEST_TABLE_SORT", 1)
    got = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes)), (n, offs.size)


def test_sorted_out_of_range_blocks(gpu, knobs):
    # blocks outside the buffer sort like any other (by their claimed size)
    # and still report SF_ERANGE with a zero digest at their own index
    knobs.set("SF_TEST_TABLE_SORT", 1)
    rng = np.random.default_rng(33_000)
    n = 1 << 20
    data = oracle.splitmix_bytes(n, 43_000)
    offs, sizes = _cdc_like(rng, n)
    bad = rng.choice(offs.size, 5, replace=False)
    offs2, sizes2 = offs.copy(), sizes.copy()
    offs2[bad[:3]] = n + 1
    sizes2[bad[3:]] = n + 100
    t = _dev(data, gpu)
    to, tz = torch.from_numpy(offs2).to(gpu), torch.from_numpy(sizes2.astype(np.int32)).to(gpu)
    with pytest.raises(SfError):
        device.index_device_blocks(t, to, tz)
    got = device.index_device_blocks(t, to, tz, check_range=False).cpu().numpy()
    good = np.setdiff1d(np.arange(offs.size), bad)
    want = oracle.index_blocks(data, offs[good], sizes[good])
    assert np.array_equal(got[good], want)
    assert not got[bad].any()


@pytest.mark.parametrize("case", range(6))
def test_sorted_weak_blocks(gpu, case, knobs):
    knobs.set("SF_TEST_TABLE_SORT", 1)
    rng = np.random.default_rng(34_000 + case)
    n = int(rng.integers(1, 6 << 20))
    data = oracle.splitmix_bytes(n, 44_000 + case)
    offs, sizes = _cdc_like(rng, n, mean=4096)
    t = _dev(data, gpu, int(rng.integers(0, 16)))
    dig, weak = device.index_device_blocks_weak(t, torch.from_numpy(offs).to(gpu),
                                                torch.from_numpy(sizes.astype(np.int32)).to(gpu))
    assert np.array_equal(dig.cpu().numpy(), oracle.index_blocks(data, offs, sizes))
    assert np.array_equal(weak.cpu().numpy().view(np.uint32), oracle.adler_blocks(data, offs, sizes))


@pytest.mark.parametrize("case", range(20))
def test_sorted_ragged_batch(gpu, case, knobs):
    # ragged many-file batches: the block table and the per-file blocks_hash
    # table (one lane per file over runs of different lengths) both sorted
    knobs.set("SF_TEST_TABLE_SORT", 1)
    rng = np.random.default_rng(35_000 + case)
    bs = int(rng.choice([64, 100, 4096, 4097, 65536]))
    nf = int(rng.integers(1, 200))
    lens = [int(rng.integers(0, 40 * bs)) for _ in range(nf)]
    align = int(rng.choice([1, 16]))
    files, off = [], 0
    for ln in lens:
        files.append((off, ln))
        off += (ln + align - 1) // align * align
    data = oracle.splitmix_bytes(off, 45_000 + case)
    dig, first, fh = device.index_device_batch(_dev(data, gpu), files, bs)
    dig, fh = dig.cpu().numpy(), fh.cpu().numpy()
    for k, (o, ln) in enumerate(files):
        want = oracle.index_fixed(data[o:o + ln], bs)[2]
        assert np.array_equal(dig[first[k]:first[k + 1]], want), (k, ln, bs)
        assert bytes(fh[k]) == oracle.blocks_hash(want), (k, ln, bs)


def test_sorted_with_launch_split(gpu, knobs):
    # a list larger than one launch: each piece sorted on its own
    knobs.set("SF_TEST_TABLE_SORT", 1)
    knobs.set("SF_TEST_LAUNCH_MAX_BLOCKS", 48)
    rng = np.random.default_rng(36_000)
    n = 3 << 20
    data = oracle.splitmix_bytes(n, 46_000)
    offs, sizes = _cdc_like(rng, n, mean=2048)
    got = device.index_device_blocks(_dev(data, gpu, 3), torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes))


@pytest.mark.parametrize("n", [50 * 8192, 100 * 8192, 300 * 8192, 8415 * 8192, 1 << 30])
def test_default_sort_cdc_lists(gpu, knobs, n):
    # from two waves of blocks (65) the launcher sorts by itself: ~50 blocks
    # stay in list order, ~100, ~300, configs[0]'s one-window list (~8.4 K)
    # and a 1 GiB list (~131 K) are sorted; every digest equals the
    # list-order launch and the oracle
    knobs.set("SF_TEST_TABLE_SORT", -1)
    rng = np.random.default_rng(37_000 + n % 1000)
    data = oracle.splitmix_bytes(n, 47_000)
    offs, sizes = _cdc_like(rng, n)
    t = _dev(data, gpu, 5)
    to, tz = torch.from_numpy(offs).to(gpu), torch.from_numpy(sizes.astype(np.int32)).to(gpu)
    got = device.index_device_blocks(t, to, tz).cpu().numpy()
    knobs.set("SF_TEST_TABLE_SORT", 0)
    assert np.array_equal(got, device.index_device_blocks(t, to, tz).cpu().numpy())
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes))


@pytest.mark.parametrize("nblocks", [64 * 2047, 64 * 2048 - 1, 64 * 2048, 64 * 2048 + 1, 64 * 3072 + 5])
def test_sorted_round_reversal_edges(gpu, knobs, nblocks):
    # wave round 1 (groups 1024..2047 of the sorted order) takes its groups
    # in reverse when the launch holds it whole (kTableReversedRounds): lists just
    # below, at and above 2048 groups, small blocks of every class, every
    # digest at its own index = the oracle
    knobs.set("SF_TEST_TABLE_SORT", 1)
    rng = np.random.default_rng(38_000 + nblocks)
    sizes = rng.integers(0, 600, nblocks).astype(np.int64)
    n = int(sizes.sum()) + 64
    data = oracle.splitmix_bytes(n, 48_000 + nblocks)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64) + int(rng.integers(0, 64))
    t = _dev(data, gpu, 3)
    got = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(got, oracle.index_blocks(data, offs, sizes)), nblocks


def test_sorted_round_reversal_weak(gpu, knobs):
    # the weak-sum form of the kernel maps its waves the same way
    knobs.set("SF_TEST_TABLE_SORT", 1)
    nblocks = 64 * 2048 + 77
    rng = np.random.default_rng(39_000)
    sizes = rng.integers(0, 600, nblocks).astype(np.int64)
    n = int(sizes.sum())
    data = oracle.splitmix_bytes(n, 49_000)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    dig, weak = device.index_device_blocks_weak(_dev(data, gpu), torch.from_numpy(offs).to(gpu),
                                                torch.from_numpy(sizes.astype(np.int32)).to(gpu))
    assert np.array_equal(dig.cpu().numpy(), oracle.index_blocks(data, offs, sizes))
    assert np.array_equal(weak.cpu().numpy().view(np.uint32), oracle.adler_blocks(data, offs, sizes))


def _class_keys(sizes, mbits=4):
    """length_class(n_chunks(size), mbits mantissa bits) clamped at
    (16 << max(mbits, 4)) - 1 (sf_kernels.hpp, sf_capi.hip), in numpy."""
    nch = (sizes.astype(np.int64) + 8) // 64 + 1
    e = np.floor(np.log2(nch)).astype(np.int64)
    k = np.where(nch < (1 << mbits), nch,
                 (e << mbits) + ((nch >> np.maximum(e - mbits, 0)) & ((1 << mbits) - 1)))
    return np.minimum(k, (16 << max(mbits, 4)) - 1)


@pytest.mark.parametrize("n", [1, 63, 64, 2047, 2048, 2049, 100_000, 1 << 20, (1 << 23) + 77])
def test_class_order_is_the_stable_descending_class_sort(gpu, n):
    # the counting sort behind sha1_table_kernel's `order` (sf_sort.hip):
    # classes descending, list order within a class, a permutation of [0, n)
    import ctypes

    from syncfast_amd._lib import check, lib
    rng = np.random.default_rng(38_000 + n)
    sizes = np.concatenate([rng.geometric(1 / 8192, n // 2), rng.integers(0, 1 << 31, n - n // 2)])
    sizes = rng.permutation(np.minimum(sizes, (1 << 31) - 1)).astype(np.uint32)
    sizes[: min(n, 5)] = [0, 1, 55, 56, (1 << 31) - 1][: min(n, 5)]
    ts = torch.from_numpy(sizes.view(np.int32)).to(gpu)
    order = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    check(lib().sf_test_table_order(ts.data_ptr(), n, order.data_ptr(),
                                    ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)),
          "sf_test_table_order")
    got = order.cpu().numpy().view(np.uint32)
    want = np.argsort((255 - _class_keys(sizes)).astype(np.uint8), kind="stable")  # descending, stable
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mbits", [2, 5, 6])
@pytest.mark.parametrize("n", [1, 2049, 100_000, (1 << 21) + 3])
def test_class_order_wider_keys(gpu, n, mbits):
    # the 9- and 10-bit keys of the SF_TABLE_CLASS_BITS knob take the same
    # counting sort with 512 / 1024 bins
    import ctypes

    from syncfast_amd._lib import check, lib
    rng = np.random.default_rng(39_500 + n + mbits)
    sizes = np.concatenate([rng.geometric(1 / 8192, n // 2), rng.integers(0, 1 << 31, n - n // 2)])
    sizes = rng.permutation(np.minimum(sizes, (1 << 31) - 1)).astype(np.uint32)
    ts = torch.from_numpy(sizes.view(np.int32)).to(gpu)
    order = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    check(lib().sf_test_table_order_bits(ts.data_ptr(), n, mbits, order.data_ptr(),
                                         ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)),
          "sf_test_table_order_bits")
    got = order.cpu().numpy().view(np.uint32)
    want = np.argsort(-_class_keys(sizes, mbits), kind="stable")  # descending, stable
    assert np.array_equal(got, want)
