"""GPU: sf_index_buffer_blocks -- an explicit block list over HOST memory, the
form a Rust caller uses when it keeps the reference's own chunker
(cdchunking ZPAQ, src/index.rs:622-625) on the host and hands the bytes and
boundaries to the library: every digest and the blocks_hash in list order
must equal the oracle's restatement of src/index.rs:621-682, across stage
edges (SF_TEST_STREAM_STAGE_MIB shrinks the ~256 MiB stages), for overlapping and
empty blocks, blocks larger than a stage, and lists long enough for the
launcher's length sort (> 64 blocks in one stage)."""
import hashlib
import os

import numpy as np
import pytest

import oracle
from syncfast_amd import host
from syncfast_amd.index import BoundaryChunker, signatures_of_bytes

pytestmark = pytest.mark.gpu

KAT_OFFS = [0, 11579, 44347]
KAT_SIZES = [11579, 32768, 546]
KAT_DIGESTS = ["fb5ef7ebadd82c8085c5ff63823622bae0e263f6", "570d8b30fcfd585e4127b561f5ecd376ff4d0101",
               "b9a8c2641af2cf8fd8f36a2456a3eaa95c029127"]
KAT_BLOCKS_HASH = "84c25d78edcdb67631639c43604cf0149564f044"


@pytest.fixture
def small_stages(knobs):
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)
    yield
    host.release_cache()


def _check(data, offs, sizes):
    rows, bh = host.index_buffer_blocks(data, offs, sizes)
    want = oracle.index_blocks(data, np.asarray(offs, np.uint64), np.asarray(sizes, np.uint32))
    assert rows.size == len(offs)
    assert np.array_equal(rows["offset"], np.asarray(offs, np.uint64))
    assert np.array_equal(rows["size"], np.asarray(sizes, np.uint32))
    assert np.array_equal(rows["sha1"], want)
    assert bh == oracle.blocks_hash(want)
    return rows


def _cdc_like(rng, n, mean=8192, cap=32768):
    sizes = np.minimum(rng.geometric(1.0 / mean, size=n // 64 + 16), cap)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    b = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    return b[:-1], np.diff(b).astype(np.uint32)


def test_reference_kat(gpu):
    """src/index.rs:747-793: the KAT file's three blocks and its blocks_hash."""
    rows, bh = host.index_buffer_blocks(oracle.kat_input(), KAT_OFFS, KAT_SIZES)
    assert [bytes(r).hex() for r in rows["sha1"]] == KAT_DIGESTS
    assert bh.hex() == KAT_BLOCKS_HASH
    assert rows["offset"].tolist() == KAT_OFFS and rows["size"].tolist() == KAT_SIZES


def test_index_kat_through_boundary_chunker(gpu):
    rows = signatures_of_bytes(oracle.kat_input(), BoundaryChunker(lambda d: KAT_SIZES))
    assert [(o, s, d.hex()) for o, s, d in rows] == list(zip(KAT_OFFS, KAT_SIZES, KAT_DIGESTS))


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4096, 1_000_003])
def test_cdc_like_one_stage(gpu, n):
    rng = np.random.default_rng(n)
    data = oracle.splitmix_bytes(n, 0x5EED0000 + n)
    offs, sizes = _cdc_like(rng, n)
    _check(data, offs, sizes)


@pytest.mark.parametrize("n", [3 << 20, (5 << 20) + 777])
def test_cdc_like_many_stages(gpu, small_stages, n):
    rng = np.random.default_rng(n)
    data = oracle.splitmix_bytes(n, 0x5EED0001)
    offs, sizes = _cdc_like(rng, n)
    _check(data, offs, sizes)


def test_blocks_larger_than_a_stage(gpu, small_stages):
    """A 3 MiB block against 1 MiB stages is a stage of its own; the blocks
    around it are staged as usual."""
    n = 8 << 20
    data = oracle.splitmix_bytes(n, 11)
    offs = [0, 1000, 1000 + (3 << 20), (5 << 20) + 1, (5 << 20) + 2]
    sizes = [1000, 3 << 20, 5, (3 << 20) - 3, 1]
    _check(data, offs, sizes)


def test_overlapping_empty_and_gapped_blocks(gpu, small_stages):
    rng = np.random.default_rng(3)
    n = 4 << 20
    data = oracle.splitmix_bytes(n, 12)
    offs = np.sort(rng.integers(0, n, 3000)).astype(np.uint64)
    sizes = np.minimum(rng.integers(0, 70000, offs.size), n - offs).astype(np.uint32)
    sizes[::17] = 0  # SHA-1 of no bytes
    _check(data, offs, sizes)
    # repeated offsets, every block the same range
    _check(data, np.full(100, 12345, np.uint64), np.full(100, 4096, np.uint32))


def test_sorted_launch_inside_a_stage(gpu):
    """2^18 tiny blocks in one stage: the launcher sorts them by length class
    (> 64) and every digest still lands at its own row."""
    rng = np.random.default_rng(9)
    n = 1 << 22
    data = oracle.splitmix_bytes(n, 13)
    sizes = rng.integers(1, 31, 1 << 18).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes, dtype=np.uint64)[:-1]]).astype(np.uint64)
    assert int(offs[-1]) + int(sizes[-1]) <= n
    _check(data, offs, sizes)


def test_fixed_tiling_as_a_list_matches_index_buffer(gpu):
    n = (16 << 20) + 100
    data = oracle.splitmix_bytes(n, 14)
    offs = np.arange(0, n, 4096, dtype=np.uint64)
    sizes = np.minimum(4096, n - offs).astype(np.uint32)
    rows = _check(data, offs, sizes)
    fixed = host.index_buffer(data, 4096)
    assert np.array_equal(rows, fixed)


def test_unaligned_host_buffer(gpu, small_stages):
    """The caller's buffer at an odd address and windows starting mid-word."""
    n = 3 << 20
    raw = oracle.splitmix_bytes(n + 3, 15)
    data = raw[3:]
    assert data.ctypes.data % 4 != 0 or n == 0
    rng = np.random.default_rng(15)
    offs, sizes = _cdc_like(rng, n, mean=3000, cap=9000)
    _check(data, offs, sizes)


def test_errors_leave_nothing_running(gpu):
    data = oracle.splitmix_bytes(1000, 16)
    from syncfast_amd._lib import SF_EINVAL, SF_ERANGE, SfError
    with pytest.raises(SfError) as e:
        host.index_buffer_blocks(data, [0, 999], [10, 2])
    assert e.value.errno == -SF_ERANGE
    with pytest.raises(SfError) as e:
        host.index_buffer_blocks(data, [10, 0], [1, 1])
    assert e.value.errno == -SF_EINVAL
    rows, bh = host.index_buffer_blocks(data, [0], [1000])  # the next call is unaffected
    assert bytes(rows["sha1"][0]) == hashlib.sha1(data.tobytes()).digest()
    assert bh == hashlib.sha1(hashlib.sha1(data.tobytes()).digest()).digest()


def test_stage_knob_does_not_change_results(gpu, knobs):
    rng = np.random.default_rng(17)
    n = 6 << 20
    data = oracle.splitmix_bytes(n, 17)
    offs, sizes = _cdc_like(rng, n)
    a = host.index_buffer_blocks(data, offs, sizes)
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 2)
    try:
        b = host.index_buffer_blocks(data, offs, sizes)
    finally:
        host.release_cache()
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]


def test_file_form_equals_buffer_form(gpu, tmp_path, small_stages):
    """sf_index_file_blocks preads the windows the buffer form copies: same
    rows, same blocks_hash, across 1 MiB stages, with a block past 1 MiB."""
    rng = np.random.default_rng(21)
    n = (5 << 20) + 321
    data = oracle.splitmix_bytes(n, 21)
    p = tmp_path / "cdc.bin"
    data.tofile(p)
    offs, sizes = _cdc_like(rng, n)
    a = host.index_file_blocks(p, offs, sizes)
    b = host.index_buffer_blocks(data, offs, sizes)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]
    _check(data, offs, sizes)
    big_offs = [0, 100, 100 + (3 << 20)]
    big_sizes = [100, 3 << 20, n - 100 - (3 << 20)]
    c = host.index_file_blocks(p, big_offs, big_sizes)
    d = _check(data, big_offs, big_sizes)
    assert np.array_equal(c[0], d)


def test_file_form_reference_kat(gpu, tmp_path):
    p = tmp_path / "kat"
    p.write_bytes(oracle.kat_input())
    rows, bh = host.index_file_blocks(p, KAT_OFFS, KAT_SIZES)
    assert [bytes(r).hex() for r in rows["sha1"]] == KAT_DIGESTS
    assert bh.hex() == KAT_BLOCKS_HASH


def test_file_form_errors(gpu, tmp_path):
    from syncfast_amd._lib import SF_EIO, SF_ERANGE, SfError
    p = tmp_path / "short"
    p.write_bytes(b"x" * 5000)
    with pytest.raises(SfError) as e:
        host.index_file_blocks(p, [0, 4000], [4000, 1001])
    assert e.value.errno == -SF_ERANGE
    fifo = tmp_path / "fifo"
    os.mkfifo(fifo)  # no writer: the library must not wait for one
    with pytest.raises(SfError) as e:
        host.index_file_blocks(fifo, [0], [1])
    assert e.value.errno == -SF_EIO


@pytest.mark.parametrize("env", [{}, {"SF_NO_HOSTREG": 1}, {"SF_TEST_INPLACE_FAIL_AT": 0},
                                 {"SF_TEST_INPLACE_FAIL_AT": 2}])
def test_in_place_and_staged_routes_agree(gpu, env, knobs):
    """The buffer form copies a chunker's list in place (page-locked region by
    region) or through the pinned stages (SF_NO_HOSTREG=1, overlapping
    windows, or a region that cannot be page-locked -- SF_TEST_INPLACE_FAIL_AT=k
    from region k on); every route gives the oracle's rows and blocks_hash."""
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)
    for k, v in env.items():
        knobs.set(k, v)
    rng = np.random.default_rng(33)
    n = (6 << 20) + 4321
    raw = oracle.splitmix_bytes(n + 5, 33)
    for data in (raw[:n], raw[5:]):  # page-aligned-ish and odd start
        offs, sizes = _cdc_like(rng, n)
        _check(data, offs, sizes)
    host.release_cache()


def test_concurrent_in_place_calls_on_shared_pages(gpu):
    """Threads indexing the same host buffer and overlapping slices of it at
    once: each in-place call page-locks its regions; a region another call of
    ours holds is bounced, never copied from while that call may unregister
    it.  Every result equals the oracle's (sf_index_buffer and the list form)."""
    import threading
    n = 48 << 20
    data = oracle.splitmix_bytes(n, 44)
    rng = np.random.default_rng(44)
    offs, sizes = _cdc_like(rng, n)
    want_list = oracle.index_blocks(data, offs, sizes)
    want_fixed = oracle.index_fixed(data, 4096)[2]
    half = (n // 2) + 4096 * 3 + 100  # overlapping halves, sharing pages
    sub = data[n // 2 - 12345:]
    want_sub = oracle.index_fixed(sub, 4096)[2]
    errors = []

    def work(kind):
        try:
            for _ in range(3):
                if kind == 0:
                    rows, _ = host.index_buffer_blocks(data, offs, sizes)
                    assert np.array_equal(rows["sha1"], want_list)
                elif kind == 1:
                    assert np.array_equal(host.index_buffer(data, 4096)["sha1"], want_fixed)
                elif kind == 2:
                    assert np.array_equal(host.index_buffer(sub, 4096)["sha1"], want_sub)
                else:
                    rows = host.index_buffer(data[:half], 4096)
                    assert np.array_equal(rows["sha1"], oracle.index_fixed(data[:half], 4096)[2])
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append((kind, e))

    th = [threading.Thread(target=work, args=(k % 4,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
