"""GPU parity: the HIP path (through the C-ABI) vs the oracle, bit for bit.

Sizes are chosen so the oracle finishes in seconds; full-size properties are
in test_gpu_fullsize.py.  Every case checks all 20 bytes of every digest.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import SfError, _lib, device, host

pytestmark = pytest.mark.gpu


def to_dev(b, dev):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) if len(b) else torch.empty(0, dtype=torch.uint8, device=dev)


def hexes(d):
    return [bytes(r).hex() for r in (d.cpu().numpy() if isinstance(d, torch.Tensor) else d)]


def test_device_generator_matches_oracle(gpu):
    for n, seed, start in [(1 << 20, 0x5EED0000, 0), (12345, 7, 3), (4097, 9, 16), (0, 1, 0)]:
        t = torch.empty(n, dtype=torch.uint8, device=gpu)
        device.fill_splitmix(t, seed, start)
        assert np.array_equal(t.cpu().numpy(), oracle.splitmix_bytes(n, seed, start))


def test_reference_kat_on_device(gpu, golden):
    g = golden["reference_kat"]
    t = to_dev(oracle.kat_input(), gpu)
    offs = torch.tensor([b["offset"] for b in g["blocks"]], dtype=torch.int64, device=gpu)
    sizes = torch.tensor([b["size"] for b in g["blocks"]], dtype=torch.int32, device=gpu)
    d = device.index_device_blocks(t, offs, sizes)
    assert hexes(d) == [b["sha1"] for b in g["blocks"]]
    assert host.blocks_hash(d.cpu().numpy()).hex() == g["blocks_hash"]


def test_fixed_golden_on_device(gpu, golden):
    for case in golden["fixed"]:
        t = torch.empty(case["len"], dtype=torch.uint8, device=gpu)
        device.fill_splitmix(t, case["seed"])
        d = device.index_device(t, case["block_size"])
        assert hexes(d) == case["digests"], (case["len"], case["block_size"])
        assert host.blocks_hash(d.cpu().numpy()).hex() == case["blocks_hash"]


def test_ragged_golden_on_device(gpu, golden):
    for case in golden["ragged"]:
        t = torch.empty(case["len"], dtype=torch.uint8, device=gpu)
        device.fill_splitmix(t, case["seed"])
        offs = torch.tensor(case["offsets"], dtype=torch.int64, device=gpu)
        sizes = torch.tensor(case["sizes"], dtype=torch.int32, device=gpu)
        d = device.index_device_blocks(t, offs, sizes)
        assert hexes(d) == case["digests"]


@pytest.mark.parametrize("bs", [1, 16, 64, 80, 100, 1000, 4080, 4095, 4096, 4097, 4112, 8192, 65536, 1 << 20])
def test_fixed_random_lengths(gpu, bs):
    rng = np.random.default_rng(bs)
    for _ in range(3):
        nblk = int(rng.integers(1, 300)) if bs < 65536 else int(rng.integers(1, 40))
        n = max(0, nblk * bs + int(rng.integers(-bs + 1, bs)))
        data = oracle.splitmix_bytes(n, int(rng.integers(0, 1 << 62)))
        d = device.index_device(to_dev(data.tobytes(), gpu), bs)
        _, _, want = oracle.index_fixed(data, bs)
        assert np.array_equal(d.cpu().numpy(), want), (bs, n)


@pytest.mark.parametrize("shift", [1, 2, 3, 4, 8, 12, 15])
def test_misaligned_base_pointer(gpu, shift):
    # data pointer not 16-B aligned -> the per-lane (non-LDS) path
    n = 4096 * 70 + 333
    raw = oracle.splitmix_bytes(n + shift, 5)
    t = to_dev(raw.tobytes(), gpu)[shift:]
    assert t.data_ptr() % 16 != 0
    d = device.index_device(t, 4096)
    _, _, want = oracle.index_fixed(raw[shift:], 4096)
    assert np.array_equal(d.cpu().numpy(), want)


def test_empty_input(gpu):
    d = device.index_device(torch.empty(0, dtype=torch.uint8, device=gpu), 4096)
    assert d.shape == (0, 20)


def test_table_unsorted_overlapping_empty_blocks(gpu):
    rng = np.random.default_rng(11)
    n = 500_000
    data = oracle.splitmix_bytes(n, 77)
    t = to_dev(data.tobytes(), gpu)
    m = 1000
    sizes = rng.integers(0, 40_000, m).astype(np.int64)
    sizes[rng.integers(0, m, 50)] = 0
    offs = np.array([int(rng.integers(0, n - s + 1)) for s in sizes], np.int64)
    # a few 16-B aligned runs so some waves take the LDS path
    offs[:128] = (offs[:128] // 16) * 16
    d = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu), torch.from_numpy(sizes.astype(np.int32)).to(gpu))
    want = oracle.index_blocks(data, offs, sizes)
    assert np.array_equal(d.cpu().numpy(), want)


def test_table_aligned_contiguous_blocks(gpu):
    # every block 16-B aligned and contiguous: all waves on the LDS path, with
    # ragged per-lane sizes (mixed full tiles + per-lane tails)
    rng = np.random.default_rng(12)
    sizes = (rng.integers(1, 600, 777) * 16 + rng.integers(0, 16, 777) * (rng.random(777) < 0.3)).astype(np.int64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(((sizes + 15) // 16) * 16)[:-1]
    n = int(offs[-1] + sizes[-1])
    data = oracle.splitmix_bytes(n, 78)
    t = to_dev(data.tobytes(), gpu)
    d = device.index_device_blocks(t, torch.from_numpy(offs).to(gpu), torch.from_numpy(sizes.astype(np.int32)).to(gpu))
    assert np.array_equal(d.cpu().numpy(), oracle.index_blocks(data, offs, sizes))


def test_table_out_of_range_reports_erange(gpu):
    t = to_dev(b"x" * 1000, gpu)
    offs = torch.tensor([0, 990], dtype=torch.int64, device=gpu)
    sizes = torch.tensor([10, 11], dtype=torch.int32, device=gpu)
    with pytest.raises(SfError) as e:
        device.index_device_blocks(t, offs, sizes)
    assert e.value.code == -34


def test_batch_contiguous_files(gpu):
    nfiles, flen, bs = 37, 8 * 4096, 4096
    data = oracle.splitmix_bytes(nfiles * flen, 90)
    t = to_dev(data.tobytes(), gpu)
    files = [(i * flen, flen) for i in range(nfiles)]
    dig, first, fh = device.index_device_batch(t, files, bs)
    _, _, want = oracle.index_fixed(data, bs)
    assert np.array_equal(dig.cpu().numpy(), want)
    assert list(first) == [i * 8 for i in range(nfiles + 1)]
    fhn = fh.cpu().numpy()
    for i in range(nfiles):
        assert bytes(fhn[i]) == oracle.blocks_hash(want[8 * i:8 * i + 8])


def test_batch_ragged_files(gpu):
    rng = np.random.default_rng(91)
    bs = 4096
    lens = [int(x) for x in rng.integers(0, 60_000, 50)]
    lens[3] = 0
    lens[7] = 4096 * 3
    offs, o = [], 0
    for ln in lens:
        offs.append(o)
        o += ln + int(rng.integers(0, 40))  # gaps, unaligned file starts
    data = oracle.splitmix_bytes(o, 92)
    t = to_dev(data.tobytes(), gpu)
    dig, first, fh = device.index_device_batch(t, list(zip(offs, lens)), bs)
    dign, fhn = dig.cpu().numpy(), fh.cpu().numpy()
    for i, (fo, ln) in enumerate(zip(offs, lens)):
        _, _, want = oracle.index_fixed(data[fo:fo + ln], bs)
        got = dign[first[i]:first[i + 1]]
        assert np.array_equal(got, want), i
        assert bytes(fhn[i]) == oracle.blocks_hash(want), i


def test_index_buffer_end_to_end(gpu):
    n = 3 * (256 << 20) // 2 + 12345  # > one pipeline stage
    data = oracle.splitmix_bytes(n, 93)
    rows = host.index_buffer(data, 4096)
    want = oracle.index_fixed_mt(data, 4096, 8)
    assert np.array_equal(rows["sha1"], want)
    assert rows["offset"][1] == 4096 and int(rows["size"].sum()) == n


def test_index_file_end_to_end(gpu):
    data = oracle.splitmix_bytes(5 * 1000 * 1000 + 7, 94)
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(data.tobytes())
        path = f.name
    try:
        rows, bh = host.index_file(path, 65536)
    finally:
        os.unlink(path)
    _, _, want = oracle.index_fixed(data, 65536)
    assert np.array_equal(rows["sha1"], want)
    assert bh == oracle.blocks_hash(want)


def test_index_file_large_never_page_locks(gpu):
    # sf_index_file reads the file with pread into the pinned stages; it never
    # maps and page-locks it (a truncation under a registered file mapping
    # hung the GPU queues), even when it is in the page cache
    data = oracle.splitmix_bytes((96 << 20) + 4093, 95)
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(data.tobytes())
        path = f.name
    locked = _lib.get_stat("pages_locked")
    try:
        rows, bh = host.index_file(path, 4096)
    finally:
        os.unlink(path)
    assert _lib.get_stat("pages_locked") == locked
    offs, sizes, want = oracle.index_fixed(data, 4096)
    assert np.array_equal(rows["sha1"], want)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    assert bh == oracle.blocks_hash(want)


@pytest.fixture(scope="module")
def inplace_case():
    # 2.4 pipeline stages (256 MiB each) + a ragged tail, so stage and
    # page-lock region edges both fall inside blocks
    n = 5 * (256 << 20) // 2 + 4093
    data = oracle.splitmix_bytes(n + 3, 96)
    return data, oracle.index_fixed_mt(data[3:], 4096, 8)


@pytest.mark.parametrize("knob", [("", ""), ("SF_INPLACE_SERIAL", "1"), ("SF_TEST_INPLACE_FAIL_AT", "0"),
                                  ("SF_TEST_INPLACE_FAIL_AT", "1"), ("SF_TEST_INPLACE_FAIL_AT", "2")])
def test_index_buffer_inplace_routes(gpu, inplace_case, knob, knobs):
    # sf_index_buffer page-locks the caller's pages one region ahead of the
    # copy that reads them; data[3:] is not page-aligned, so a stage reads the
    # last page of the previous region.  FAIL_AT=0: nothing can be locked
    # (staged route); FAIL_AT=k>0: regions >= k are copied through a bounce
    # buffer; SERIAL: whole range locked up front, rows after the last stage.
    if knob[0]:
        knobs.set(knob[0], int(knob[1]))
    data, want = inplace_case
    n = data.size - 3
    rows = host.index_buffer(data[3:], 4096)
    assert np.array_equal(rows["sha1"], want)
    assert rows["offset"][-1] == (n - 1) // 4096 * 4096 and int(rows["size"].sum()) == n


def test_index_buffer_already_pinned(gpu, inplace_case):
    # a caller buffer that is already page-locked (torch pinned memory =
    # hipHostMalloc): hipHostRegister reports it registered, and the stages
    # are copied from it in place
    data, want = inplace_case
    pinned = torch.empty(data.size, dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = data
    rows = host.index_buffer(pinned.numpy()[3:], 4096)
    assert np.array_equal(rows["sha1"], want)


def test_host_cache_reuse_release_and_threads(gpu, inplace_case):
    # the per-device set kept between calls: a smaller call after a larger
    # one, a release, and two threads at once (one takes the cached set, the
    # other a private one) all give the oracle's rows
    import threading
    data, want = inplace_case
    small = data[3:3 + (100 << 20) + 77]
    want_small = oracle.index_fixed_mt(small, 4096, 8)  # its last block is short
    assert np.array_equal(host.index_buffer(data[3:], 4096)["sha1"], want)
    assert np.array_equal(host.index_buffer(small, 4096)["sha1"], want_small)
    host.release_cache()
    assert np.array_equal(host.index_buffer(small, 4096)["sha1"], want_small)
    got = [None, None]

    def run(i):
        torch.cuda.set_device(gpu)
        got[i] = host.index_buffer(data[3:] if i == 0 else small, 4096)["sha1"]

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert np.array_equal(got[0], want) and np.array_equal(got[1], want_small)


def test_index_file_multi_stage(gpu, inplace_case, tmp_path):
    # a file of 2.4 stages through the pread pipeline, blocks_hash folded in
    # stage by stage
    data, want = inplace_case
    path = tmp_path / "f.bin"
    path.write_bytes(data[3:].tobytes())
    rows, bh = host.index_file(str(path), 4096)
    assert np.array_equal(rows["sha1"], want)
    assert bh == oracle.blocks_hash(want)


@pytest.mark.parametrize("min_mib", ["", "1024"])
def test_small_buffer_and_file_routes(gpu, min_mib, knobs, tmp_path):
    # defaults: buffers >= 1 MiB in place; SF_INPLACE_MIN_MIB=1024 stages them
    # through the pinned buffers; files always take the pread pipeline
    if min_mib:
        knobs.set("SF_INPLACE_MIN_MIB", int(min_mib))
    for n, seed in [((2 << 20) + 13, 97), ((20 << 20) + 4095, 98)]:
        data = oracle.splitmix_bytes(n + 5, seed)
        _, _, want = oracle.index_fixed(data[5:], 4096)
        assert np.array_equal(host.index_buffer(data[5:], 4096)["sha1"], want)
        path = tmp_path / f"f{seed}.bin"
        path.write_bytes(data[5:].tobytes())
        rows, bh = host.index_file(str(path), 4096)
        assert np.array_equal(rows["sha1"], want) and bh == oracle.blocks_hash(want)


def test_launch_ignores_stale_thread_error(gpu, tmp_path):
    # a failing HIP call earlier on the same thread (here hipSetDevice on a
    # device that does not exist, through the runtime the library is linked
    # against) leaves hipGetLastError() set; the launchers clear it before
    # their own launch, so it is not reported as a launch failure (round 5's
    # full GPU run failed once this way: SF_ENODEV from a good in-place call)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    data = oracle.splitmix_bytes((2 << 20) + 13, 99)
    _, _, want = oracle.index_fixed(data, 4096)
    offs = np.arange(0, data.size, 5000, dtype=np.uint64)
    sizes = np.minimum(5000 + (np.arange(offs.size) % 7) * 100, data.size - offs).astype(np.uint32)
    path = tmp_path / "f.bin"
    path.write_bytes(data.tobytes())
    t = to_dev(data.tobytes(), gpu)

    def poison():
        assert hip.hipSetDevice(ctypes.c_int(1 << 20)) != 0
    poison()
    assert np.array_equal(host.index_buffer(data, 4096)["sha1"], want)
    poison()
    rows, _ = host.index_buffer_blocks(data, offs, sizes)
    assert [bytes(r) for r in rows["sha1"][:3]] == [oracle.sha1(data[o:o + s]) for o, s in zip(offs[:3], sizes[:3])]
    poison()
    rows, bh = host.index_file(str(path), 4096)
    assert np.array_equal(rows["sha1"], want) and bh == oracle.blocks_hash(want)
    poison()
    assert np.array_equal(device.index_device(t, 4096).cpu().numpy(), want)


def test_block_digest_independent_of_neighbours(gpu):
    # the same block bytes at different positions / in different waves give
    # the same digest (no cross-lane leakage through the LDS tile)
    bs = 4096
    blk = oracle.splitmix_bytes(bs, 1234)
    noise = oracle.splitmix_bytes(200 * bs, 4321)
    buf = noise.copy()
    for i in (0, 63, 64, 65, 127, 199):
        buf[i * bs:(i + 1) * bs] = blk
    d = device.index_device(to_dev(buf.tobytes(), gpu), bs).cpu().numpy()
    ref = oracle.sha1(blk)
    for i in (0, 63, 64, 65, 127, 199):
        assert bytes(d[i]) == ref


@pytest.mark.parametrize("nfiles,nbf", [(64, 1024), (3, 256), (130, 64)])
def test_batch_staged_chains(gpu, nfiles, nbf):
    # equal-size contiguous files: column stages + per-file chains on a side stream
    bs = 4096
    data = oracle.splitmix_bytes(nfiles * nbf * bs, 95 + nbf)
    t = to_dev(data.tobytes(), gpu)
    files = [(i * nbf * bs, nbf * bs) for i in range(nfiles)]
    dig, first, fh = device.index_device_batch(t, files, bs)
    want = oracle.index_fixed_mt(data, bs, 8)
    assert np.array_equal(dig.cpu().numpy(), want)
    fhn = fh.cpu().numpy()
    for i in range(nfiles):
        assert bytes(fhn[i]) == oracle.blocks_hash(want[i * nbf:(i + 1) * nbf]), i


def test_batch_staged_repeated_calls_no_stale_digests(gpu):
    # the chains read digests written by other CUs/XCDs of a concurrently
    # running kernel: call repeatedly into the SAME output buffers with
    # different data and check every result (a missing release/acquire
    # shows up as stale digests from the previous call)
    nfiles, nbf, bs = 128, 512, 4096
    n = nfiles * nbf * bs
    t = torch.empty(n, dtype=torch.uint8, device=gpu)
    dig = torch.empty((nfiles * nbf, 20), dtype=torch.uint8, device=gpu)
    fh = torch.empty((nfiles, 20), dtype=torch.uint8, device=gpu)
    files = [(i * nbf * bs, nbf * bs) for i in range(nfiles)]
    for seed in (7001, 7002, 7003):
        device.fill_splitmix(t, seed)
        device.index_device_batch(t, files, bs, out=dig, hashes_out=fh)
        want = oracle.index_fixed_mt(oracle.splitmix_bytes(n, seed), bs, 8)
        assert np.array_equal(dig.cpu().numpy(), want), seed
        fhn = fh.cpu().numpy()
        for i in range(nfiles):
            assert bytes(fhn[i]) == oracle.blocks_hash(want[i * nbf:(i + 1) * nbf]), (seed, i)


def test_max_block_size(gpu):
    # SF_MAX_BLOCK_SIZE = 32 MiB: 64 such blocks span 2 GiB (still one LDS span)
    bs = 32 << 20
    n = 2 * bs + 12345
    data = oracle.splitmix_bytes(n, 96)
    d = device.index_device(to_dev(data.tobytes(), gpu), bs)
    _, _, want = oracle.index_fixed(data, bs)
    assert np.array_equal(d.cpu().numpy(), want)
    with pytest.raises(SfError):
        device.index_device(to_dev(b"x" * 100, gpu), bs + 1)


def test_concurrent_host_threads_own_streams(gpu):
    # include/syncfast_amd.h: device entry points may be called from several
    # host threads on different streams -- every result still exact
    import threading
    bufs = [oracle.splitmix_bytes(4096 * 300 + 17 * k, 600 + k) for k in range(4)]
    outs, errs = [None] * 4, []

    def work(k):
        try:
            s = torch.cuda.Stream(device=gpu)
            with torch.cuda.stream(s):
                t = to_dev(bufs[k].tobytes(), gpu)
                for _ in range(3):
                    d = device.index_device(t, 4096, stream=s)
                    w = device.index_device_weak(t, 4096, stream=s)[0]
                s.synchronize()
                outs[k] = (d.cpu().numpy(), w.cpu().numpy())
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for k in range(4):
        want = oracle.index_fixed(bufs[k], 4096)[2]
        assert np.array_equal(outs[k][0], want) and np.array_equal(outs[k][1], want)


@pytest.mark.parametrize("n,bs,stage_mib", [((20 << 20) + 4095, 4096, "3"), ((7 << 20) + 1, 1000, "1"),
                                           ((6 << 20), 65536, "1"), (4096 * 3, 4096, "1")])
def test_index_file_pread_small_stages(gpu, knobs, tmp_path, n, bs, stage_mib):
    # the pread pipeline with small stages: many stage edges, rows and the
    # streaming blocks_hash emitted stage by stage in file order
    knobs.set("SF_TEST_STREAM_STAGE_MIB", int(stage_mib))
    data = oracle.splitmix_bytes(n, 990 + bs % 97)
    path = tmp_path / "s.bin"
    data.tofile(path)
    rows, bh = host.index_file(str(path), bs)
    offs, sizes, want = oracle.index_fixed(data, bs)
    assert np.array_equal(rows["sha1"], want)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    assert bh == oracle.blocks_hash(want)
