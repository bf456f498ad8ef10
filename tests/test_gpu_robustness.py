"""GPU: failure paths of the C-ABI report errors instead of wrong results.

- Equal-size batches with every file's blocks_hash (sf_index_device_batch):
  since round 6 no wave waits for another -- the batch is hashed in two
  column halves with the first half of the chains beside the second half's
  blocks, then the second half of the chains alone (the batch stream's last
  batch) -- so there is no bound to give up at and no SF_ETIMEDOUT (its one
  occurrence, round 5, came from the single fused launch whose chain lanes
  polled stage counters).  Checked for ragged file groups, 70,000 files,
  under uneven load (a long kernel on another stream of the device), two
  streams of batches, the blocks-then-chains form (SF_BATCH_FUSED=0) and
  unaligned outputs; a status word passed in is never written.
- The XCD litmus (sf_test_xcd_litmus): a counter read after other XCDs'
  adds, by a relaxed agent-scope atomic load and by an atomic add of an
  opaque zero.
- A file truncated while indexed (default pread route): no hang or SIGBUS,
  an error or a complete result.
- index_file sized from a stale stat retries with the need (SF_ENOSPC).
- The library's stream-ordered scratch (sf_alloc.cpp): many-file batches and
  a one-file fused cut, alternating in one process with small stages, every
  digest right with the default scratch pool (round 6: the device's default
  pool, which releases freed blocks at every synchronisation, made such a
  loop read wrong data through the sort's workspace)."""
import ctypes
import os
import threading

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, host
from syncfast_amd._lib import FileDesc, SfError, lib

pytestmark = pytest.mark.gpu


def _equal_batch(gpu, nfiles, nbf, bs, seed):
    data = oracle.splitmix_bytes(nfiles * nbf * bs, seed)
    t = torch.from_numpy(data).to(gpu)
    files = [(i * nbf * bs, nbf * bs) for i in range(nfiles)]
    return data, t, files


def _check_batch(data, nfiles, nbf, bs, dig, fh, every=1):
    want = oracle.index_fixed_mt(data, bs, 8)
    assert np.array_equal(dig.cpu().numpy(), want)
    fhn = fh.cpu().numpy()
    for i in list(range(0, nfiles, every)) + [nfiles - 1]:
        assert bytes(fhn[i]) == oracle.blocks_hash(want[i * nbf:(i + 1) * nbf]), i


@pytest.mark.parametrize("nbf", [64, 128, 1024, 2048, 1028])
@pytest.mark.parametrize("nfiles", [1, 63, 64, 65, 130])
def test_batch_halves_every_shape(gpu, nbf, nfiles):
    # files of 64 .. 2048 blocks (64: one column wave, no halves; 1028: not
    # a multiple of 64, blocks then chains) and ragged last chain waves (files
    # not a multiple of 64); the status word passed in is never written
    bs = 1024
    data, t, files = _equal_batch(gpu, nfiles, nbf, bs, 500 + nbf + nfiles)
    st = torch.full((1,), 7, dtype=torch.int32, device=gpu)
    dig, _, fh = device.index_device_batch(t, files, bs, status=st)
    assert int(st.item()) == 7
    _check_batch(data, nfiles, nbf, bs, dig, fh)


def test_staged_under_uneven_load(gpu):
    # a long kernel on another stream of the device holds most of the CUs
    # while fused launches run: the waves of a launch complete in an order
    # far from the dispatch order, and no wave waits for another anyway
    big = device.splitmix_tensor(8 << 30, 9, device=gpu)
    side = torch.cuda.Stream(gpu)
    data, t, files = _equal_batch(gpu, 64, 1024, 4096, 502)
    torch.cuda.synchronize(gpu)
    outs = []
    for r in range(4):
        device.index_device(big, 4096, stream=side)  # ~2.4 ms beside the launches below
        dig = torch.empty((64 * 1024, 20), dtype=torch.uint8, device=gpu)
        fh = torch.empty((64, 20), dtype=torch.uint8, device=gpu)
        device.index_device_batch(t, files, 4096, out=dig, hashes_out=fh)
        outs.append((dig, fh))
    torch.cuda.synchronize(gpu)
    for dig, fh in outs:
        _check_batch(data, 64, 1024, 4096, dig, fh)


@pytest.mark.parametrize("fused", [1, 0])
def test_staged_two_streams(gpu, knobs, fused):
    # fused launches alternating on two streams with nothing between them
    # (sf_index_files' pattern), and the same with SF_BATCH_FUSED=0
    knobs.set("SF_BATCH_FUSED", fused)
    data, t, files = _equal_batch(gpu, 32, 2048, 4096, 503)
    ss = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    outs = []
    for i in range(40):
        s = ss[i & 1]
        with torch.cuda.stream(s):
            dig = torch.empty((32 * 2048, 20), dtype=torch.uint8, device=gpu)
            fh = torch.empty((32, 20), dtype=torch.uint8, device=gpu)
            device.index_device_batch(t, files, 4096, out=dig, hashes_out=fh, stream=s)
            outs.append((dig, fh))
    torch.cuda.synchronize(gpu)
    for dig, fh in outs[:2] + outs[-2:]:
        _check_batch(data, 32, 2048, 4096, dig, fh, every=7)


def test_xcd_counter_litmus(gpu):
    # The poll's read-modify-write (mode 1) returns every add made on other
    # XCDs after the reader's first read put the counter's line in its XCD's
    # L2.  Mode 0 (the relaxed atomic load the poll used until round 6) is run
    # and reported; its outcome is the hardware's, recorded in DESIGN.md 3.3
    # (scripts/xcd_litmus.py), so only its hand-shake is asserted here.
    torch.cuda.set_device(gpu)
    for mode in (1, 0, 1, 0):
        out = (ctypes.c_uint32 * 8)()
        assert lib().sf_test_xcd_litmus(mode, out) == 0
        status, xcc, adders, v0, v1, fresh = list(out)[:6]
        assert status == 0 and adders > 0 and v0 == 0, list(out)
        assert fresh == adders, list(out)  # the read-modify-write read sees every add
        if mode == 1:
            assert v1 == adders, list(out)
        print(f"litmus mode {mode}: reader XCD {xcc}, {adders} adds from other XCDs, second read {v1}")


def test_index_files_blocks_hash(gpu, tmp_path):
    # sf_index_files: every stage's blocks and blocks_hash chains through
    # sf_index_device_batch; every blocks_hash equals the oracle's
    paths = []
    for i in range(32):
        p = tmp_path / f"f{i}"
        p.write_bytes(oracle.splitmix_bytes(8 << 20, 600 + i).tobytes())
        paths.append(str(p))
    rows, first, fh = host.index_files(paths, 4096)
    for i in (0, 5, 31):
        w = oracle.index_fixed(np.fromfile(paths[i], np.uint8), 4096)[2]
        assert bytes(fh[i]) == oracle.blocks_hash(w), i


def test_null_status_raw_call(gpu):
    # the raw C-ABI call with no status word: the same fused launch
    nfiles, nbf, bs = 64, 1024, 4096
    data, t, files = _equal_batch(gpu, nfiles, nbf, bs, 503)
    descs = (FileDesc * nfiles)(*[FileDesc(o, ln) for o, ln in files])
    dig = torch.empty((nfiles * nbf, 20), dtype=torch.uint8, device=gpu)
    fh = torch.empty((nfiles, 20), dtype=torch.uint8, device=gpu)
    nb = ctypes.c_uint64()
    rc = lib().sf_index_device_batch(t.data_ptr(), t.numel(), descs, nfiles, bs, dig.data_ptr(), nfiles * nbf,
                                     fh.data_ptr(), None, ctypes.byref(nb), None,
                                     torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    _check_batch(data, nfiles, nbf, bs, dig, fh, every=31)


def test_wide_batch(gpu):
    # 70,000 equal files, 1094 file groups x 2 stages of chain slices
    nfiles, nbf, bs = 70_000, 128, 64
    data, t, files = _equal_batch(gpu, nfiles, nbf, bs, 504)
    dig, _, fh = device.index_device_batch(t, files, bs)
    _check_batch(data, nfiles, nbf, bs, dig, fh, every=997)


def test_unaligned_outputs(gpu):
    # a hashes_out 20 B into a larger tensor (any alignment is fine for the
    # hashes) and a digest table 4 B off a 16-B boundary (file runs not 16-B
    # aligned: blocks then the per-lane chain kernel); same hashes
    data, t, files = _equal_batch(gpu, 70, 1024, 4096, 505)
    buf = torch.empty((71, 20), dtype=torch.uint8, device=gpu)
    fh = buf[1:]
    dig, _, _ = device.index_device_batch(t, files, 4096, hashes_out=fh)
    _check_batch(data, 70, 1024, 4096, dig, fh, every=13)
    big = torch.empty(70 * 1024 * 20 + 4, dtype=torch.uint8, device=gpu)
    dig2 = big[4:].view(70 * 1024, 20)
    fh2 = torch.empty((70, 20), dtype=torch.uint8, device=gpu)
    device.index_device_batch(t, files, 4096, out=dig2, hashes_out=fh2)
    _check_batch(data, 70, 1024, 4096, dig2, fh2, every=13)


def test_truncated_while_indexed_no_hang(gpu, tmp_path):
    # the default file route only reads the file (pread into pinned stages):
    # a concurrent truncation gives SF_EIO (short read) or a complete result,
    # never a hang or SIGBUS.  (A route that registered the file's mapping
    # with the GPU hung the queues when the file was truncated mid-copy; no
    # route of the library page-locks file-backed memory any more -- DESIGN.md
    # section 6, test_file_mapping_buffer_is_staged_not_page_locked.)
    size, bs = 768 << 20, 4096
    data = oracle.splitmix_bytes(size, 505)
    p = tmp_path / "shrinking"
    outcomes = []
    for k in range(4):
        data.tofile(p)
        cut = threading.Timer(0.004 * k, lambda: os.truncate(p, 3 << 20))
        cut.start()
        try:
            rows, bh = host.index_file(p, bs)
            outcomes.append(("ok", len(rows)))
            got = np.stack([r["sha1"] for r in rows[:4]])
            assert np.array_equal(got, oracle.index_fixed(data[:4 * bs], bs)[2])
            assert len(rows) in (size // bs, (3 << 20) // bs)
        except SfError as e:
            outcomes.append((e.code, None))
        finally:
            cut.join()
    assert all(o[0] in ("ok", -5) for o in outcomes), outcomes


@pytest.mark.parametrize("form", ["fixed", "list"])
def test_file_mapping_buffer_is_staged_not_page_locked(gpu, tmp_path, form):
    """A caller's MAP_SHARED file mapping (Rust's memmap pattern) handed to
    sf_index_buffer / sf_index_buffer_blocks is never page-locked (a GPU
    userptr over a file that can be truncated under the copies hung the
    queues): the library sees it is not private anonymous memory, copies it
    through the pinned stages, and the rows are the oracle's.  An anonymous
    buffer of the same bytes is page-locked in place (the counter moves), so
    the test tells the routes apart."""
    import mmap
    from syncfast_amd import _lib
    n = (40 << 20) + 4093
    data = oracle.splitmix_bytes(n, 507)
    p = tmp_path / "mapped.bin"
    data.tofile(p)
    rng = np.random.default_rng(507)
    if form == "list":
        sizes = np.minimum(32768, np.maximum(1, rng.geometric(1 / 8192, n // 4096))).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        keep = offs + sizes <= n
        offs, sizes = offs[keep], sizes[keep]
        want = oracle.index_blocks(data, offs, sizes)
    else:
        want = oracle.index_fixed(data, 4096)[2]

    def run(buf):
        if form == "list":
            rows, bh = host.index_buffer_blocks(buf, offs, sizes)
            assert bh == oracle.blocks_hash(want)
            return rows
        return host.index_buffer(buf, 4096)

    with open(p, "rb") as f:
        mm = mmap.mmap(f.fileno(), n, mmap.MAP_SHARED, mmap.PROT_READ)
    locked, refused = _lib.get_stat("pages_locked"), _lib.get_stat("not_anon_refused")
    view = np.frombuffer(mm, np.uint8)
    try:
        rows = run(view)
    finally:
        del view  # the array's buffer export must go before the mapping closes
        mm.close()
    assert np.array_equal(rows["sha1"], want)
    assert _lib.get_stat("pages_locked") == locked, "a file mapping was page-locked"
    assert _lib.get_stat("not_anon_refused") > refused
    anon = data.copy()
    locked = _lib.get_stat("pages_locked")
    assert np.array_equal(run(anon)["sha1"], want)
    assert _lib.get_stat("pages_locked") > locked  # the anonymous buffer took the in-place route


def test_index_file_retries_when_the_file_grew(gpu, monkeypatch, tmp_path):
    p = tmp_path / "grows"
    data = oracle.splitmix_bytes(5 * 4096 + 7, 506)
    data.tofile(p)
    real = os.path.getsize
    monkeypatch.setattr(host.os.path, "getsize", lambda path: real(path) - 3 * 4096)  # a stale, smaller size
    rows, bh = host.index_file(p, 4096)
    offs, sizes, want = oracle.index_fixed(data, 4096)
    assert len(rows) == 6 and np.array_equal(np.stack([r["sha1"] for r in rows]), want)
    assert bh == oracle.blocks_hash(want)


def test_concurrent_mixed_host_calls(gpu, tmp_path):
    # the per-device cache under contention: six threads mixing buffer, file,
    # fd, file-range and many-file calls (ctypes drops the GIL, so they run in
    # parallel in the library) while a seventh releases the cache; every
    # result equals the oracle's
    import concurrent.futures as cf
    bs = 4096
    big = oracle.splitmix_bytes((48 << 20) + 999, 510)
    small = [oracle.splitmix_bytes(n, 520 + i) for i, n in enumerate([0, 1, 5000, 70_000, 300_000])]
    pb = tmp_path / "big"
    big.tofile(pb)
    ps = []
    for i, d in enumerate(small):
        p = tmp_path / f"s{i}"
        d.tofile(p)
        ps.append(p)
    want_big = oracle.index_fixed(big, bs)[2]
    want_small = [oracle.index_fixed(d, bs)[2] for d in small]

    def job(kind):
        torch.cuda.set_device(gpu)
        for _ in range(4):
            if kind == 0:
                assert np.array_equal(host.index_buffer(big, bs)["sha1"], want_big)
            elif kind == 1:
                rows, bh = host.index_file(pb, bs)
                assert np.array_equal(rows["sha1"], want_big) and bh == oracle.blocks_hash(want_big)
            elif kind == 2:
                fd = os.open(pb, os.O_RDONLY)
                try:
                    rows, bh = host.index_fd(fd, bs)
                finally:
                    os.close(fd)
                assert np.array_equal(rows["sha1"], want_big)
            elif kind == 3:
                half = (big.size // 2) // bs * bs
                a = host.index_file_range(pb, 0, half, bs)
                b = host.index_file_range(pb, half, big.size - half, bs)
                assert np.array_equal(np.concatenate([a, b])["sha1"], want_big)
            elif kind == 4:
                rows, first, fh = host.index_files(ps, bs)
                for k, w in enumerate(want_small):
                    assert np.array_equal(rows[int(first[k]):int(first[k + 1])]["sha1"].reshape(-1, 20), w)
                    assert bytes(fh[k]) == oracle.blocks_hash(w)
            elif kind == 5:
                assert np.array_equal(host.index_buffer(small[3], bs)["sha1"].reshape(-1, 20), want_small[3])
            else:
                host.release_cache()
        return kind

    with cf.ThreadPoolExecutor(7) as ex:
        assert sorted(ex.map(job, range(7))) == list(range(7))


def test_side_stream_status_is_read_on_that_stream(gpu):
    # status words are zeroed, written and read on the caller's stream: an
    # out-of-range block on a side stream, queued behind a long kernel there,
    # is still reported; a clean call on the same stream is not
    data = torch.from_numpy(oracle.splitmix_bytes(1 << 20, 3)).to(gpu)
    big = torch.empty(1 << 30, dtype=torch.uint8, device=gpu)
    s = torch.cuda.Stream(device=gpu)
    offs = torch.tensor([0, 1 << 20], dtype=torch.int64, device=gpu)
    sizes = torch.tensor([100, 1], dtype=torch.int32, device=gpu)
    for _ in range(3):
        device.index_device(big, 4096, stream=s)  # keeps the side stream busy
        with pytest.raises(SfError):
            device.index_device_blocks(data, offs, sizes, stream=s)
        device.index_device(big, 4096, stream=s)
        got = device.index_device_blocks(data, offs[:1], sizes[:1], stream=s)
        s.synchronize()
        assert bytes(got[0].cpu().numpy()) == oracle.sha1(oracle.splitmix_bytes(100, 3))


@pytest.mark.parametrize("pool", [1, 2])
def test_scratch_pool_under_alternating_calls(gpu, knobs, tmp_path, pool):
    # sf_index_fds_blocks (1 MiB stages on two streams, every stage's list
    # sorted through the scratch pool) and sf_index_fd_cut (one 2 MiB window,
    # its list sorted) in turn, 25 times: every row = the oracle's.  Pool 1 is
    # the default; 2 the same pool with the runtime's cross-stream reuse on
    # (both kept their blocks and were right in 480 iterations, the pools
    # that release at every synchronisation wrong in most:
    # scripts/sort_race_stress.py)
    import ctypes as C
    knobs.set("SF_TEST_STREAM_POOL", pool)
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)
    Z = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "build",
                            "libzpaq_standin.so"))
    Z.sf_zpaq_standin_ops.restype = C.c_void_p
    Z.sf_zpaq_standin_ops.argtypes = [C.c_uint, C.c_uint32]
    ops = Z.sf_zpaq_standin_ops(13, 32768)
    rng = np.random.default_rng(77)
    files = []
    for k, n in enumerate([int(x) for x in rng.integers(1, 300_000, 24)]):
        p = tmp_path / f"s{k:02d}"
        d = oracle.splitmix_bytes(n, 5_100 + k)
        d.tofile(p)
        z = oracle.zpaq_standin_sizes(d).astype(np.uint32)
        o = np.concatenate([[0], np.cumsum(z, dtype=np.uint64)[:-1]]).astype(np.uint64)
        files.append((str(p), o, z, oracle.index_blocks(d, o, z)))
    big = oracle.splitmix_bytes(2 << 20, 5_199)
    bp = tmp_path / "big"
    big.tofile(bp)
    bz = oracle.zpaq_standin_sizes(big).astype(np.uint32)
    bwant = oracle.index_blocks(big, np.concatenate([[0], np.cumsum(bz, dtype=np.uint64)[:-1]]).astype(np.uint64), bz)
    for it in range(25):
        fds = [os.open(p, os.O_RDONLY) for p, *_ in files]
        try:
            rows, first, _bh, st = host.index_fds_blocks(fds, [(o, z) for _p, o, z, _w in files])
        finally:
            for fd in fds:
                os.close(fd)
        for k, (_p, _o, _z, want) in enumerate(files):
            assert int(st[k]) == 0 and np.array_equal(rows["sha1"][first[k]:first[k + 1]].reshape(-1, 20), want), \
                (it, k)
        fd = os.open(bp, os.O_RDONLY)
        try:
            got, _ = host.index_fd_cut(fd, ops, 4)
        finally:
            os.close(fd)
        assert np.array_equal(got["sha1"].reshape(-1, 20), bwant), it
