"""GPU: failure paths of the C-ABI report errors instead of wrong results.

- The fused many-file launch (sha1_staged_kernel): its blocks_hash lanes wait
  (bounded) for block digests; a wait that gives up must surface as
  SF_ETIMEDOUT in the caller's status word (or SfError from the Python
  wrapper), never as an all-zero blocks_hash with rc = 0 (the reference never
  yields a hash it did not compute, src/index.rs:661-682); sf_index_files
  never takes the waiting path.  Forced with SF_TEST_CHAIN_SPIN_LIMIT=0 (one
  poll per wait; test hook).
- The lanes' poll sees every XCD's arrivals: a lane whose first poll comes
  before the block waves finish and whose next comes after they all have
  (SF_TEST_CHAIN_POLL_GAP_US) completes at the default bound, and the XCD
  litmus (sf_test_xcd_litmus) shows the poll's read-modify-write seeing adds
  made on other XCDs after its XCD's L2 holds the line.
- Batches too wide for the fused launch's chain workgroups to stay below the
  resident capacity, and callers without a status word, take the non-waiting
  path: correct hashes even with the spin limit at 0.
- A file truncated while indexed (default pread route): no hang or SIGBUS,
  an error or a complete result.
- index_file sized from a stale stat retries with the need (SF_ENOSPC)."""
import ctypes
import os
import threading

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, host
from syncfast_amd._lib import SF_ETIMEDOUT, FileDesc, SfError, lib

pytestmark = pytest.mark.gpu


def _equal_batch(gpu, nfiles, nbf, bs, seed):
    data = oracle.splitmix_bytes(nfiles * nbf * bs, seed)
    t = torch.from_numpy(data).to(gpu)
    files = [(i * nbf * bs, nbf * bs) for i in range(nfiles)]
    return data, t, files


def test_staged_chain_timeout_is_reported(gpu, knobs):
    knobs.set("SF_TEST_CHAIN_SPIN_LIMIT", 0)
    data, t, files = _equal_batch(gpu, 64, 1024, 4096, 501)  # 256 MiB: stage 0 cannot be done at the first poll
    # the asynchronous form: the caller's status word carries it
    st = torch.zeros(1, dtype=torch.int32, device=gpu)
    device.index_device_batch(t, files, 4096, status=st)
    assert int(st.item()) == SF_ETIMEDOUT
    # without one, the wrapper raises: no hash it did not compute, no rerun
    with pytest.raises(SfError) as e:
        device.index_device_batch(t, files, 4096)
    assert e.value.code == SF_ETIMEDOUT


@pytest.mark.parametrize("gap_us", [50_000, 20])
def test_staged_poll_after_every_block_wave_finished(gpu, knobs, gap_us):
    # A lane's first poll of stage 0 comes right at the launch's start (the
    # chain workgroups are dispatched first), before the stage is done; with a
    # 50 ms gap its next poll comes after every block wave of the 256 MiB
    # launch has finished, when no XCD adds to the counters any more (the
    # window in which an L2-served load of the counter line stays stale);
    # with 20 us it polls many times while they run.  The default bound
    # holds either way and every blocks_hash is the oracle's.
    knobs.set("SF_TEST_CHAIN_POLL_GAP_US", gap_us)
    data, t, files = _equal_batch(gpu, 64, 1024, 4096, 508)
    st = torch.zeros(1, dtype=torch.int32, device=gpu)
    dig, _, fh = device.index_device_batch(t, files, 4096, status=st)
    assert int(st.item()) == 0
    want = oracle.index_fixed_mt(data, 4096, 8)
    assert np.array_equal(dig.cpu().numpy(), want)
    fhn = fh.cpu().numpy()
    for i in range(64):
        assert bytes(fhn[i]) == oracle.blocks_hash(want[i * 1024:(i + 1) * 1024]), i


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


def test_staged_default_spin_limit_is_green(gpu):
    data, t, files = _equal_batch(gpu, 64, 1024, 4096, 502)
    st = torch.zeros(1, dtype=torch.int32, device=gpu)
    dig, _, fh = device.index_device_batch(t, files, 4096, status=st)
    assert int(st.item()) == 0
    want = oracle.index_fixed_mt(data, 4096, 8)
    assert np.array_equal(dig.cpu().numpy(), want)
    assert bytes(fh.cpu().numpy()[63]) == oracle.blocks_hash(want[63 * 1024:])


def test_index_files_never_waits(gpu, tmp_path, knobs):
    # sf_index_files hashes each stage on the batch path that never waits
    # (no status word: block kernel, then chain kernel), so a zero spin limit
    # changes nothing: every blocks_hash equals the oracle's
    paths = []
    for i in range(32):
        p = tmp_path / f"f{i}"
        p.write_bytes(oracle.splitmix_bytes(8 << 20, 600 + i).tobytes())
        paths.append(str(p))
    rows, first, fh = host.index_files(paths, 4096)  # green first
    want = oracle.index_fixed(np.fromfile(paths[5], np.uint8), 4096)[2]
    assert bytes(fh[5]) == oracle.blocks_hash(want)
    knobs.set("SF_TEST_CHAIN_SPIN_LIMIT", 0)
    rows2, first2, fh2 = host.index_files(paths, 4096)
    assert np.array_equal(rows2, rows) and np.array_equal(first2, first) and np.array_equal(fh2, fh)
    for i in (0, 5, 31):
        w = oracle.index_fixed(np.fromfile(paths[i], np.uint8), 4096)[2]
        assert bytes(fh2[i]) == oracle.blocks_hash(w), i


def test_null_status_takes_nonwaiting_path(gpu, knobs):
    # no status word: the batch runs block kernel + chain kernel (no waits),
    # so even a zero spin limit gives the right hashes
    knobs.set("SF_TEST_CHAIN_SPIN_LIMIT", 0)
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
    want = oracle.index_fixed_mt(data, bs, 8)
    fhn = fh.cpu().numpy()
    assert np.array_equal(dig.cpu().numpy(), want)
    for i in (0, 31, 63):
        assert bytes(fhn[i]) == oracle.blocks_hash(want[i * nbf:(i + 1) * nbf]), i


def test_wide_batch_keeps_chains_below_residency(gpu, knobs):
    # 70,000 equal files: more chain workgroups (274) than CUs (256) -> the
    # non-waiting path; with the spin limit at 0 a fused launch would time out
    knobs.set("SF_TEST_CHAIN_SPIN_LIMIT", 0)
    nfiles, nbf, bs = 70_000, 128, 64
    data, t, files = _equal_batch(gpu, nfiles, nbf, bs, 504)
    dig, _, fh = device.index_device_batch(t, files, bs)
    want = oracle.index_fixed_mt(data, bs, 8)
    assert np.array_equal(dig.cpu().numpy(), want)
    fhn = fh.cpu().numpy()
    per = want.reshape(nfiles, nbf, 20)
    for i in list(range(0, nfiles, 997)) + [nfiles - 1]:
        assert bytes(fhn[i]) == oracle.blocks_hash(per[i]), i


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
