"""GPU: the descriptor routes -- sf_index_fd_blocks / sf_index_fd_fixed hash
the regular file OPEN on the caller's descriptor, the handle its chunker just
streamed, as the reference takes the mtime, the boundaries and the bytes from
one File::open (src/index.rs:615-625).

* A file renamed over the path between chunking and hashing changes nothing:
  the rows are the oracle's over the ORIGINAL bytes (the path route,
  sf_index_file_blocks, re-opens the path and hashes the new file).
* A file written in place, appended to, truncated, or written with its mtime
  put back while the call reads it (a read hook fires between two windows)
  gives SF_EAGAIN, never a table that mixes two versions; Index.index_file
  then opens the file again and stores the new version's rows."""
import os
import time

import numpy as np
import pytest

import oracle
from syncfast_amd import _lib, host
from syncfast_amd.index import BoundaryChunker, FixedChunker, Index

pytestmark = pytest.mark.gpu

MIB = 1 << 20


@pytest.fixture
def small_stages(knobs):
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)  # ~1 MiB windows: a multi-MiB file is read in several
    yield
    _lib.set_read_hook(None)
    host.release_cache()


def _cdc_like_sizes(n, seed, mean=8192, cap=32768):
    rng = np.random.default_rng(seed)
    sizes = np.minimum(rng.geometric(1.0 / mean, size=n // 64 + 16), cap)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    return np.diff(np.concatenate([[0], cuts, [n]])).astype(np.uint32)


def _offs(sizes):
    o = np.zeros(len(sizes), np.uint64)
    o[1:] = np.cumsum(sizes.astype(np.uint64))[:-1]
    return o


def _want(data, offs, sizes):
    dig = oracle.index_blocks(np.frombuffer(data, np.uint8), offs, sizes)
    return dig, oracle.blocks_hash(dig)


def test_fd_blocks_equal_oracle_across_windows(gpu, tmp_path, small_stages):
    """Plain parity: a CDC-like list over a 5 MiB file read in ~1 MiB windows,
    and the reference KAT file's three blocks."""
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(5 * MIB + 4321, 6100).tobytes()
    p.write_bytes(data)
    sizes = _cdc_like_sizes(len(data), 6101)
    offs = _offs(sizes)
    with open(p, "rb") as f:
        st = host.file_stamp(f.fileno())
        rows, bh = host.index_fd_blocks(f.fileno(), offs, sizes, st)
    dig, wbh = _want(data, offs, sizes)
    assert np.array_equal(rows["sha1"], dig) and bh == wbh
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    k = tmp_path / "kat"
    k.write_bytes(oracle.kat_input())
    with open(k, "rb") as f:
        rows, bh = host.index_fd_blocks(f.fileno(), [0, 11579, 44347], [11579, 32768, 546])
    assert bh.hex() == "84c25d78edcdb67631639c43604cf0149564f044"


def test_fd_fixed_equals_oracle(gpu, tmp_path, small_stages):
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(3 * MIB + 999, 6110).tobytes()
    p.write_bytes(data)
    with open(p, "rb") as f:
        f.read(1000)  # the descriptor's position is not used
        rows, bh = host.index_fd_fixed(f.fileno(), 4096, host.file_stamp(f.fileno()))
        assert f.tell() == 1000
    offs, sizes, want = oracle.index_fixed(np.frombuffer(data, np.uint8), 4096)
    assert np.array_equal(rows["sha1"], want) and bh == oracle.blocks_hash(want)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)


def test_rename_over_the_path_between_chunking_and_hashing(gpu, tmp_path, small_stages):
    """Save-by-rename (the editor pattern) after the chunker read the file:
    the descriptor route hashes the file the chunker cut; the path route
    would hash the new file with the old file's boundaries."""
    p = tmp_path / "f"
    a = oracle.splitmix_bytes(3 * MIB + 77, 6120).tobytes()
    b = oracle.splitmix_bytes(3 * MIB + 77, 6121).tobytes()
    p.write_bytes(a)
    with open(p, "rb") as f:
        st = host.file_stamp(f.fileno())
        f.read()  # the chunker streams the open file
        sizes = _cdc_like_sizes(len(a), 6122)
        offs = _offs(sizes)
        tmp = tmp_path / "f.new"
        tmp.write_bytes(b)
        os.replace(tmp, p)  # another file now has the path
        rows, bh = host.index_fd_blocks(f.fileno(), offs, sizes, st)
        fixed, fbh = host.index_fd_fixed(f.fileno(), 4096, st)
    dig, wbh = _want(a, offs, sizes)
    assert np.array_equal(rows["sha1"], dig) and bh == wbh
    _o, _s, want_fixed = oracle.index_fixed(np.frombuffer(a, np.uint8), 4096)
    assert np.array_equal(fixed["sha1"], want_fixed) and fbh == oracle.blocks_hash(want_fixed)
    # the path route re-opens: B's bytes under A's boundaries (why the splice uses the descriptor)
    prow, _pbh = host.index_file_blocks(p, offs, sizes)
    assert np.array_equal(prow["sha1"], _want(b, offs, sizes)[0])
    assert not np.array_equal(prow["sha1"], dig)


def _writer(p, how, size):
    def w():
        time.sleep(0.02)  # past the filesystem clock's tick: the write's ctime differs from the stamp's
        if how == "overwrite":  # same size, different bytes in window 3
            with open(p, "r+b") as g:
                g.seek(3 * MIB + 100)
                g.write(b"\xAA" * 4096)
        elif how == "overwrite_keep_mtime":  # the writer puts the mtime back: only the ctime moves
            st = os.stat(p)
            with open(p, "r+b") as g:
                g.seek(2 * MIB + 5)
                g.write(b"\x55" * 100)
            os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
        elif how == "append":
            with open(p, "ab") as g:
                g.write(b"tail" * 1000)
        elif how == "truncate":  # a short read in a later window
            os.truncate(p, size // 2)
    return w


@pytest.mark.parametrize("how", ["overwrite", "overwrite_keep_mtime", "append", "truncate"])
@pytest.mark.parametrize("route", ["blocks", "fixed"])
def test_change_mid_call_is_eagain(gpu, tmp_path, small_stages, how, route):
    """The file changes after the first window is read: SF_EAGAIN, never a
    table that mixes the old bytes of window 0 with new bytes after it."""
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(5 * MIB + 13, 6130).tobytes()
    p.write_bytes(data)
    sizes = _cdc_like_sizes(len(data), 6131)
    offs = _offs(sizes)
    fired = []
    change = _writer(p, how, len(data))

    def hook(window):
        if window == 0 and not fired:
            fired.append(window)
            change()

    with open(p, "rb") as f:
        st = host.file_stamp(f.fileno())
        _lib.set_read_hook(hook)
        try:
            with pytest.raises(_lib.SfError) as e:
                if route == "blocks":
                    host.index_fd_blocks(f.fileno(), offs, sizes, st)
                else:
                    host.index_fd_fixed(f.fileno(), 4096, st)
        finally:
            _lib.set_read_hook(None)
    assert fired and e.value.code == _lib.SF_EAGAIN
    # and the path route, which takes its own stamp at the start, sees it too
    p.write_bytes(data)
    fired.clear()
    _lib.set_read_hook(hook)
    try:
        with pytest.raises(_lib.SfError) as e:
            host.index_file_blocks(p, offs, sizes)
    finally:
        _lib.set_read_hook(None)
    assert fired and e.value.code == _lib.SF_EAGAIN


def test_stale_stamp_before_the_call_is_eagain(gpu, tmp_path, small_stages):
    """Written between the chunker's read and the call: the caller's stamp no
    longer matches, nothing is hashed."""
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(2 * MIB, 6140).tobytes()
    p.write_bytes(data)
    with open(p, "rb") as f:
        st = host.file_stamp(f.fileno())
        sizes = _cdc_like_sizes(len(data), 6141)
        with open(p, "r+b") as g:
            g.write(b"\x00" * 10)
        with pytest.raises(_lib.SfError) as e:
            host.index_fd_blocks(f.fileno(), _offs(sizes), sizes, st)
        assert e.value.code == _lib.SF_EAGAIN


@pytest.mark.parametrize("mode", ["boundary", "fixed"])
def test_index_file_retries_a_file_written_while_indexed(gpu, tmp_path, small_stages, mode):
    """Index.index_file: the first attempt sees the file change mid-call
    (SF_EAGAIN), the second opens it again and stores the NEW version's
    rows and blocks_hash -- each row's digest is the oracle's over the file
    as it is now, none is left over from the first version."""
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(4 * MIB + 555, 6150).tobytes()
    p.write_bytes(data)
    state = {"fired": 0}

    def hook(window):
        if window == 1 and state["fired"] == 0:
            state["fired"] = 1
            time.sleep(0.02)
            with open(p, "r+b") as g:  # same size, mtime restored: only the ctime moves
                st = os.stat(p)
                g.seek(100)
                g.write(b"\x11" * 5000)
            os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))

    def chunk(f):
        n = os.fstat(f.fileno()).st_size
        f.read()
        return _cdc_like_sizes(n, 6151).tolist()

    ch = BoundaryChunker(chunk, stream=True) if mode == "boundary" else FixedChunker(4096)
    idx = Index.open_in_memory(chunker=ch)
    _lib.set_read_hook(hook)
    try:
        idx.index_file(p, "f")
    finally:
        _lib.set_read_hook(None)
    assert state["fired"] == 1
    now = p.read_bytes()
    assert now != data
    fid, _m, bh = idx.get_file("f")
    rows = idx.list_file_blocks(fid)
    offs = np.asarray([o for _h, o, _s in rows], np.uint64)
    sizes = np.asarray([s for _h, _o, s in rows], np.uint32)
    dig, wbh = _want(now, offs, sizes)
    assert [h.bytes for h, _o, _s in rows] == [bytes(d) for d in dig]
    assert bh.bytes == wbh and int(sizes.sum()) == len(now)


@pytest.mark.parametrize("mode", ["boundary", "fixed"])
def test_index_file_of_a_file_appended_on_every_window(gpu, tmp_path, small_stages, mode):
    """a file appended to after every window the library reads (a
    log) never gets through the descriptor routes; after CHANGED_RETRIES
    attempts index_file indexes the bytes of one read (the reference's single
    pass, src/index.rs:615-647) instead of failing the walk."""
    p = tmp_path / "log"
    p.write_bytes(oracle.splitmix_bytes(3 * MIB + 5, 6160).tobytes())
    seen = []

    def hook(window):
        seen.append(window)
        with open(p, "ab") as g:
            g.write(b"another line\n")

    def chunk(f):
        return _cdc_like_sizes(len(f.read()), 6161).tolist()

    ch = BoundaryChunker(chunk, stream=True) if mode == "boundary" else FixedChunker(4096)
    idx = Index.open_in_memory(chunker=ch)
    _lib.set_read_hook(hook)
    try:
        idx.index_file(p, "log")
    finally:
        _lib.set_read_hook(None)
    assert len(seen) >= 3
    fid, _m, bh = idx.get_file("log")
    rows = idx.list_file_blocks(fid)
    total = sum(s for _h, _o, s in rows)
    data = p.read_bytes()[:total]  # the bytes of the one read; the log grew only at its end since
    offs = np.asarray([o for _h, o, _s in rows], np.uint64)
    sizes = np.asarray([s for _h, _o, s in rows], np.uint32)
    dig, wbh = _want(data, offs, sizes)
    assert [h.bytes for h, _o, _s in rows] == [bytes(d) for d in dig]
    assert bh.bytes == wbh and total >= 3 * MIB + 5
