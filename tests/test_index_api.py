"""The reference library API (Index, HashDigest) on top of the C-ABI.

CPU tests mirror the reference's own unit tests (src/lib.rs:184-213) and the
SQLite row semantics of src/index.rs; GPU tests mirror the index KAT
(src/index.rs:747-793) with the reference's boundaries, and index a directory
with fixed-size blocks against the oracle."""
import datetime as dt
import hashlib
import os
from pathlib import PurePath

import numpy as np
import pytest

import oracle
from syncfast_amd import _lib
from syncfast_amd.digest import HashDigest, InvalidHashDigest
from syncfast_amd.index import BoundaryChunker, FixedChunker, Index, temp_name, untemp_name

T0 = dt.datetime(2020, 1, 2, 3, 4, 5, tzinfo=dt.timezone.utc)


# ---- src/lib.rs:184-213 ---------------------------------------------------

def test_hash_tosql():
    d = HashDigest(hashlib.sha1(b"test").digest())
    assert d.to_sql() == "a94a8fe5ccb19ba61c4c0873d391e987982fbbd3"
    assert str(d) == d.to_sql()


def test_hash_fromsql():
    d = HashDigest(hashlib.sha1(b"test").digest())
    assert HashDigest.from_sql("a94a8fe5ccb19ba61c4c0873d391e987982fbbd3") == d
    assert HashDigest.from_sql("A94A8FE5CCB19BA61C4C0873D391E987982FBBD3") == d
    with pytest.raises(InvalidHashDigest, match="wrong size"):
        HashDigest.from_sql("a94a")
    with pytest.raises(InvalidHashDigest, match="invalid character"):
        HashDigest.from_sql("zz4a8fe5ccb19ba61c4c0873d391e987982fbbd3")
    with pytest.raises(InvalidHashDigest, match="invalid character"):
        HashDigest.from_sql(" 94a8fe5ccb19ba61c4c0873d391e987982fbbd3")


def test_temp_name():
    assert temp_name("file") == PurePath(".syncfast_tmp_file")
    assert temp_name("dir/file") == PurePath("dir/.syncfast_tmp_file")
    assert untemp_name("dir/.syncfast_tmp_file") == PurePath("dir/file")


# ---- src/index.rs rows and queries (no GPU) --------------------------------

def test_schema_and_pragmas(tmp_path):
    idx = Index.open(tmp_path / "x.idx")
    assert idx.db.execute("PRAGMA application_id").fetchone()[0] == 0x51367457
    tables = {r[0] for r in idx.db.execute("SELECT name FROM sqlite_master WHERE type='table'")}
    assert tables == {"files", "blocks"}
    idx2 = Index.open(tmp_path / "x.idx")  # existing file: schema not re-created
    assert idx2.list_files() == []


def test_add_file_mtime_gate_and_blocks():
    idx = Index.open_in_memory()
    fid, up = idx.add_file("dir/name", T0)
    assert (fid, up) == (1, False)
    digs = [hashlib.sha1(bytes([i])).digest() for i in range(3)]
    idx.add_blocks(fid, [(0, 10, digs[0]), (10, 10, digs[1])])
    idx.add_block(HashDigest(digs[2]), fid, 20, 5)
    assert idx.add_file("dir/name", T0) == (1, True)
    assert idx.get_block(HashDigest(digs[1])) == (PurePath("dir/name"), 10, 10)
    assert idx.get_block(HashDigest(b"12345678901234567890")) is None
    bh = idx.compute_blocks_hash(fid)
    assert bh.bytes == hashlib.sha1(b"".join(digs)).digest()
    # size stays NULL through index_file-style inserts -> list_files reports 0
    assert idx.list_files()[0][3] == 0
    idx.set_file_size_and_compute_blocks_hash(fid, 25)
    assert idx.list_files()[0][3] == 25 and idx.list_files()[0][4] == bh
    # modified time changed -> blocks dropped, not up to date
    assert idx.add_file("dir/name", T0 + dt.timedelta(seconds=1)) == (1, False)
    assert idx.list_file_blocks(1) == []
    idx.commit()


def test_missing_blocks_and_temp_files():
    idx = Index.open_in_memory()
    tid = idx.add_temp_file("a/b")
    assert idx.list_temp_files() == [PurePath("a/.syncfast_tmp_b")]
    h = HashDigest(hashlib.sha1(b"x").digest())
    idx.add_missing_block(h, tid, 0, 1)
    assert idx.list_missing_blocks() == [h]
    assert idx.check_temp_files() == [(tid, PurePath("a/.syncfast_tmp_b"), True)]
    assert idx.get_block(h) is None  # present = 0
    idx.mark_block_present(tid, h, 0)
    assert idx.check_temp_files()[0][2] is False
    assert idx.list_block_locations(h) == [(tid, PurePath("a/.syncfast_tmp_b"), 0, 1)]
    idx.move_temp_file_into_place(tid, "a/b")
    assert idx.get_file("a/b")[0] == tid and idx.list_temp_files() == []
    idx.remove_file(tid)
    assert idx.list_files() == []


# ---- GPU: the hot path inside Index.index_file ----------------------------

def test_seekable_routes_fifo_to_stream(tmp_path):
    """Regular files take the native file routes; a FIFO is streamed from
    its one open (Index.index_file / index_path)."""
    import threading
    from syncfast_amd.index import _seekable
    reg = tmp_path / "r"
    reg.write_bytes(b"x")
    with open(reg, "rb") as f:
        assert _seekable(f)
    fifo = tmp_path / "p"
    os.mkfifo(fifo)
    th = threading.Thread(target=lambda: open(fifo, "wb").close())
    th.start()
    with open(fifo, "rb") as f:
        assert not _seekable(f)
    th.join(timeout=10)


KAT_SIZES = [11579, 32768, 546]  # src/index.rs:771,778,785


@pytest.mark.gpu
def test_reference_index_kat(gpu, tmp_path):
    """src/index.rs:747-793 with the reference's block boundaries."""
    p = tmp_path / "kat"
    p.write_bytes(oracle.kat_input())
    name = PurePath("dir/name")
    index = Index.open_in_memory(chunker=BoundaryChunker(lambda data: KAT_SIZES))
    index.index_file(p, name)
    index.commit()
    assert index.get_block(HashDigest(b"12345678901234567890")) is None
    block1 = index.get_block(HashDigest(bytes.fromhex("fb5ef7ebadd82c8085c5ff63823622bae0e263f6")))
    assert block1 == (name, 0, 11579)
    block2 = index.get_block(HashDigest(bytes.fromhex("570d8b30fcfd585e4127b561f5ecd376ff4d0101")))
    assert block2 == (name, 11579, 32768)
    block3 = index.get_block(HashDigest(bytes.fromhex("b9a8c2641af2cf8fd8f36a2456a3eaa95c029127")))
    assert block3 == (name, 44347, 546)
    assert block3[1] - block2[1] == 1 << 15  # MAX_BLOCK_SIZE
    file1 = index.get_file(name)
    assert file1[0] == 1
    assert file1[2] == HashDigest(bytes.fromhex("84c25d78edcdb67631639c43604cf0149564f044"))


@pytest.mark.gpu
@pytest.mark.parametrize("batch_bytes", [0, 1 << 30, 50_000])
def test_index_path_fixed_blocks(gpu, tmp_path, batch_bytes):
    root = tmp_path / "tree"
    (root / "sub").mkdir(parents=True)
    files = {"a.bin": 100_000, "sub/b.bin": 4096 * 3, "sub/empty": 0, "c": 1}
    for i, (n, ln) in enumerate(files.items()):
        (root / n).write_bytes(oracle.splitmix_bytes(ln, 1000 + i).tobytes())
    idx = Index.open(root / ".syncfast.idx", chunker=FixedChunker(4096))
    idx.index_path(root, batch_bytes=batch_bytes)
    idx.remove_missing_files(root)
    idx.commit()
    names = {str(f[1]) for f in idx.list_files()}
    assert names == set(files)  # the index file itself is skipped
    for i, (n, ln) in enumerate(files.items()):
        fid, _, bh = idx.get_file(n)
        data = oracle.splitmix_bytes(ln, 1000 + i)
        offs, sizes, want = oracle.index_fixed(data, 4096)
        got = idx.list_file_blocks(fid)
        assert [(g[0].bytes, g[1], g[2]) for g in got] == [(bytes(w), int(o), int(s)) for w, o, s in zip(want, offs, sizes)]
        assert bh.bytes == oracle.blocks_hash(want)
        assert idx.compute_blocks_hash(fid) == bh  # device blocks_hash == reference recomputation
    # unchanged mtimes -> nothing re-indexed; a touched file is re-indexed
    before = idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0]
    os.utime(root / "c", ns=(1, 1))
    idx.index_path(root, batch_bytes=batch_bytes)
    idx.commit()
    assert idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0] == before
    # new content: old rows deleted, new rows and blocks_hash stored; the
    # stored value is still what the reference's SELECT recomputation gives
    data = oracle.splitmix_bytes(9000, 77)
    (root / "a.bin").write_bytes(data.tobytes())
    os.utime(root / "a.bin", ns=(2, 2))
    idx.index_path(root, batch_bytes=batch_bytes)
    idx.commit()
    fid, _, bh = idx.get_file("a.bin")
    assert bh.bytes == oracle.blocks_hash(oracle.index_fixed(data, 4096)[2])
    assert idx.compute_blocks_hash(fid) == bh and len(idx.list_file_blocks(fid)) == 3
    os.remove(root / "sub" / "b.bin")
    idx.remove_missing_files(root)
    idx.commit()
    assert "sub/b.bin" not in {str(f[1]) for f in idx.list_files()}


def _toy_cdc(data: bytes):
    """A content-defined boundary function for the tests (a stand-in for the
    reference's ZPAQ): cut after every byte 0x00 that follows 7 or more bytes
    since the last cut, or at 2000 bytes."""
    sizes, start = [], 0
    for i, c in enumerate(data):
        if (c == 0 and i + 1 - start >= 8) or i + 1 - start == 2000:
            sizes.append(i + 1 - start)
            start = i + 1
    if start < len(data):
        sizes.append(len(data) - start)
    return sizes


@pytest.mark.gpu
@pytest.mark.parametrize("batch_bytes", [0, 1 << 30, 30_000])
def test_index_path_boundary_chunker_batched(gpu, tmp_path, batch_bytes):
    """index_path in the default (content-defined) mode: files cut by the host
    chunker, their blocks hashed per batch of files in one device call; the
    rows, the stored blocks_hash and its SELECT recomputation equal the
    per-file path and the oracle."""
    root = tmp_path / "tree"
    (root / "sub").mkdir(parents=True)
    files = {"a.bin": 100_000, "sub/b.bin": 12_345, "sub/empty": 0, "c": 1, "d": 7_777}
    for i, (n, ln) in enumerate(files.items()):
        (root / n).write_bytes(oracle.splitmix_bytes(ln, 3000 + i).tobytes())
    idx = Index.open(root / ".syncfast.idx", chunker=BoundaryChunker(_toy_cdc))
    idx.index_path(root, batch_bytes=batch_bytes)
    idx.commit()
    assert {str(f[1]) for f in idx.list_files()} == set(files)
    for i, (n, ln) in enumerate(files.items()):
        fid, _, bh = idx.get_file(n)
        data = oracle.splitmix_bytes(ln, 3000 + i).tobytes()
        sizes = _toy_cdc(data)
        offs = [sum(sizes[:k]) for k in range(len(sizes))]
        want = oracle.py_index_blocks(data, offs, sizes)
        got = idx.list_file_blocks(fid)
        assert [(g[0].bytes, g[1], g[2]) for g in got] == list(zip(want, offs, sizes)), n
        assert bh.bytes == oracle.py_blocks_hash(want)
        assert idx.compute_blocks_hash(fid) == bh
    # unchanged mtimes: nothing re-indexed
    before = idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0]
    idx.index_path(root, batch_bytes=batch_bytes)
    idx.commit()
    assert idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0] == before


@pytest.mark.gpu
@pytest.mark.parametrize("via", ["index_file", "index_path"])
def test_fifo_is_streamed(gpu, tmp_path, via):
    """The reference's index_file streams any path File::open accepts; a FIFO
    (no size, no seek) gets the same rows as a regular file with its bytes."""
    import threading
    root = tmp_path / "tree"
    root.mkdir()
    fifo = root / "pipe"
    os.mkfifo(fifo)
    data = oracle.splitmix_bytes(3 * 4096 + 1234, 77)

    def writer():
        with open(fifo, "wb") as w:
            w.write(data.tobytes())

    th = threading.Thread(target=writer)
    th.start()
    idx = Index.open_in_memory(chunker=FixedChunker(4096))
    if via == "index_file":
        idx.index_file(fifo, PurePath("pipe"))
    else:
        idx.index_path(root)
    th.join(timeout=30)
    idx.commit()
    fid, _, bh = idx.get_file("pipe")
    offs, sizes, want = oracle.index_fixed(data, 4096)
    got = idx.list_file_blocks(fid)
    assert [(g[0].bytes, g[1], g[2]) for g in got] == [(bytes(w), int(o), int(s)) for w, o, s in zip(want, offs, sizes)]
    assert bh.bytes == oracle.blocks_hash(want)


@pytest.mark.gpu
def test_boundary_chunker_random(gpu):
    rng = np.random.default_rng(5)
    data = oracle.splitmix_bytes(200_000, 77).tobytes()
    cuts = sorted(set(int(x) for x in rng.integers(1, len(data), 40)))
    sizes = np.diff([0] + cuts + [len(data)]).tolist()
    from syncfast_amd.index import signatures_of_bytes
    rows = signatures_of_bytes(data, BoundaryChunker(lambda d: sizes))
    assert [r[2] for r in rows] == oracle.py_index_blocks(data, [r[0] for r in rows], sizes)


def test_walk_visits_entries_in_readdir_order(tmp_path):
    # src/index.rs:698 iterates read_dir() as the filesystem yields it (no
    # sort); os.listdir is the same readdir(3) order, so file_ids follow it
    root = tmp_path / "w"
    (root / "sub").mkdir(parents=True)
    for n in ["zeta", "alpha", "Mid", "b10", "b9", ".hidden"]:
        (root / n).write_bytes(b"x")
        (root / "sub" / n).write_bytes(b"y")
    (root / ".syncfast.idx").write_bytes(b"")
    todo = []
    Index.open_in_memory()._index_path_rec(root, PurePath(""), todo)

    def expect(rel):
        out = []
        for e in os.listdir(root / rel):
            if e == ".syncfast.idx":
                continue
            if (root / rel / e).is_dir():
                out += expect(rel / e)
            else:
                out.append(rel / e)
        return out

    assert [str(r) for _p, r in todo] == [str(r) for r in expect(PurePath(""))]
    assert len(todo) == 12


@pytest.mark.gpu
def test_mtime_gate_at_nanosecond_resolution(gpu, tmp_path):
    # src/index.rs:183 compares DateTime values: a file whose mtime moved by
    # 1 us is re-indexed; one rewritten with its exact old mtime is not (the
    # reference's gate cannot see that either)
    root = tmp_path / "t"
    root.mkdir()
    p = root / "f"
    p.write_bytes(oracle.splitmix_bytes(50_000, 1).tobytes())
    t0 = 1_700_000_000_123_456_789
    os.utime(p, ns=(t0, t0))
    idx = Index.open_in_memory(chunker=FixedChunker(4096))
    idx.index_path(root)
    fid, m, bh1 = idx.get_file("f")
    assert m.ns == os.stat(p).st_mtime_ns
    p.write_bytes(oracle.splitmix_bytes(50_000, 2).tobytes())
    os.utime(p, ns=(t0, m.ns))  # same stored instant
    idx.index_path(root)
    assert idx.get_file("f")[2] == bh1  # gate: up to date
    os.utime(p, ns=(t0, m.ns + 1000))
    idx.index_path(root)
    bh2 = idx.get_file("f")[2]
    want = oracle.index_fixed(oracle.splitmix_bytes(50_000, 2), 4096)[2]
    assert bh2.bytes == oracle.blocks_hash(want) != bh1.bytes


def test_walk_of_a_file_names_it_empty(tmp_path):
    # index_path(file): rel = Path::new("") (src/index.rs:686, 706-713), so the
    # file is indexed under the empty name, not "."
    p = tmp_path / "single"
    p.write_bytes(b"x")
    todo = []
    Index.open_in_memory()._index_path_rec(p, PurePath(""), todo)
    assert len(todo) == 1 and todo[0][1] == ""
    from syncfast_amd.index import _name_str
    assert _name_str(todo[0][1]) == ""


# ---- the drop-in's block semantics: rows read back by (offset, size) -------

def _reference_read_block(path, offset, chunker_fn):
    """What the reference's read_block does (src/sync/fs.rs:26-40): open,
    seek to `offset`, run a FRESH chunker and return its first chunk (here
    with the test's stand-in boundary function)."""
    with open(path, "rb") as f:
        f.seek(offset)
        rest = f.read()
    sizes = chunker_fn(rest)
    if not sizes:
        raise ValueError("No such chunk in file")
    return rest[:sizes[0]]


def _oracle_device_calls(monkeypatch):
    """CPU stand-ins for the two explicit-list entry points (the GPU tests
    run the real ones): the oracle's digests, in the SIG_DTYPE row layout."""
    from syncfast_amd import host

    def rows_of(raw, offs, sizes):
        offs = np.asarray(offs, np.uint64)
        sizes = np.asarray(sizes, np.uint32)
        rows = np.zeros(offs.size, host.SIG_DTYPE)
        rows["offset"], rows["size"] = offs, sizes
        dig = oracle.index_blocks(np.frombuffer(raw, np.uint8), offs, sizes) if offs.size else np.zeros((0, 20), np.uint8)
        rows["sha1"] = dig
        return rows, oracle.blocks_hash(dig)

    monkeypatch.setattr(host, "index_buffer_blocks", lambda data, offs, sizes: rows_of(bytes(data), offs, sizes))
    monkeypatch.setattr(host, "index_file_blocks",
                        lambda path, offs, sizes: rows_of(open(path, "rb").read(), offs, sizes))
    monkeypatch.setattr(host, "index_fd_blocks",
                        lambda fd, offs, sizes, stamp=None: rows_of(_pread_all(fd), offs, sizes))

    def fds_rows(fds, lists, stamps=None, stage_bytes=0):
        parts, first, hashes = [], [0], []
        for fd, (offs, sizes) in zip(fds, lists):
            rows, bh = rows_of(_pread_all(fd), offs, sizes)
            parts.append(rows)
            first.append(first[-1] + rows.shape[0])
            hashes.append(np.frombuffer(bh, np.uint8))
        rows = np.concatenate(parts) if parts else np.zeros(0, host.SIG_DTYPE)
        return (rows, np.asarray(first, np.uint64), np.asarray(hashes, np.uint8).reshape(-1, 20),
                np.zeros(len(fds), np.int32))

    monkeypatch.setattr(host, "index_fds_blocks", fds_rows)


def _pread_all(fd):
    """The whole file open on fd, read with pread (the descriptor's position
    is the chunker's, as in the library)."""
    size = os.fstat(fd).st_size
    return os.pread(fd, size, 0) if size else b""


def _tree(root, seed):
    (root / "sub").mkdir(parents=True)
    files = {"a.bin": 50_000, "sub/b.bin": 12_345, "sub/empty": 0, "c": 1, "d": 7_777}
    for i, (n, ln) in enumerate(files.items()):
        (root / n).write_bytes(oracle.splitmix_bytes(ln, seed + i).tobytes())
    return files


def _stream_toy_cdc(f):
    return _toy_cdc(f.read())


def _check_read_back(idx, root, files, chunker_fn):
    from syncfast_amd.index import read_block
    for n in files:
        fid, _, bh = idx.get_file(n)
        data = (root / n).read_bytes()
        rows = idx.list_file_blocks(fid)
        # the rows tile the file in offset order, and every block's bytes,
        # read back by (offset, size), hash to the stored digest
        assert b"".join(read_block(root / n, o, s) for _h, o, s in rows) == data
        for h, o, s in rows:
            assert hashlib.sha1(read_block(root / n, o, s)).digest() == h.bytes
            if chunker_fn is not None:  # the reference's re-chunking reader gets the same bytes
                assert _reference_read_block(root / n, o, chunker_fn) == read_block(root / n, o, s)
        assert idx.compute_blocks_hash(fid) == bh


@pytest.mark.parametrize("stream", [False, True])
def test_boundary_rows_read_back_by_offset_size(tmp_path, monkeypatch, stream):
    """Index a tree with a BoundaryChunker (the reference's mode; the device
    calls replaced by the oracle here, the GPU test below runs them), then
    read every block back by its row's (offset, size) and re-hash it; the
    reference's own reader (re-chunking from the offset, src/sync/fs.rs:
    26-40) returns the same bytes for these rows, because a chunker's state
    resets at every boundary."""
    _oracle_device_calls(monkeypatch)
    root = tmp_path / "tree"
    files = _tree(root, 4000)
    ch = BoundaryChunker(_stream_toy_cdc, stream=True) if stream else BoundaryChunker(_toy_cdc)
    idx = Index.open(root / ".syncfast.idx", chunker=ch)
    idx.index_path(root)
    idx.commit()
    _check_read_back(idx, root, files, _toy_cdc)


def test_fixed_rows_need_the_offset_size_reader(tmp_path, monkeypatch):
    """Why fixed tiling is opt-in: for FixedChunker rows the reference's
    re-chunking reader returns other bytes than the row names (here with the
    stand-in chunker), so a drop-in that indexes with fixed tiling must read
    blocks by (offset, size) -- syncfast_amd.index.read_block, INTEGRATION.md
    "Fixed tiling"."""
    from syncfast_amd import host
    from syncfast_amd.index import read_block
    root = tmp_path / "t"
    root.mkdir()
    data = oracle.splitmix_bytes(20_000, 4100).tobytes()
    (root / "f").write_bytes(data)

    def fake_index_fd_fixed(fd, bs, stamp=None):
        offs, sizes, dig = oracle.index_fixed(np.frombuffer(_pread_all(fd), np.uint8), bs)
        rows = np.zeros(len(offs), host.SIG_DTYPE)
        rows["offset"], rows["size"], rows["sha1"] = offs, sizes, dig
        return rows, oracle.blocks_hash(dig)

    monkeypatch.setattr(host, "index_fd_fixed", fake_index_fd_fixed)
    idx = Index.open_in_memory(chunker=FixedChunker(4096))
    idx.index_file(root / "f", "f")
    rows = idx.list_file_blocks(idx.get_file("f")[0])
    assert all(hashlib.sha1(read_block(root / "f", o, s)).digest() == h.bytes for h, o, s in rows)
    assert any(_reference_read_block(root / "f", o, _toy_cdc) != read_block(root / "f", o, s) for _h, o, s in rows)


def test_index_without_a_chunker_refuses_to_index(tmp_path):
    """No silent default: an Index opened without a chunker answers queries
    but index_file / index_path raise, naming the two modes."""
    from syncfast_amd.index import SyncfastError
    p = tmp_path / "f"
    p.write_bytes(b"x" * 100)
    idx = Index.open_in_memory()
    with pytest.raises(SyncfastError, match="BoundaryChunker"):
        idx.index_file(p, "f")
    with pytest.raises(SyncfastError, match="FixedChunker"):
        idx.index_path(tmp_path)
    assert idx.list_files() == []


def test_read_block_short_file(tmp_path):
    from syncfast_amd.index import SyncfastError, read_block
    p = tmp_path / "f"
    p.write_bytes(b"abcdef")
    assert read_block(p, 2, 3) == b"cde"
    with pytest.raises(SyncfastError, match="No such chunk"):
        read_block(p, 4, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", [False, True])
def test_boundary_rows_read_back_on_the_gpu(gpu, tmp_path, stream):
    """The same through the real device calls: sf_index_fd_blocks (the
    chunker streamed the open file, the library re-reads that descriptor by
    windows) and
    sf_index_buffer_blocks (the bytes in memory)."""
    root = tmp_path / "tree"
    files = _tree(root, 4200)
    ch = BoundaryChunker(_stream_toy_cdc, stream=True) if stream else BoundaryChunker(_toy_cdc)
    idx = Index.open(root / ".syncfast.idx", chunker=ch)
    idx.index_path(root)
    idx.commit()
    _check_read_back(idx, root, files, _toy_cdc)


@pytest.mark.parametrize("threads", [1, 3])
@pytest.mark.parametrize("batch_bytes", [0, 1 << 30, 20_000])
def test_index_path_stream_chunker_many_files(tmp_path, monkeypatch, threads, batch_bytes):
    """index_path in the reference's default mode (BoundaryChunker(stream=True)):
    files cut on a thread pool, batches through sf_index_fds_blocks (the oracle
    stands in for the device here); rows, blocks_hash and file_ids (walk order)
    equal the file-by-file path's."""
    _oracle_device_calls(monkeypatch)
    root = tmp_path / "tree"
    files = _tree(root, 4300)
    for k in range(20):
        (root / f"x{k:02d}").write_bytes(oracle.splitmix_bytes(3000 * k, 4400 + k).tobytes())
    idx = Index.open(root / ".syncfast.idx", chunker=BoundaryChunker(_stream_toy_cdc, stream=True))
    idx.index_path(root, batch_bytes=batch_bytes, chunk_threads=threads)
    idx.commit()
    ref = Index.open_in_memory(chunker=BoundaryChunker(_stream_toy_cdc, stream=True))
    ref.index_path(root, batch_bytes=0)
    ref.commit()
    assert idx.db.execute("SELECT file_id, name FROM files ORDER BY file_id").fetchall() == \
        ref.db.execute("SELECT file_id, name FROM files ORDER BY file_id").fetchall()
    q = "SELECT file_id, hash, offset, size, present FROM blocks ORDER BY rowid"
    assert idx.db.execute(q).fetchall() == ref.db.execute(q).fetchall()
    q = "SELECT file_id, blocks_hash FROM files ORDER BY file_id"
    assert idx.db.execute(q).fetchall() == ref.db.execute(q).fetchall()
    _check_read_back(idx, root, files, _toy_cdc)
    _check_read_back(idx, root, [f"x{k:02d}" for k in range(20)], None)
    before = idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0]
    idx.index_path(root, batch_bytes=batch_bytes, chunk_threads=threads)  # mtimes unchanged: nothing again
    assert idx.db.execute("SELECT COUNT(*) FROM blocks").fetchone()[0] == before


def test_index_path_stream_chunker_file_changed_is_reindexed(tmp_path, monkeypatch):
    """A file the many-file call reports SF_EAGAIN for (written while it was
    read) is indexed again in its place; its rows are the new bytes'."""
    from syncfast_amd import host
    _oracle_device_calls(monkeypatch)
    root = tmp_path / "tree"
    files = _tree(root, 4500)
    real = host.index_fds_blocks
    victim = root / "sub" / "b.bin"

    def fake(fds, lists, stamps=None, stage_bytes=0):
        rows, first, hashes, status = real(fds, lists, stamps, stage_bytes)
        for k, fd in enumerate(fds):
            if os.fstat(fd).st_ino == os.stat(victim).st_ino and not fake.done:
                fake.done = True
                status[k] = _lib.SF_EAGAIN
                hashes[k] = 0
                victim.write_bytes(oracle.splitmix_bytes(22_222, 4599).tobytes())
        return rows, first, hashes, status
    fake.done = False
    monkeypatch.setattr(host, "index_fds_blocks", fake)
    idx = Index.open_in_memory(chunker=BoundaryChunker(_stream_toy_cdc, stream=True))
    idx.index_path(root)
    assert fake.done
    _check_read_back(idx, root, files, _toy_cdc)
    fid = idx.get_file("sub/b.bin")[0]
    assert sum(s for _h, _o, s in idx.list_file_blocks(fid)) == 22_222


@pytest.mark.parametrize("mode", ["boundary", "fixed"])
def test_index_file_that_keeps_changing_falls_back_to_one_pass(tmp_path, monkeypatch, mode):
    """a file that changes on every attempt (a log being appended
    to) is not an error: after CHANGED_RETRIES attempts index_file hashes the
    bytes of ONE read, as the reference's single pass does
    (src/index.rs:615-647), and index_path goes on."""
    from syncfast_amd import host
    from syncfast_amd.index import CHANGED_RETRIES
    _oracle_device_calls(monkeypatch)
    p = tmp_path / "log"
    p.write_bytes(oracle.splitmix_bytes(30_000, 4600).tobytes())
    calls = {"n": 0}

    def always_changed(*_a, **_k):
        calls["n"] += 1
        with open(p, "ab") as g:
            g.write(b"line\n")
        raise _lib.SfError(_lib.SF_EAGAIN, "changed")

    monkeypatch.setattr(host, "index_fd_blocks", always_changed)
    monkeypatch.setattr(host, "index_fd_fixed", always_changed)

    def buffer_rows(data, bs):
        offs, sizes, dig = oracle.index_fixed(np.frombuffer(bytes(data), np.uint8), bs)
        rows = np.zeros(len(offs), host.SIG_DTYPE)
        rows["offset"], rows["size"], rows["sha1"] = offs, sizes, dig
        return rows

    monkeypatch.setattr(host, "index_buffer", buffer_rows)
    ch = BoundaryChunker(_stream_toy_cdc, stream=True) if mode == "boundary" else FixedChunker(4096)
    idx = Index.open_in_memory(chunker=ch)
    idx.index_file(p, "log")
    assert calls["n"] == CHANGED_RETRIES
    data = p.read_bytes()
    fid, _m, bh = idx.get_file("log")
    rows = idx.list_file_blocks(fid)
    assert b"".join(data[o:o + s] for _h, o, s in rows) == data
    assert all(hashlib.sha1(data[o:o + s]).digest() == h.bytes for h, o, s in rows)
    assert idx.compute_blocks_hash(fid) == bh


def test_index_path_stream_chunker_property(tmp_path, monkeypatch):
    """Property (hypothesis, seeded): for random trees (nested directories,
    files of 0 B .. 40 KB), batch sizes and chunker thread counts, the
    default mode's many-file pipeline (the oracle standing in for the device
    call) stores exactly what the file-by-file path stores: the same files
    in the same order, the same rows in the same order, the same
    blocks_hash."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    _oracle_device_calls(monkeypatch)
    counter = [0]

    @settings(max_examples=15, deadline=None, derandomize=True,
              suppress_health_check=[HealthCheck.function_scoped_fixture])
    @given(sizes=st.lists(st.integers(0, 40_000), min_size=1, max_size=25),
           depth=st.lists(st.integers(0, 2), min_size=25, max_size=25),
           batch=st.sampled_from([1, 5_000, 60_000, 1 << 30]), threads=st.integers(1, 4))
    def check(sizes, depth, batch, threads):
        counter[0] += 1
        root = tmp_path / f"t{counter[0]}"
        for k, n in enumerate(sizes):
            d = root.joinpath(*[f"d{j}" for j in range(depth[k])])
            d.mkdir(parents=True, exist_ok=True)
            (d / f"f{k:02d}").write_bytes(oracle.splitmix_bytes(n, 9500 + k).tobytes())
        got = Index.open_in_memory(chunker=BoundaryChunker(_stream_toy_cdc, stream=True))
        got.index_path(root, batch_bytes=batch, chunk_threads=threads)
        ref = Index.open_in_memory(chunker=BoundaryChunker(_stream_toy_cdc, stream=True))
        ref.index_path(root, batch_bytes=0)
        for q in ("SELECT file_id, name, blocks_hash FROM files ORDER BY file_id",
                  "SELECT file_id, hash, offset, size, present FROM blocks ORDER BY rowid"):
            assert got.db.execute(q).fetchall() == ref.db.execute(q).fetchall()

    check()
    assert counter[0] >= 10  # the examples ran


def _standin_ops_lib():
    import ctypes
    import subprocess as _sp
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "examples", "build", "libzpaq_standin.so")
    if not os.path.exists(so):
        _sp.check_call(["make", "-s", "-C", os.path.join(root, "examples"), "build/libzpaq_standin.so"])
    lib = ctypes.CDLL(so)
    lib.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    lib.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    lib.sf_zpaq_standin_ops_free.argtypes = [ctypes.c_void_p]
    return lib


def test_native_chunker_matches_the_python_chunker(tmp_path, monkeypatch):
    """Index with a NativeChunker (the stand-in's sf_chunker_ops): index_file
    (sf_index_fd_cut: the library cuts on its threads -- really, sf_cut_fd is
    host-only -- with the oracle standing in for the device's hashes),
    index_path (one thread per file, batches through sf_index_fds_blocks),
    and the one-pass fallback (the ops driven from Python over one read's
    bytes) all store what a Python BoundaryChunker with the oracle's
    one-stream stand-in stores."""
    from syncfast_amd import host
    from syncfast_amd.index import NativeChunker
    _oracle_device_calls(monkeypatch)

    def fd_cut(fd, ops, threads=0, stamp=None):
        offs, sizes = host.cut_fd(fd, ops, threads, stamp)
        raw = _pread_all(fd)
        rows = np.zeros(offs.size, host.SIG_DTYPE)
        rows["offset"], rows["size"] = offs, sizes
        dig = oracle.index_blocks(np.frombuffer(raw, np.uint8), offs, sizes) if offs.size else np.zeros((0, 20), np.uint8)
        rows["sha1"] = dig
        return rows, oracle.blocks_hash(dig)

    monkeypatch.setattr(host, "index_fd_cut", fd_cut)
    lib = _standin_ops_lib()
    ops = lib.sf_zpaq_standin_ops(13, 32768)
    try:
        root = tmp_path / "tree"
        (root / "sub").mkdir(parents=True)
        for k, n in enumerate([0, 1, 5000, 70_000, (9 << 20) + 3, 300_000]):
            (root / ("sub" if k % 2 else ".") / f"f{k}").write_bytes(oracle.splitmix_bytes(n, 9700 + k).tobytes())
        ref = Index.open_in_memory(chunker=BoundaryChunker(lambda raw: oracle.zpaq_standin_sizes(raw).tolist()))
        ref.index_path(root, batch_bytes=0)
        q_files = "SELECT file_id, name, blocks_hash FROM files ORDER BY file_id"
        q_blocks = "SELECT file_id, hash, offset, size, present FROM blocks ORDER BY file_id, offset"
        for batch in (0, 1 << 30):  # index_file per file (fused route), then the batched walk
            got = Index.open_in_memory(chunker=NativeChunker(ops, threads=4))
            got.index_path(root, batch_bytes=batch)
            assert got.db.execute(q_files).fetchall() == ref.db.execute(q_files).fetchall(), batch
            assert got.db.execute(q_blocks).fetchall() == ref.db.execute(q_blocks).fetchall(), batch
        # the one-pass fallback cuts one read's bytes through the ops from Python
        nc = NativeChunker(ops)
        data = oracle.splitmix_bytes(200_000, 9800)
        import io
        assert nc.fn(io.BytesIO(data.tobytes())) == oracle.zpaq_standin_sizes(data).tolist()
    finally:
        lib.sf_zpaq_standin_ops_free(ops)


@pytest.mark.timeout(120)
def test_index_path_large_files_and_fifo_keep_walk_order(tmp_path, monkeypatch):
    """Index.index_path with a NativeChunker: files of at least
    large_file_bytes are cut on the chunker's threads and hashed from one read
    (sf_index_fd_cut; the oracle stands in for the device) in their walk
    position, a FIFO is streamed from its own open, and both wait for every
    batch before them to be stored: the files and the blocks, in rowid order,
    are exactly what the file-by-file walk stores (get_block returns the first
    row for a digest, src/index.rs:80-90, so the order is observable)."""
    import threading
    from syncfast_amd import host
    from syncfast_amd.index import NativeChunker
    _oracle_device_calls(monkeypatch)
    calls = []

    def fd_cut(fd, ops, threads=0, stamp=None):
        calls.append(os.fstat(fd).st_size)
        offs, sizes = host.cut_fd(fd, ops, threads, stamp)
        raw = _pread_all(fd)
        rows = np.zeros(offs.size, host.SIG_DTYPE)
        rows["offset"], rows["size"] = offs, sizes
        dig = oracle.index_blocks(np.frombuffer(raw, np.uint8), offs, sizes) if offs.size else np.zeros((0, 20), np.uint8)
        rows["sha1"] = dig
        return rows, oracle.blocks_hash(dig)

    monkeypatch.setattr(host, "index_fd_cut", fd_cut)
    lib = _standin_ops_lib()
    ops = lib.sf_zpaq_standin_ops(13, 32768)
    root = tmp_path / "tree"
    (root / "sub").mkdir(parents=True)
    sizes = [40_000, 3_000, (2 << 20) + 17, 90_000, 0, 55_555, (1 << 20), 12_000, 70_000, 1, 33_000, 64_000]
    for k, n in enumerate(sizes):
        # the same bytes twice (k and k + 6): duplicate digests across files
        (root / ("sub" if k % 3 == 0 else ".") / f"f{k:02d}").write_bytes(
            oracle.splitmix_bytes(n, 9900 + k % 6).tobytes())
    fifo = root / "pipe"
    os.mkfifo(fifo)
    fdata = oracle.splitmix_bytes(100_000, 9950).tobytes()

    second = threading.Event()

    def writer():  # one writer per reader's open (a writer reopening at once could meet the last reader)
        for k in range(2):
            if k:
                second.wait(60)
            with open(fifo, "wb") as w:
                w.write(fdata)

    th = threading.Thread(target=writer, daemon=True)
    th.start()
    try:
        ref = Index.open_in_memory(chunker=NativeChunker(ops, threads=4))
        ref.index_path(root, batch_bytes=0)
        second.set()
        calls.clear()
        got = Index.open_in_memory(chunker=NativeChunker(ops, threads=4))
        got.index_path(root, batch_bytes=100_000, chunk_threads=3, large_file_bytes=1 << 20)
        th.join(timeout=30)
        assert sorted(calls) == [1 << 20, (2 << 20) + 17]  # the two large files, nothing else
        for q in ("SELECT file_id, name, blocks_hash FROM files ORDER BY file_id",
                  "SELECT file_id, hash, offset, size, present FROM blocks ORDER BY rowid"):
            assert got.db.execute(q).fetchall() == ref.db.execute(q).fetchall(), q
        assert got.get_file("pipe") is not None
    finally:
        lib.sf_zpaq_standin_ops_free(ops)
