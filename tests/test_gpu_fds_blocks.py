"""GPU: sf_index_fds_blocks -- the reference's default mode over many files as
ONE pipeline (index_path -> index_file per file, src/index.rs:685-715 ->
610-659): every file cut by the caller's chunker on its own open descriptor,
read again with pread into packed pinned stages, one sort + one explicit-list
kernel launch per stage.

* A tree of 0-B, 1-B, 32 KiB-capped, CDC-like and larger-than-a-stage files:
  every row and every blocks_hash equal to the oracle's, at several stage
  sizes, with and without stamps.
* A file rewritten while the call reads it (a read hook between stages) is
  named by bad_file with SF_EAGAIN; every other file's rows stay equal to the
  oracle's.  A stale stamp, a list past the end, offsets going backwards and
  a pipe fail for their file alone."""
import os
import time

import numpy as np
import pytest

import oracle
from syncfast_amd import _lib, host

pytestmark = pytest.mark.gpu

KIB, MIB = 1 << 10, 1 << 20


def _cdc_like_sizes(n, seed, mean=8192, cap=32768):
    if n == 0:
        return np.zeros(0, np.uint32)
    rng = np.random.default_rng(seed)
    sizes = np.minimum(rng.geometric(1.0 / mean, size=n // 64 + 16), cap)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    return np.diff(np.concatenate([[0], cuts, [n]])).astype(np.uint32)


def _offs(sizes):
    o = np.zeros(len(sizes), np.uint64)
    if len(sizes):
        o[1:] = np.cumsum(sizes.astype(np.uint64))[:-1]
    return o


def _tree(tmp_path, lens, seed):
    files = []
    for k, n in enumerate(lens):
        p = tmp_path / f"f{k:04d}"
        data = oracle.splitmix_bytes(n, seed + k).tobytes() if n else b""
        p.write_bytes(data)
        sizes = _cdc_like_sizes(n, seed + 1000 + k)
        files.append((p, data, _offs(sizes), sizes))
    return files


def _check(files, rows, first, hashes, status, skip=()):
    for k, (_p, data, offs, sizes) in enumerate(files):
        if k in skip:
            continue
        assert status[k] == 0, k
        mine = rows[int(first[k]):int(first[k + 1])]
        assert mine.shape[0] == len(sizes)
        dig = oracle.index_blocks(np.frombuffer(data, np.uint8), offs, sizes) if len(sizes) else \
            np.zeros((0, 20), np.uint8)
        assert np.array_equal(mine["sha1"], dig), k
        assert np.array_equal(mine["offset"], offs) and np.array_equal(mine["size"], sizes), k
        assert bytes(hashes[k]) == oracle.blocks_hash(dig), k


def _run(files, stamps=True, stage_bytes=0):
    fs = [open(p, "rb") for p, *_ in files]
    try:
        st = [host.file_stamp(f.fileno()) for f in fs] if stamps else None
        return host.index_fds_blocks([f.fileno() for f in fs], [(o, s) for _p, _d, o, s in files], st,
                                     stage_bytes=stage_bytes)
    finally:
        for f in fs:
            f.close()


@pytest.mark.parametrize("stage_bytes", [0, 1 * MIB, 300 * KIB])
def test_tree_equals_oracle(gpu, tmp_path, stage_bytes):
    """0-B, 1-B, one capped block, CDC-like files of 1 B .. 3 MiB and a file
    larger than the stage (several windows, blocks_hash streamed over them)."""
    lens = [0, 1, 32768, 32769, 0, 5, 100_000, 3 * MIB + 17, 64, 200 * KIB, 1, 0, 777_777, 16, 2 * MIB]
    files = _tree(tmp_path, lens, 7000)
    rows, first, hashes, status = _run(files, stage_bytes=stage_bytes)
    assert int(first[-1]) == sum(len(s) for *_r, s in files)
    _check(files, rows, first, hashes, status)
    assert bytes(hashes[0]).hex() == "da39a3ee5e6b4b0d3255bfef95601890afd80709"  # no blocks: SHA1("")


def test_many_small_files_and_reference_kat(gpu, tmp_path):
    """600 files of 0-200 KiB in several stages, and the reference KAT file's
    three blocks among them (src/index.rs:747-793)."""
    rng = np.random.default_rng(7100)
    lens = [int(x) for x in rng.integers(0, 200 * KIB, 600)]
    files = _tree(tmp_path, lens, 7100)
    k = tmp_path / "kat"
    k.write_bytes(oracle.kat_input())
    files.insert(300, (k, oracle.kat_input(), np.array([0, 11579, 44347], np.uint64),
                       np.array([11579, 32768, 546], np.uint32)))
    rows, first, hashes, status = _run(files, stage_bytes=8 * MIB)
    _check(files, rows, first, hashes, status)
    assert bytes(hashes[300]).hex() == "84c25d78edcdb67631639c43604cf0149564f044"


def test_more_blocks_than_a_stage_holds(gpu, tmp_path):
    """A file of 4.5 M tiny blocks (1-3 B): more blocks than one stage takes
    (2^22), so its window splits by block count, not bytes, and its
    blocks_hash is streamed over the pieces; the files around it stay exact."""
    rng = np.random.default_rng(7150)
    tiny = rng.integers(1, 4, 4_500_000).astype(np.uint32)
    n = int(tiny.sum())
    p = tmp_path / "tiny"
    data = oracle.splitmix_bytes(n, 7151).tobytes()
    p.write_bytes(data)
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    files = (_tree(tmp_path / "a", [1 * MIB + 3], 7152) + [(p, data, _offs(tiny), tiny)]
             + _tree(tmp_path / "b", [200 * KIB, 0, 9], 7160))
    rows, first, hashes, status = _run(files)
    _check(files, rows, first, hashes, status)


def test_odd_lists(gpu, tmp_path):
    """Lists a chunker would not make but the contract allows: gaps, overlaps,
    empty blocks, blocks not covering the file, a 4 KiB fixed-like list."""
    data = oracle.splitmix_bytes(300_000, 7200).tobytes()
    p = tmp_path / "a"
    p.write_bytes(data)
    lists = [
        (np.array([0, 0, 10, 10, 5000, 299_999], np.uint64), np.array([0, 100, 0, 50_000, 7, 1], np.uint32)),
        (np.arange(0, 299_000, 4096, dtype=np.uint64), np.full(73, 4096, np.uint32)),
        (np.array([123_456], np.uint64), np.array([176_544], np.uint32)),
    ]
    files = [(p, data, o, s) for o, s in lists]
    rows, first, hashes, status = _run(files, stage_bytes=64 * KIB)
    _check(files, rows, first, hashes, status)


def test_rewritten_mid_call_is_named_and_others_exact(gpu, tmp_path):
    """A file in a later stage is rewritten (same size, mtime restored: only
    the ctime moves) right after stage 0 is read: SF_EAGAIN for that file,
    bad_file = its index; every other file equals the oracle."""
    lens = [400 * KIB] * 12
    files = _tree(tmp_path, lens, 7300)
    victim = 9
    fired = []

    def hook(stage):
        if stage == 0 and not fired:
            fired.append(stage)
            time.sleep(0.02)  # past the filesystem clock's tick
            p = files[victim][0]
            st = os.stat(p)
            with open(p, "r+b") as g:
                g.seek(1000)
                g.write(b"\x5A" * 3000)
            os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))

    _lib.set_read_hook(hook)
    try:
        rows, first, hashes, status = _run(files, stage_bytes=1 * MIB)
    finally:
        _lib.set_read_hook(None)
    assert fired
    assert status[victim] == _lib.SF_EAGAIN and bytes(hashes[victim]) == bytes(20)
    _check(files, rows, first, hashes, status, skip=(victim,))
    # the raw call names it
    fs = [open(p, "rb") for p, *_ in files]
    try:
        import ctypes
        n = len(files)
        bad = ctypes.c_uint32(99)
        offs = [np.ascontiguousarray(o) for _p, _d, o, _s in files]
        szs = [np.ascontiguousarray(s) for *_r, s in files]
        po = (ctypes.c_void_p * n)(*[o.ctypes.data for o in offs])
        pz = (ctypes.c_void_p * n)(*[z.ctypes.data for z in szs])
        nb = np.array([o.size for o in offs], np.uint64)
        stamps = (_lib.FileStamp * n)(*[host.file_stamp(f.fileno()) for f in fs])
        with open(files[4][0], "r+b") as g:  # stale stamp for file 4
            time.sleep(0.02)
            g.write(b"\x01")
        total = int(nb.sum())
        out = np.zeros(total, host.SIG_DTYPE)
        first2 = np.zeros(n + 1, np.uint64)
        hh = np.zeros((n, 20), np.uint8)
        fda = np.array([f.fileno() for f in fs], np.int32)
        rc = _lib.lib().sf_index_fds_blocks(fda.ctypes.data, stamps, n, po, pz, nb.ctypes.data, 0,
                                            out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)), total,
                                            first2.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), hh.ctypes.data,
                                            None, ctypes.byref(bad))
        assert rc == _lib.SF_EAGAIN and bad.value == 4
    finally:
        for f in fs:
            f.close()


def test_per_file_failures(gpu, tmp_path):
    """A stale stamp, a list past the end, offsets going backwards and a pipe
    fail for their own file; the others are exact."""
    lens = [50_000, 60_000, 70_000, 80_000, 90_000]
    files = _tree(tmp_path, lens, 7400)
    fs = [open(p, "rb") for p, *_ in files]
    r, w = os.pipe()
    try:
        stamps = [host.file_stamp(f.fileno()) for f in fs]
        lists = [(o, s) for _p, _d, o, s in files]
        with open(files[0][0], "r+b") as g:  # file 0 written after its stamp
            time.sleep(0.02)
            g.write(b"\x00" * 10)
        o1, s1 = lists[1]
        s1 = s1.copy()
        s1[-1] += 1  # file 1: last block one byte past the end
        lists[1] = (o1, s1)
        o3, s3 = lists[3]
        if len(o3) > 2:  # file 3: offsets going backwards
            o3 = o3.copy()
            o3[1], o3[2] = o3[2], o3[1]
        lists[3] = (o3, s3)
        fds = [f.fileno() for f in fs]
        fds[4] = r  # file 4: a pipe
        lists[4] = (np.array([0], np.uint64), np.array([1], np.uint32))
        rows, first, hashes, status = host.index_fds_blocks(fds, lists, stamps[:4] + [host.file_stamp(r)])
    finally:
        for f in fs:
            f.close()
        os.close(r)
        os.close(w)
    assert list(status) == [_lib.SF_EAGAIN, _lib.SF_ERANGE, 0, _lib.SF_EINVAL, _lib.SF_EINVAL]
    _check(files, rows, first, hashes, status, skip=(0, 1, 3, 4))


def test_descriptor_position_unused(gpu, tmp_path):
    files = _tree(tmp_path, [123_457, 1], 7500)
    fs = [open(p, "rb") for p, *_ in files]
    try:
        fs[0].read(1000)
        rows, first, hashes, status = host.index_fds_blocks([f.fileno() for f in fs],
                                                            [(o, s) for _p, _d, o, s in files])
        assert fs[0].tell() == 1000
    finally:
        for f in fs:
            f.close()
    _check(files, rows, first, hashes, status)


def _toy_chunker(f):
    """A content-defined stand-in over the open file (cut after a byte whose
    low 12 bits of a running sum hit 0, 32 KiB cap), as a stream chunker."""
    data = np.frombuffer(f.read(), np.uint8)
    sizes, start = [], 0
    h = np.cumsum(data.astype(np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFF) if data.size else data
    cuts = np.nonzero(h == 0)[0] if data.size else []
    for c in cuts:
        while c + 1 - start > 32768:
            sizes.append(32768)
            start += 32768
        if c + 1 > start:
            sizes.append(int(c + 1 - start))
            start = int(c + 1)
    while data.size - start > 32768:
        sizes.append(32768)
        start += 32768
    if data.size > start:
        sizes.append(int(data.size - start))
    return sizes


@pytest.mark.parametrize("threads", [1, 8])
def test_index_path_default_mode_on_the_gpu(gpu, tmp_path, threads):
    """Index.index_path with BoundaryChunker(stream=True): files cut on a pool,
    batches through sf_index_fds_blocks; a file rewritten while its batch is
    read is indexed again in its place.  Every stored row and blocks_hash
    equals the oracle's over the file's bytes at the end."""
    from syncfast_amd.index import BoundaryChunker, Index
    root = tmp_path / "tree"
    (root / "d").mkdir(parents=True)
    rng = np.random.default_rng(7600)
    names = [f"d/f{k:03d}" if k % 3 else f"g{k:03d}" for k in range(80)]
    for k, n in enumerate(names):
        (root / n).write_bytes(oracle.splitmix_bytes(int(rng.integers(0, 300 * KIB)), 7600 + k).tobytes())
    victim = root / names[60]
    fired = []

    def hook(stage):
        if stage == 0 and not fired:
            fired.append(stage)
            time.sleep(0.02)
            victim.write_bytes(oracle.splitmix_bytes(123_457, 7699).tobytes())

    idx = Index.open(root / ".syncfast.idx", chunker=BoundaryChunker(_toy_chunker, stream=True))
    _lib.set_read_hook(hook)
    try:
        idx.index_path(root, batch_bytes=2 * MIB, chunk_threads=threads)
    finally:
        _lib.set_read_hook(None)
    idx.commit()
    assert fired
    for n in names:
        data = (root / n).read_bytes()
        fid, _m, bh = idx.get_file(n)
        rows = idx.list_file_blocks(fid)
        sizes = np.asarray([s for _h, _o, s in rows], np.uint32)
        offs = np.asarray([o for _h, o, _s in rows], np.uint64)
        with open(root / n, "rb") as f:
            assert sizes.tolist() == _toy_chunker(f), n
        dig = oracle.index_blocks(np.frombuffer(data, np.uint8), offs, sizes) if len(sizes) else \
            np.zeros((0, 20), np.uint8)
        assert [h.bytes for h, _o, _s in rows] == [bytes(d) for d in dig], n
        assert bh.bytes == oracle.blocks_hash(dig) and idx.compute_blocks_hash(fid) == bh, n


def _odd_list(n, rng):
    """An allowed but unusual list over an n-byte file: sorted offsets, gaps,
    overlaps, empty blocks, blocks up to the end."""
    k = int(rng.integers(0, 40))
    offs = np.sort(rng.integers(0, n + 1, k)).astype(np.uint64) if n else np.zeros(k, np.uint64)
    sizes = np.array([int(rng.integers(0, n - o + 1)) if n > o else 0 for o in offs], np.uint32)
    return offs, sizes


@pytest.mark.parametrize("seed", range(12))
def test_fds_fuzz(gpu, tmp_path, seed):
    """Seeded random calls: 1-40 files of 0 B .. 2 MiB, each with a CDC-like,
    4 KiB fixed-like or odd list, stage sizes from 64 KiB to 4 MiB, with and
    without stamps; every row and blocks_hash against the oracle."""
    rng = np.random.default_rng(7900 + seed)
    nf = int(rng.integers(1, 41))
    files = []
    for k in range(nf):
        n = int(rng.choice([0, 1, int(rng.integers(2, 70_000)), int(rng.integers(70_000, 2 * MIB))]))
        data = oracle.splitmix_bytes(n, 8000 + 100 * seed + k).tobytes() if n else b""
        p = tmp_path / f"z{k:03d}"
        p.write_bytes(data)
        kind = int(rng.integers(0, 3))
        if kind == 0:
            sizes = _cdc_like_sizes(n, 9000 + 100 * seed + k, mean=int(rng.choice([512, 8192])))
            offs = _offs(sizes)
        elif kind == 1:
            offs = np.arange(0, n, 4096, dtype=np.uint64)
            sizes = np.minimum(4096, n - offs).astype(np.uint32)
        else:
            offs, sizes = _odd_list(n, rng)
        files.append((p, data, offs, sizes))
    stage = int(rng.choice([64 * KIB, 300 * KIB, 1 * MIB, 4 * MIB]))
    rows, first, hashes, status = _run(files, stamps=bool(rng.integers(0, 2)), stage_bytes=stage)
    _check(files, rows, first, hashes, status)


def _standin_ops():
    import ctypes
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "build",
                      "libzpaq_standin.so")
    assert os.path.exists(so), f"{so} not built: run __graft_entry__.build()"
    lib = ctypes.CDLL(so)
    lib.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    lib.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    lib.sf_zpaq_standin_ops_free.argtypes = [ctypes.c_void_p]
    return lib, lib.sf_zpaq_standin_ops(13, 32768)


@pytest.mark.parametrize("n", [0, 1, 70_000, (37 << 20) + 99, (600 << 20) + 5])
def test_index_fd_cut_equals_oracle(gpu, tmp_path, n):
    """sf_index_fd_cut: the stand-in chunker on 16 threads, the file read once
    and hashed from HBM by windows of up to 512 MiB (a 600 MiB file: two
    windows, the second starting at the first's last boundary); rows and
    blocks_hash equal the one-stream cut hashed by the oracle, and a stale
    stamp is SF_EAGAIN."""
    lib, ops = _standin_ops()
    try:
        data = oracle.splitmix_bytes(n, 7700 + n % 97)
        p = tmp_path / "f"
        data.tofile(p)
        sizes = oracle.zpaq_standin_sizes(data).astype(np.uint32)
        offs = _offs(sizes)
        dig = oracle.index_blocks(data, offs, sizes) if sizes.size else np.zeros((0, 20), np.uint8)
        with open(p, "rb") as f:
            st = host.file_stamp(f.fileno())
            rows, bh = host.index_fd_cut(f.fileno(), ops, 16, st)
        assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
        assert np.array_equal(rows["sha1"], dig) and bh == oracle.blocks_hash(dig)
        if n > 1:
            with open(p, "r+b") as g:
                g.write(b"\x01")
            os.utime(p, ns=(st.mtime_sec * 10**9 + st.mtime_nsec, st.mtime_sec * 10**9 + st.mtime_nsec + 1))
            with open(p, "rb") as f:
                with pytest.raises(_lib.SfError) as e:
                    host.index_fd_cut(f.fileno(), ops, 16, st)
            assert e.value.code == _lib.SF_EAGAIN
    finally:
        lib.sf_zpaq_standin_ops_free(ops)


@pytest.mark.parametrize("batch", [0, 1 << 30])
def test_index_native_chunker_on_the_gpu(gpu, tmp_path, batch):
    """Index(chunker=NativeChunker(stand-in ops)): index_file through
    sf_index_fd_cut (batch 0) or the walk through sf_cut_fd per file and
    sf_index_fds_blocks (batched); every stored row and blocks_hash against
    the oracle's one-stream stand-in."""
    from syncfast_amd.index import Index, NativeChunker
    lib, ops = _standin_ops()
    try:
        root = tmp_path / "t"
        root.mkdir()
        datas = {}
        for k, n in enumerate([0, 1, 9_999, (5 << 20) + 1, (17 << 20) + 321]):
            d = oracle.splitmix_bytes(n, 7800 + k)
            (root / f"f{k}").write_bytes(d.tobytes())
            datas[f"f{k}"] = d
        idx = Index.open_in_memory(chunker=NativeChunker(ops, threads=16))
        idx.index_path(root, batch_bytes=batch)
        for name, d in datas.items():
            fid, _, bh = idx.get_file(name)
            rows = idx.list_file_blocks(fid)
            sizes = oracle.zpaq_standin_sizes(d).astype(np.uint32)
            offs = _offs(sizes)
            dig = oracle.index_blocks(d, offs, sizes) if sizes.size else np.zeros((0, 20), np.uint8)
            assert [(o, s) for _h, o, s in rows] == list(zip(offs.tolist(), sizes.tolist())), name
            assert [h.to_sql() for h, _o, _s in rows] == [bytes(x).hex() for x in dig], name
            assert bh.to_sql() == oracle.blocks_hash(dig).hex(), name
    finally:
        lib.sf_zpaq_standin_ops_free(ops)


@pytest.mark.parametrize("window_mib,n", [(1, 5 << 20), (8, (20 << 20) + 12345), (16, (37 << 20) + 1)])
def test_index_fd_cut_small_windows(gpu, tmp_path, knobs, window_mib, n):
    """sf_index_fd_cut by windows (SF_TEST_CUT_WINDOW_MIB here, 512 MiB by
    default; 8 and 16 MiB windows hold 2 and 4 segments): every window ends at
    the last boundary inside it and the next starts there, so the chunk across
    each seam is cut again; rows and blocks_hash still equal the one-stream
    cut hashed by the oracle."""
    knobs.set("SF_TEST_CUT_WINDOW_MIB", window_mib)
    lib, ops = _standin_ops()
    try:
        data = oracle.splitmix_bytes(n, 7750)
        p = tmp_path / "w"
        data.tofile(p)
        sizes = oracle.zpaq_standin_sizes(data).astype(np.uint32)
        offs = _offs(sizes)
        dig = oracle.index_blocks(data, offs, sizes)
        for threads in (1, 4, 16):
            with open(p, "rb") as f:
                rows, bh = host.index_fd_cut(f.fileno(), ops, threads)
            assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes), threads
            assert np.array_equal(rows["sha1"], dig) and bh == oracle.blocks_hash(dig), threads
    finally:
        lib.sf_zpaq_standin_ops_free(ops)


def test_index_fd_cut_chunk_longer_than_window(gpu, tmp_path, knobs):
    """sf_index_fd_cut when a whole window holds no boundary (a chunk longer
    than the window: here a 1 MiB window and a stand-in with max_size 3 MiB +
    7 that practically never cuts by content, bits = 32): the call falls back
    to sf_cut_fd + sf_index_fd_blocks after giving its window buffers back
    (the fallback used to lease the device cache again while
    holding it).  Rows = the one-thread cut, digests and blocks_hash = the
    oracle's, on 1 and 16 threads, twice in a row (the cache is whole after)."""
    import ctypes
    knobs.set("SF_TEST_CUT_WINDOW_MIB", 1)
    lib, ops13 = _standin_ops()
    ops = lib.sf_zpaq_standin_ops(32, (3 << 20) + 7)
    try:
        n = (10 << 20) + 123
        data = oracle.splitmix_bytes(n, 7760)
        p = tmp_path / "long"
        data.tofile(p)
        with open(p, "rb") as f:
            offs, sizes = host.cut_fd(f.fileno(), ops, 1)
        assert int(np.asarray(sizes).max()) > (1 << 20)  # the window holds no boundary
        offs = np.asarray(offs, np.uint64)
        sizes = np.asarray(sizes, np.uint32)
        dig = oracle.index_blocks(data, offs, sizes)
        for threads in (1, 16, 16):
            with open(p, "rb") as f:
                rows, bh = host.index_fd_cut(f.fileno(), ops, threads)
            assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes), threads
            assert np.array_equal(rows["sha1"], dig) and bh == oracle.blocks_hash(dig), threads
    finally:
        lib.sf_zpaq_standin_ops_free(ctypes.c_void_p(ops))
        lib.sf_zpaq_standin_ops_free(ops13)


def test_index_path_large_file_among_small_files(gpu, tmp_path):
    """Index.index_path(NativeChunker) over a tree of one 600 MiB file and
    several hundred small ones (the reference's entry point,
    src/main.rs:122 -> src/index.rs:685-715 -> :610-659, cut a large file on
    one thread): the large file goes through sf_index_fd_cut on the chunker's
    threads in its walk position, the small ones through the batched
    pipeline.  Every row and blocks_hash equals the oracle's one-stream cut,
    and the blocks are stored in walk order (file_id non-decreasing by
    rowid)."""
    from syncfast_amd.index import Index, NativeChunker
    lib, ops = _standin_ops()
    try:
        root = tmp_path / "t"
        for d in ("a", "b"):
            (root / d).mkdir(parents=True)
        rng = np.random.default_rng(61)
        datas = {}
        for k in range(300):
            n = int(rng.integers(0, 60_000))
            name = f"{'a' if k % 2 else 'b'}/s{k:03d}"
            d = oracle.splitmix_bytes(n, 12000 + k)
            d.tofile(root / name)
            datas[name] = d
        big = oracle.splitmix_bytes((600 << 20) + 5, 12999)
        big.tofile(root / "a" / "big")
        datas["a/big"] = big
        idx = Index.open_in_memory(chunker=NativeChunker(ops, threads=16))
        idx.index_path(root)
        for name, d in datas.items():
            fid, _, bh = idx.get_file(name)
            rows = idx.list_file_blocks(fid)
            sizes = oracle.zpaq_standin_sizes(d).astype(np.uint32)
            offs = _offs(sizes)
            dig = oracle.index_blocks(d, offs, sizes) if sizes.size else np.zeros((0, 20), np.uint8)
            assert [(o, s) for _h, o, s in rows] == list(zip(offs.tolist(), sizes.tolist())), name
            assert [h.to_sql() for h, _o, _s in rows] == [bytes(x).hex() for x in dig], name
            assert bh.to_sql() == oracle.blocks_hash(dig).hex(), name
        fids = [r[0] for r in idx.db.execute("SELECT file_id FROM blocks ORDER BY rowid")]
        assert fids == sorted(fids)
    finally:
        lib.sf_zpaq_standin_ops_free(ops)
