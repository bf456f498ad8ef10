"""CPU: the C-ABI library loads, exports what include/syncfast_amd.h declares,
validates arguments, and its host stage (blocks_hash SHA-1) is exact.
No GPU compute is called here."""
import ctypes
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import syncfast_amd
from syncfast_amd import _lib, host

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(header="syncfast_amd.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sf_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    L = syncfast_amd.lib()
    names = header_functions()
    assert len(names) >= 13
    assert sorted(_lib.EXPORTED) == names
    for n in names:
        assert hasattr(L, n), n
    tnames = header_functions("syncfast_amd_test.h")
    assert sorted(_lib.EXPORTED_TEST) == tnames
    for n in tnames:
        assert hasattr(L, n), n


def test_every_include_header_is_checked():
    assert sorted(os.listdir(os.path.join(ROOT, "include"))) == ["syncfast_amd.h", "syncfast_amd_test.h"]


# A/B forms retired from the product sources in round 5:
# they live in git history and DESIGN.md's records, not in the shipped code.
RETIRED_MACROS = ("SF_EXPERIMENT_SEQ", "SF_EXPERIMENT_NOLOAD", "SF_PIPE", "SF_SCALAR_ISSUE", "SF_PRIO_EXP",
                  "SF_TUNING", "SF_VARIANT", "SF_STAGED_EXP", "SF_TABLE_PRIO", "SF_TABLE_PERSIST", "SF_TABLE_WPS",
                  "SF_OPAQUE_LANE", "SF_LIST_ALIGNED_TOO", "SF_CHAIN_PACK", "SF_WAVE_TRACE", "SF_CLASS_SORT",
                  "SF_CLASS_BITS_FORCE", "SF_NO_CHAIN_HELPER", "SF_FIXED_WPE", "SF_STAGED_WPE", "SF_TABLE_SNAKE",
                  "SF_TABLE_LB", "SF_TABLE_WG", "SF_TABLE_ROUND", "SF_CHAIN_DEPTH", "SF_SORT_ROUNDS", "SF_LOAD_AUX",
                  "SF_LIST_LOAD_AUX", "SF_CHAIN_PRIO")
# The only preprocessor conditionals the product sources may hold: the
# translation-unit switch of the shared kernel header, the host compiler's
# HIP platform define and the host SHA-NI path.
ALLOWED_CONDITIONALS = ("SF_STREAM_TU", "__HIP_PLATFORM_AMD__", "__x86_64__", "SF_WIRE_CHUNK_DEFAULT")


def _product_sources():
    csrc = os.path.join(ROOT, "syncfast_amd", "csrc")
    for fn in sorted(os.listdir(csrc)):
        if fn.endswith((".hip", ".hpp", ".cpp", ".h")) or fn == "Makefile":
            yield fn, open(os.path.join(csrc, fn)).read()


def test_product_kernels_carry_no_retired_ab_forms():
    for fn, src in _product_sources():
        for m in RETIRED_MACROS:
            assert not re.search(r"\b%s\b" % m, src), (fn, m)
        for line in src.splitlines():
            t = line.strip()
            if re.match(r"#\s*(if|ifdef|ifndef|elif)\b", t):
                assert any(a in t for a in ALLOWED_CONDITIONALS), (fn, t)


def test_stream_ordered_scratch_only_from_the_library_pool():
    """Every stream-ordered allocation of the library goes through
    stream_alloc (sf_alloc.cpp): the device's default pool, which gives its
    freed blocks back at every synchronisation, made file calls read wrong
    data through the sort's workspace ("The scratch pool")."""
    for fn, src in _product_sources():
        if fn == "sf_alloc.cpp":
            continue
        assert "hipMallocAsync" not in src and "hipMallocFromPoolAsync" not in src, fn


def test_environment_read_only_at_load():
    """Knobs are latched once when the library is loaded (sf_knobs.cpp): no
    other translation unit of the shipped library calls getenv, so nothing on
    a launch or copy path consults the environment."""
    csrc = os.path.join(ROOT, "syncfast_amd", "csrc")
    for fn in sorted(os.listdir(csrc)):
        if fn.endswith((".hip", ".hpp", ".cpp", ".h")) and fn != "sf_knobs.cpp":
            src = open(os.path.join(csrc, fn)).read()
            assert "getenv" not in src, fn


def test_knobs_latched_at_load_and_set_by_the_hook(monkeypatch):
    """A knob set in the environment after the library was loaded changes
    nothing; sf_test_set_knob does.  Result- or error-changing hooks carry the
    SF_TEST_ prefix; the old unprefixed names are gone."""
    syncfast_amd.lib()
    before = _lib.get_knob("SF_TEST_TABLE_SORT")
    monkeypatch.setenv("SF_TEST_TABLE_SORT", "1" if before != 1 else "0")
    assert _lib.get_knob("SF_TEST_TABLE_SORT") == before
    old = _lib.set_knob("SF_TEST_TABLE_SORT", 1)
    try:
        assert old == before and _lib.get_knob("SF_TEST_TABLE_SORT") == 1
    finally:
        _lib.set_knob("SF_TEST_TABLE_SORT", before)
    for gone in ("SF_TEST_CHAIN_SPIN_LIMIT", "SF_TEST_CHAIN_POLL_GAP_US", "SF_TEST_STAGES", "SF_TABLE_SORT", "SF_CHAIN_SPIN_LIMIT", "SF_LAUNCH_MAX_BLOCKS", "SF_INPLACE_FAIL_AT", "SF_STAGES",
                 "SF_FILE_INPLACE", "SF_MAP_MIN_MIB"):
        with pytest.raises(_lib.SfError):
            _lib.get_knob(gone)
    for name in ("SF_BATCH_FUSED", "SF_TEST_LAUNCH_MAX_BLOCKS", "SF_TEST_INPLACE_FAIL_AT",
                 "SF_TEST_WIRE_CHUNK", "SF_TEST_STREAM_STAGE_MIB", "SF_IO_THREADS"):
        _lib.get_knob(name)
    assert _lib.get_stat("pages_locked") >= 0 and _lib.get_stat("not_anon_refused") >= 0


def test_knobs_from_the_environment_at_load(tmp_path):
    """The environment at load time sets the knobs (a fresh process)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from syncfast_amd import _lib; "
            "print(_lib.get_knob('SF_TEST_TABLE_SORT'), _lib.get_knob('SF_IO_THREADS'))" % ROOT)
    env = dict(os.environ, SF_TEST_TABLE_SORT="0", SF_IO_THREADS="7")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.split() == ["0", "7"]


def test_version_and_errors():
    L = syncfast_amd.lib()
    assert b"gfx950" in L.sf_version()
    for code in (_lib.SF_EINVAL, _lib.SF_ENOSPC, _lib.SF_ERANGE, _lib.SF_ENODEV, _lib.SF_EIO, _lib.SF_ENOMEM):
        assert L.sf_strerror(code).decode() not in ("", "unknown error")


def test_struct_layout():
    assert ctypes.sizeof(_lib.BlockSig) == 32
    assert _lib.BlockSig.sha1.offset == 12
    assert ctypes.sizeof(_lib.FileDesc) == 16
    assert ctypes.sizeof(_lib.ChainJob) == 40  # include/syncfast_amd.h sf_chain_job


def test_chained_cols_validation_without_device():
    # sf_index_device_batch_chained_cols checks its column range before any
    # device work: whole 64-block waves of whole-wave files, lo < hi <= blocks
    L = syncfast_amd.lib()
    jobs = (_lib.ChainJob * 1)()

    def call(nf, flen, bs, lo, hi, data=None, dig=None, nj=0):
        return L.sf_index_device_batch_chained_cols(data, nf, flen, bs, lo, hi, dig, jobs, nj, None)

    E = _lib.SF_EINVAL
    assert call(2, 4096 * 128, 0, 0, 64) == E  # block size 0
    assert call(2, 4096 * 96, 4096, 0, 64) == E  # 96 blocks per file: not whole waves
    for lo, hi in [(0, 100), (32, 128), (64, 64), (128, 64), (0, 192)]:
        assert call(2, 4096 * 128, 4096, lo, hi, 1 << 20, 1 << 20) == E, (lo, hi)
    assert call(2, 4096 * 128, 4096, 0, 64) == E  # no data / digests
    assert call(2, 4096 * 128, 4096, 0, 128, 1 << 20, 1 << 20, nj=3) == E  # at most two jobs
    assert call(0, 4096 * 128, 4096, 0, 128) == 0  # nothing to hash, no jobs: nothing launched


def test_batch_stream_column_split():
    # BatchStream.push_last's cut: the first half of a chain (part 1) reads
    # digests [0, ceil(64 * half / 20)), rounded up to whole 64-block waves
    from syncfast_amd.device import BatchStream
    assert BatchStream(1024, 8 << 20, 4096)._half_cols() == 1024
    assert BatchStream(40, 128 * 4096, 4096)._half_cols() == 64
    assert BatchStream(9, 192 * 1024, 1024)._half_cols() == 128
    assert BatchStream(4, 64 * 4096, 4096)._half_cols() is None  # one wave per file
    assert BatchStream(4, 100 * 4096, 4096)._half_cols() is None  # not whole waves
    assert BatchStream(4, 1024 * 4096, 4096, split=False)._half_cols() is None
    for nbf in range(128, 4097, 64):
        cut = BatchStream(3, nbf * 4096, 4096)._half_cols()
        half = (nbf * 20 // 64) // 2
        assert cut is not None and cut % 64 == 0 and cut * 20 >= half * 64 and cut - 64 < -(-half * 64 // 20)


def test_argument_validation_without_device():
    L = syncfast_amd.lib()
    n = ctypes.c_uint64(0)
    # block size 0 / too large are rejected before any device work
    assert L.sf_index_device_fixed(None, 100, 0, None, 0, ctypes.byref(n), None) == _lib.SF_EINVAL
    assert L.sf_index_device_fixed(None, 100, (32 << 20) + 1, None, 0, ctypes.byref(n), None) == _lib.SF_EINVAL
    # capacity check reports the need
    assert L.sf_index_device_fixed(None, 10000, 4096, None, 1, ctypes.byref(n), None) == _lib.SF_ENOSPC
    assert n.value == 3
    # empty input: zero blocks, nothing launched
    assert L.sf_index_device_fixed(None, 0, 4096, None, 0, ctypes.byref(n), None) == 0 and n.value == 0
    assert L.sf_index_device_blocks(None, 0, None, None, 0, None, None, None) == 0
    assert L.sf_index_device_blocks(None, 5, None, None, 3, None, None, None) == _lib.SF_EINVAL
    out = np.zeros(4, host.SIG_DTYPE)
    assert L.sf_index_buffer(None, 0, 4096, out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)), 0,
                             ctypes.byref(n)) == 0 and n.value == 0
    assert L.sf_index_file(b"/nonexistent/file", 4096, None, 0, ctypes.byref(n), None) == _lib.SF_EIO
    assert L.sf_blocks_hash(None, 0, None) == _lib.SF_EINVAL


def test_buffer_blocks_validation_without_device():
    """sf_index_buffer_blocks checks the whole list before anything moves:
    an empty list is the empty blocks_hash, a block past the end is SF_ERANGE
    (the device form zeroes it instead), offsets going backwards SF_EINVAL."""
    L = syncfast_amd.lib()
    data = np.arange(100, dtype=np.uint8)
    out = np.zeros(4, host.SIG_DTYPE)
    pout = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))
    bh = (ctypes.c_uint8 * 20)()
    assert L.sf_index_buffer_blocks(data.ctypes.data, data.size, None, None, 0, None, bh) == 0
    assert bytes(bh) == hashlib.sha1(b"").digest()
    rows, h = host.index_buffer_blocks(b"", [], [])
    assert rows.size == 0 and h == hashlib.sha1(b"").digest()

    def call(offs, sizes, length=data.size):
        o = np.asarray(offs, np.uint64)
        s = np.asarray(sizes, np.uint32)
        return L.sf_index_buffer_blocks(data.ctypes.data, length, o.ctypes.data, s.ctypes.data, o.size, pout, None)

    assert call([0, 90], [10, 11]) == _lib.SF_ERANGE  # 90 + 11 > 100
    assert call([101], [0]) == _lib.SF_ERANGE
    assert call([0, 50, 40], [10, 10, 10]) == _lib.SF_EINVAL  # offsets go backwards
    assert call([0], [1], length=0) == _lib.SF_ERANGE
    assert L.sf_index_buffer_blocks(None, 10, None, None, 0, None, None) == _lib.SF_EINVAL  # len > 0, no data
    o = np.zeros(1, np.uint64)
    assert L.sf_index_buffer_blocks(data.ctypes.data, data.size, o.ctypes.data, None, 1, pout, None) == _lib.SF_EINVAL
    with pytest.raises(_lib.SfError):
        host.index_buffer_blocks(data, [0, 95], [10, 10])


def test_file_blocks_validation_without_device(tmp_path):
    """sf_index_file_blocks: a path that does not open or is not a regular
    file is SF_EIO, a block past the FILE's end SF_ERANGE, offsets going
    backwards SF_EINVAL -- all before any device call."""
    L = syncfast_amd.lib()
    p = tmp_path / "f"
    p.write_bytes(bytes(range(256)) * 4)
    out = np.zeros(4, host.SIG_DTYPE)
    pout = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))

    def call(path, offs, sizes):
        o = np.asarray(offs, np.uint64)
        s = np.asarray(sizes, np.uint32)
        return L.sf_index_file_blocks(path, o.ctypes.data, s.ctypes.data, o.size, pout, None)

    assert call(b"/nonexistent/file", [0], [1]) == _lib.SF_EIO
    assert call(bytes(tmp_path), [0], [1]) == _lib.SF_EIO  # a directory
    fifo = tmp_path / "fifo"
    os.mkfifo(fifo)  # no writer: refused at once, not waited on
    assert call(bytes(fifo), [0], [1]) == _lib.SF_EIO
    assert call(bytes(p), [0, 1000], [1000, 25]) == _lib.SF_ERANGE  # 1025 > 1024
    assert call(bytes(p), [10, 5], [1, 1]) == _lib.SF_EINVAL
    assert L.sf_index_file_blocks(None, None, None, 0, None, None) == _lib.SF_EINVAL
    rows, bh = host.index_file_blocks(p, [], [])
    assert rows.size == 0 and bh == hashlib.sha1(b"").digest()
    with pytest.raises(_lib.SfError, match="nonexistent"):
        host.index_file_blocks("/nonexistent/file", [0], [1])


def test_fd_routes_validation_without_device(tmp_path):
    """sf_index_fd_blocks / sf_index_fd_fixed (the chunker's own descriptor):
    stamps, argument checks and the stamp comparison all run before any
    device call.  A stamp that no longer matches the open file is SF_EAGAIN
    (the caller re-chunks); a non-regular descriptor is SF_EINVAL."""
    L = syncfast_amd.lib()
    p = tmp_path / "f"
    p.write_bytes(bytes(range(256)) * 4)
    out = np.zeros(4, host.SIG_DTYPE)
    pout = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))
    n = ctypes.c_uint64(77)
    with open(p, "rb") as f:
        fd = f.fileno()
        st = host.file_stamp(fd)
        sb = os.fstat(fd)
        assert (st.dev, st.ino, st.size, st.nlink) == (sb.st_dev, sb.st_ino, 1024, sb.st_nlink)
        assert st.mtime_sec * 10**9 + st.mtime_nsec == sb.st_mtime_ns
        assert st.ctime_sec * 10**9 + st.ctime_nsec == sb.st_ctime_ns
        o = np.asarray([0, 1000], np.uint64)
        s = np.asarray([1000, 25], np.uint32)
        assert L.sf_index_fd_blocks(fd, ctypes.byref(st), o.ctypes.data, s.ctypes.data, 2, pout, None) == \
            _lib.SF_ERANGE
        s2 = np.asarray([10, 5], np.uint64)
        assert L.sf_index_fd_blocks(fd, None, s2.ctypes.data, s.ctypes.data, 2, pout, None) == _lib.SF_EINVAL
        assert L.sf_index_fd_blocks(-1, None, None, None, 0, None, None) == _lib.SF_EINVAL
        assert L.sf_index_fd_blocks(fd, None, None, None, 1, None, None) == _lib.SF_EINVAL
        rows, bh = host.index_fd_blocks(fd, [], [], st)
        assert rows.size == 0 and bh == hashlib.sha1(b"").digest()
        # cap too small: the need, nothing read
        assert L.sf_index_fd_fixed(fd, ctypes.byref(st), 512, pout, 1, ctypes.byref(n), None) == _lib.SF_ENOSPC
        assert n.value == 2
        assert L.sf_index_fd_fixed(fd, None, 0, pout, 4, ctypes.byref(n), None) == _lib.SF_EINVAL
        assert L.sf_index_fd_fixed(-1, None, 4096, pout, 4, ctypes.byref(n), None) == _lib.SF_EINVAL
        # the file changes after the stamp: in place (same size, mtime put back), appended, replaced
        stale = host.file_stamp(fd)
        stale.ctime_nsec += 1  # what a write with the mtime restored leaves: only the ctime moves
        for call in (lambda: host.index_fd_blocks(fd, [0], [10], stale),
                     lambda: host.index_fd_fixed(fd, 4096, stale)):
            with pytest.raises(_lib.SfError) as e:
                call()
            assert e.value.code == _lib.SF_EAGAIN
        # a link added or removed moves the ctime but not the bytes: still the same file
        moved = host.file_stamp(fd)
        moved.nlink += 1
        moved.ctime_nsec += 1
        assert _lib.same_stamp(moved, host.file_stamp(fd))
        with open(p, "ab") as w:
            w.write(b"more")
        with pytest.raises(_lib.SfError) as e:
            host.index_fd_blocks(fd, [0], [10], st)
        assert e.value.code == _lib.SF_EAGAIN
    # an empty file: no blocks, SHA1("") -- no device needed
    e0 = tmp_path / "empty"
    e0.write_bytes(b"")
    with open(e0, "rb") as f:
        rows, bh = host.index_fd_fixed(f.fileno(), 4096, host.file_stamp(f.fileno()))
        assert rows.size == 0 and bh == hashlib.sha1(b"").digest()
    # a pipe is not a regular file: the list cannot be read again
    r, w = os.pipe()
    try:
        assert L.sf_index_fd_blocks(r, None, None, None, 0, None, None) == _lib.SF_EINVAL
        assert L.sf_index_fd_fixed(r, None, 4096, pout, 4, ctypes.byref(n), None) == _lib.SF_EINVAL
    finally:
        os.close(r)
        os.close(w)


def test_host_paths_without_device():
    """Without a GPU the host-memory entry points fail cleanly: the in-place
    route (>= 1 MiB) cannot page-lock, the staged route cannot set up its
    streams, and the call returns SF_ENODEV; releasing the (empty) per-device
    cache is a no-op."""
    L = syncfast_amd.lib()
    nd = ctypes.c_int(0)
    if L.sf_device_count(ctypes.byref(nd)) == 0 and nd.value > 0:
        pytest.skip("a device is visible")
    n = ctypes.c_uint64(0)
    data = np.zeros(64 << 20, np.uint8)
    out = np.zeros((64 << 20) // 4096, host.SIG_DTYPE)
    rc = L.sf_index_buffer(data.ctypes.data, data.size, 4096, out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)),
                           out.size, ctypes.byref(n))
    assert rc == _lib.SF_ENODEV and n.value == out.size
    offs = np.arange(0, data.size, 8192, dtype=np.uint64)
    sizes = np.full(offs.size, 8192, np.uint32)
    rc = L.sf_index_buffer_blocks(data.ctypes.data, data.size, offs.ctypes.data, sizes.ctypes.data, offs.size,
                                  out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)), None)
    assert rc == _lib.SF_ENODEV
    assert L.sf_release_host_cache() == 0


def test_index_files_validation_without_device(tmp_path):
    """sf_index_files sizes every file and checks capacity before any read or
    device call: empty list, missing file (named by index), ENOSPC."""
    L = syncfast_amd.lib()
    n, bad = ctypes.c_uint64(7), ctypes.c_uint32(99)
    first = np.zeros(4, np.uint64)
    fh = np.zeros((3, 20), np.uint8)
    pfirst = first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    none = (ctypes.c_char_p * 1)()
    assert L.sf_index_files(none, 0, 4096, 0, None, 0, pfirst, fh.ctypes.data, ctypes.byref(n),
                            ctypes.byref(bad)) == 0 and n.value == 0
    a, b = tmp_path / "a", tmp_path / "b"
    a.write_bytes(b"x" * 5000)
    b.write_bytes(b"")
    paths = (ctypes.c_char_p * 3)(bytes(a), b"/nonexistent/file", bytes(b))
    assert L.sf_index_files(paths, 3, 4096, 0, None, 0, pfirst, fh.ctypes.data, ctypes.byref(n),
                            ctypes.byref(bad)) == _lib.SF_EIO and bad.value == 1
    paths = (ctypes.c_char_p * 3)(bytes(a), bytes(b), bytes(tmp_path))  # a directory is not a file
    assert L.sf_index_files(paths, 3, 4096, 0, None, 0, pfirst, fh.ctypes.data, ctypes.byref(n),
                            ctypes.byref(bad)) == _lib.SF_EIO and bad.value == 2
    paths = (ctypes.c_char_p * 3)(bytes(a), bytes(b), bytes(a))
    assert L.sf_index_files(paths, 3, 4096, 0, None, 3, pfirst, fh.ctypes.data, ctypes.byref(n),
                            ctypes.byref(bad)) == _lib.SF_ENOSPC and n.value == 4
    assert first.tolist() == [0, 2, 2, 4]
    assert L.sf_index_files(paths, 3, 0, 0, None, 9, pfirst, fh.ctypes.data, ctypes.byref(n),
                            ctypes.byref(bad)) == _lib.SF_EINVAL
    with pytest.raises(_lib.SfError, match="nonexistent"):
        host.index_files([a, "/nonexistent/file"], 4096)


def test_device_count_is_queryable():
    assert syncfast_amd.device_count() >= 0


@pytest.mark.parametrize("length", [0, 1, 55, 56, 63, 64, 65, 119, 120, 1000, 65536 + 7])
def test_host_sha1_exact(length):
    data = oracle.splitmix_bytes(length, length + 5).tobytes()
    want = hashlib.sha1(data).digest()
    assert host.sha1(data) == want
    # both host code paths (SHA-NI when present, scalar)
    L = syncfast_amd.lib()
    L.sf_host_sha1_impl.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    for force_scalar in (0, 1):
        a = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        out = (ctypes.c_uint8 * 20)()
        L.sf_host_sha1_impl(a.ctypes.data, length, out, force_scalar)
        assert bytes(out) == want


def test_blocks_hash_matches_reference_kat(golden):
    g = golden["reference_kat"]
    digs = b"".join(bytes.fromhex(b["sha1"]) for b in g["blocks"])
    assert host.blocks_hash(digs).hex() == g["blocks_hash"]
    assert host.blocks_hash(b"").hex() == "da39a3ee5e6b4b0d3255bfef95601890afd80709"


def test_blocks_hash_golden(golden):
    for case in golden["fixed"] + golden["ragged"]:
        digs = b"".join(bytes.fromhex(h) for h in case["digests"])
        assert host.blocks_hash(digs).hex() == case["blocks_hash"]


def test_blocks_hash_sigs_rows():
    rows = np.zeros(5, host.SIG_DTYPE)
    rng = np.random.default_rng(3)
    rows["sha1"] = rng.integers(0, 256, (5, 20), dtype=np.uint8)
    out = (ctypes.c_uint8 * 20)()
    L = syncfast_amd.lib()
    assert L.sf_blocks_hash_sigs(rows.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)), 5, out) == 0
    assert bytes(out) == hashlib.sha1(rows["sha1"].tobytes()).digest()


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "syncfast_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                src = open(os.path.join(dirpath, fn), errors="replace").read()
                assert "import oracle" not in src and "from oracle" not in src, fn
                assert "sf_oracle" not in src and "sfo_" not in src, fn


def test_traffic_profile_is_for_this_kernel():
    # bench.py reports roofline.traffic only when profiles/traffic.json was
    # measured on the same machine code of the headline kernel; this keeps the
    # committed PMC pass in step with it (refresh it after any change to that
    # kernel: PROFILE=1 scripts/gpu_round.sh, then scripts/pmc_traffic.py)
    import json
    from syncfast_amd._lib import kernel_code_sha256
    h = kernel_code_sha256()
    assert len(h) == 64
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
        tr = json.load(f)
    assert tr["config2"]["kernel_code_sha256"] == h


@pytest.mark.parametrize("n", [0, 1, 3276, 3277, 10_000])
def test_blocks_hash_sigs_across_its_gather_buffer(n):
    # sf_blocks_hash_sigs gathers digests a fixed buffer (3276 rows) at a time
    rows = np.zeros(max(n, 1), host.SIG_DTYPE)[:n]
    rows["sha1"] = np.random.default_rng(n).integers(0, 256, (n, 20), dtype=np.uint8)
    out = (ctypes.c_uint8 * 20)()
    assert syncfast_amd.lib().sf_blocks_hash_sigs(rows.ctypes.data_as(ctypes.POINTER(_lib.BlockSig)), n, out) == 0
    assert bytes(out) == hashlib.sha1(rows["sha1"].tobytes()).digest()


def test_pmc_traffic_averages_full_shard_launches(tmp_path):
    # scripts/pmc_traffic.py: only the largest grid of the pass counts (the
    # bench's shard launches), not smaller launches in the same process
    import csv
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(ROOT, "scripts", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    p = tmp_path / "pmc.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (grid, v) in enumerate([(2097152, 100.0), (2097152, 102.0), (65536, 3.0), (16777216, 7.0)]):
            name = "sf::fill_splitmix_kernel" if grid == 16777216 else "void sf::sha1_fixed_kernel<128, 1, false>"
            w.writerow({"Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name, "Counter_Name": "FETCH_SIZE",
                        "Counter_Value": v})
    assert mod.avg(str(p), "FETCH_SIZE") == (101.0, 2)


def test_chained_kernel_is_the_measured_one():
    # sha1_fixed_chained_kernel<128>'s block part ran at the plain kernel's
    # rate only in some compiled forms: the committed
    # launch-sequence measurement names the machine code it measured
    import json
    from syncfast_amd._lib import CHAINED_KERNEL, kernel_code_sha256
    with open(os.path.join(ROOT, "profiles", "r03", "c3", "chained_kernel.json")) as f:
        rec = json.load(f)
    assert kernel_code_sha256(symbol=CHAINED_KERNEL) == rec["kernel_code_sha256"], \
        "the chained kernel changed: re-measure with scripts/c3_seq.sh and update the record"



def test_fds_blocks_checks_before_any_device_call(tmp_path):
    """sf_index_fds_blocks: the plan (first_row), SF_ENOSPC and each file's
    own checks (stale stamp, a list past the end or going backwards, a pipe)
    come before any device work; files with no blocks get SHA1("") -- so all
    of this runs without a GPU."""
    import time
    paths = []
    for k, n in enumerate([0, 100, 200, 0]):
        p = tmp_path / f"f{k}"
        p.write_bytes(bytes(range(256))[:n] if n <= 256 else b"")
        paths.append(p)
    fs = [open(p, "rb") for p in paths]
    r, w = os.pipe()
    try:
        stamps = [host.file_stamp(f.fileno()) for f in fs]
        time.sleep(0.02)
        with open(paths[1], "r+b") as g:
            g.write(b"\x00")
        lists = [([], []), ([0, 50], [50, 50]), ([0, 100, 50], [100, 50, 50]), ([], [])]
        rows, first, hashes, status = host.index_fds_blocks([f.fileno() for f in fs], lists, stamps)
        assert list(first) == [0, 0, 2, 5, 5]
        assert list(status) == [0, _lib.SF_EAGAIN, _lib.SF_EINVAL, 0]
        assert bytes(hashes[0]).hex() == bytes(hashes[3]).hex() == "da39a3ee5e6b4b0d3255bfef95601890afd80709"
        assert bytes(hashes[1]) == bytes(20) and bytes(hashes[2]) == bytes(20)
        # past the end; a pipe
        rows, first, hashes, status = host.index_fds_blocks([fs[2].fileno(), r], [([150], [51]), ([0], [1])])
        assert list(status) == [_lib.SF_ERANGE, _lib.SF_EINVAL]
        # capacity and arguments: call-level errors
        L = syncfast_amd.lib()
        first = np.zeros(2, np.uint64)
        nb = np.array([2], np.uint64)
        o = np.array([0, 50], np.uint64)
        s = np.array([50, 50], np.uint32)
        po = (ctypes.c_void_p * 1)(o.ctypes.data)
        pz = (ctypes.c_void_p * 1)(s.ctypes.data)
        fd = np.array([fs[2].fileno()], np.int32)
        hh = np.zeros(20, np.uint8)
        out = np.zeros(2, host.SIG_DTYPE)
        sig = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))
        u64p = first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        assert L.sf_index_fds_blocks(fd.ctypes.data, None, 1, po, pz, nb.ctypes.data, 0, sig, 1, u64p,
                                     hh.ctypes.data, None, None) == _lib.SF_ENOSPC
        assert list(first) == [0, 2]
        assert L.sf_index_fds_blocks(None, None, 1, po, pz, nb.ctypes.data, 0, sig, 2, u64p, hh.ctypes.data,
                                     None, None) == _lib.SF_EINVAL
        assert L.sf_index_fds_blocks(fd.ctypes.data, None, 1, po, pz, nb.ctypes.data, 0, None, 2, u64p,
                                     hh.ctypes.data, None, None) == _lib.SF_EINVAL
        assert L.sf_index_fds_blocks(None, None, 0, None, None, None, 0, None, 0, None, None, None,
                                     None) == _lib.SF_OK
    finally:
        for f in fs:
            f.close()
        os.close(r)
        os.close(w)


def test_shard_range_c_equals_python():
    """sf_shard_range (the multi-device forms' partition) is
    syncfast_amd.shard.shard_range, the one-process-per-GPU partition."""
    from syncfast_amd.shard import shard_range
    L = syncfast_amd.lib()
    s, n = ctypes.c_uint64(), ctypes.c_uint64()
    rng = np.random.default_rng(3)
    cases = [(0, 4096, 1), (1, 4096, 8), (4096 * 8, 4096, 8), (4096 * 8 + 1, 4096, 8), (10, 3, 7), (7, 100, 3)]
    cases += [(int(rng.integers(0, 1 << 40)), int(rng.integers(1, 1 << 20)), int(rng.integers(1, 9)))
              for _ in range(200)]
    for total, bs, world in cases:
        prev_end = 0
        for r in range(world):
            assert L.sf_shard_range(total, bs, world, r, ctypes.byref(s), ctypes.byref(n)) == 0
            assert (s.value, n.value) == shard_range(total, bs, world, r)
            assert s.value == prev_end or n.value == 0
            prev_end = s.value + n.value if n.value else prev_end
        assert prev_end == total
    assert L.sf_shard_range(100, 0, 2, 0, ctypes.byref(s), ctypes.byref(n)) == _lib.SF_EINVAL
    assert L.sf_shard_range(100, 10, 0, 0, ctypes.byref(s), ctypes.byref(n)) == _lib.SF_EINVAL
    assert L.sf_shard_range(100, 10, 2, 2, ctypes.byref(s), ctypes.byref(n)) == _lib.SF_EINVAL
    assert L.sf_shard_range(100, 10, 2, 0, None, ctypes.byref(n)) == _lib.SF_EINVAL


def test_multi_device_argument_checks(tmp_path):
    """The multi-device forms check their arguments before touching a device
    (on this machine, with no device, a valid call is SF_ENODEV)."""
    L = syncfast_amd.lib()
    p = tmp_path / "f"
    p.write_bytes(b"x" * 10000)
    out = np.zeros(4, host.SIG_DTYPE)
    sig = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))
    need = ctypes.c_uint64()
    bh = (ctypes.c_uint8 * 20)()
    assert L.sf_index_file_multi(os.fsencode(p), 0, 1, sig, 4, ctypes.byref(need), bh) == _lib.SF_EINVAL
    assert L.sf_index_file_multi(os.fsencode(p), (32 << 20) + 1, 1, sig, 4, ctypes.byref(need), bh) == _lib.SF_EINVAL
    assert L.sf_index_file_multi(None, 4096, 1, sig, 4, ctypes.byref(need), bh) == _lib.SF_EINVAL
    assert L.sf_index_file_multi(os.fsencode(p), 4096, 1, sig, 4, ctypes.byref(need), None) == _lib.SF_EINVAL
    one = (ctypes.c_void_p * 1)(1)
    assert L.sf_index_device_multi(0, one, 100, 4096, one, 0, 1, None) == _lib.SF_EINVAL
    assert L.sf_index_device_multi(1, one, 100, 4096, one, 1, 1, None) == _lib.SF_EINVAL  # root out of range
    assert L.sf_index_device_multi(1, None, 100, 4096, one, 0, 1, None) == _lib.SF_EINVAL
    assert L.sf_index_device_multi(1, one, 100, 0, one, 0, 1, None) == _lib.SF_EINVAL
    if _lib.device_count() == 0:
        assert L.sf_index_file_multi(os.fsencode(p), 4096, 1, sig, 4, ctypes.byref(need), bh) == _lib.SF_ENODEV
        assert L.sf_index_device_multi(1, one, 100, 4096, one, 0, 1, None) == _lib.SF_ENODEV


def test_table_kernel_is_the_measured_one():
    """the explicit-list kernel's rate depends on its compiled form
    (DESIGN.md 3.4); the committed record names the machine code the round-5
    A/B measured as the shipped form, so a change cannot silently replace it."""
    import json
    from syncfast_amd._lib import TABLE_KERNEL, kernel_code_sha256
    with open(os.path.join(ROOT, "profiles", "r05", "table_kernel.json")) as f:
        rec = json.load(f)
    assert rec["symbol"] == TABLE_KERNEL
    assert kernel_code_sha256(symbol=TABLE_KERNEL) == rec["kernel_code_sha256"], \
        "the explicit-list kernel changed: re-measure (scripts/gpu_tab_ab.sh) and update the record"


def _cxx_sanitizer_works(flag, tmp_path):
    src = tmp_path / "probe.cpp"
    src.write_text("#include <thread>\nint main(){std::thread t([]{});t.join();}\n")
    r = subprocess.run(["g++", "-std=c++17", "-pthread", flag, str(src), "-o", str(tmp_path / "probe")],
                       capture_output=True)
    return r.returncode == 0 and subprocess.run([str(tmp_path / "probe")], capture_output=True).returncode == 0


@pytest.mark.parametrize("sanitizer", ["-fsanitize=thread", "-fsanitize=address,undefined"])
def test_host_pool_stress(tmp_path, sanitizer):
    """The kept host worker threads every pipeline stage uses (sf_pool.cpp):
    concurrent callers, nested pools, a worker that throws; every work item
    runs exactly once, under ThreadSanitizer and under ASan + UBSan (the pool
    is host code: built here with g++ from the library's own source)."""
    if not _cxx_sanitizer_works(sanitizer, tmp_path):
        pytest.skip(f"g++ {sanitizer} unavailable")
    root = os.path.join(os.path.dirname(__file__), "..")
    exe = tmp_path / "pool_stress"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", sanitizer, "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", os.path.join(root, "tests", "native", "pool_stress.cpp"),
                    os.path.join(root, "syncfast_amd", "csrc", "sf_pool.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "pool_stress ok" in r.stdout, r.stderr[-2000:]
