"""Host-memory entry points (bytes in host RAM or on disk -> signature rows).

These are the end-to-end forms of the path (the reference reads files,
src/index.rs:615): the C-ABI stages the bytes through pinned buffers, runs the
HIP kernel, and copies the rows back.  ``blocks_hash`` is the host stage of
compute_blocks_hash (src/index.rs:661-682).
"""
from __future__ import annotations

import ctypes
import os
import stat
from typing import List, Sequence, Tuple

import numpy as np

from ._lib import SF_EINVAL, SF_EIO, SF_ENOSPC, BlockSig, FileStamp, check, lib

SIG_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u4"), ("sha1", "u1", (20,))], align=True)
assert SIG_DTYPE.itemsize == ctypes.sizeof(BlockSig) == 32


def _u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(data), dtype=np.uint8)


def index_buffer(data, block_size: int) -> np.ndarray:
    """Fixed-size block signatures of a host buffer -> SIG_DTYPE rows."""
    a = _u8(data)
    n = (a.size + block_size - 1) // block_size if a.size else 0
    out = np.zeros(max(n, 1), SIG_DTYPE)
    nout = ctypes.c_uint64(0)
    check(lib().sf_index_buffer(a.ctypes.data if a.size else None, a.size, block_size,
                                out.ctypes.data_as(ctypes.POINTER(BlockSig)), n, ctypes.byref(nout)),
          "sf_index_buffer")
    return out[:n]


def index_buffer_blocks(data, offsets, sizes) -> Tuple[np.ndarray, bytes]:
    """Signatures of an explicit block list over a host buffer (block i =
    data[offsets[i]:offsets[i]+sizes[i]], offsets non-decreasing: a chunker's
    output) -> (SIG_DTYPE rows in list order, blocks_hash over their digests)
    (sf_index_buffer_blocks).  SF_ERANGE / SF_EINVAL for a block past the end
    / offsets that go backwards, before anything runs."""
    a = _u8(data)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    szs = np.ascontiguousarray(sizes, dtype=np.uint32).reshape(-1)
    if offs.size != szs.size:
        raise ValueError("offsets and sizes differ in length")
    n = offs.size
    out = np.zeros(max(n, 1), SIG_DTYPE)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_buffer_blocks(a.ctypes.data if a.size else None, a.size,
                                       offs.ctypes.data if n else None, szs.ctypes.data if n else None, n,
                                       out.ctypes.data_as(ctypes.POINTER(BlockSig)), bh),
          "sf_index_buffer_blocks")
    return out[:n], bytes(bh)


def index_file_blocks(path, offsets, sizes) -> Tuple[np.ndarray, bytes]:
    """As index_buffer_blocks over a regular file on disk, read again window
    by window with pread (sf_index_file_blocks): the boundaries came from a
    chunker that streamed the file; the file is never held whole in memory."""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    szs = np.ascontiguousarray(sizes, dtype=np.uint32).reshape(-1)
    if offs.size != szs.size:
        raise ValueError("offsets and sizes differ in length")
    n = offs.size
    out = np.zeros(max(n, 1), SIG_DTYPE)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_file_blocks(os.fsencode(path), offs.ctypes.data if n else None,
                                     szs.ctypes.data if n else None, n,
                                     out.ctypes.data_as(ctypes.POINTER(BlockSig)), bh),
          f"sf_index_file_blocks({os.fsdecode(path)})")
    return out[:n], bytes(bh)


def file_stamp(fd: int) -> FileStamp:
    """sf_file_stamp_fd: fstat's identity of the file open on fd (dev, ino,
    size, mtime, ctime), taken before a chunker reads it."""
    st = FileStamp()
    check(lib().sf_file_stamp_fd(int(fd), ctypes.byref(st)), "sf_file_stamp_fd")
    return st


def index_fd_blocks(fd: int, offsets, sizes, stamp: FileStamp = None) -> Tuple[np.ndarray, bytes]:
    """An explicit list over the regular file OPEN on fd (sf_index_fd_blocks):
    the chunker's own handle, read again with pread, so the bytes hashed are
    the file the chunker cut even if another file was renamed over its path.
    `stamp` (file_stamp before chunking): SfError SF_EAGAIN if the file
    differs from it at the call or changes before the last window is read."""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    szs = np.ascontiguousarray(sizes, dtype=np.uint32).reshape(-1)
    if offs.size != szs.size:
        raise ValueError("offsets and sizes differ in length")
    n = offs.size
    out = np.zeros(max(n, 1), SIG_DTYPE)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_fd_blocks(int(fd), ctypes.byref(stamp) if stamp is not None else None,
                                   offs.ctypes.data if n else None, szs.ctypes.data if n else None, n,
                                   out.ctypes.data_as(ctypes.POINTER(BlockSig)), bh),
          "sf_index_fd_blocks")
    return out[:n], bytes(bh)


def index_fd_fixed(fd: int, block_size: int, stamp: FileStamp = None) -> Tuple[np.ndarray, bytes]:
    """Fixed tiling of the regular file open on fd (sf_index_fd_fixed), with
    the same stamp checks as index_fd_blocks."""
    size = os.fstat(int(fd)).st_size
    n = (size + block_size - 1) // block_size if size else 0
    out = np.zeros(max(n, 1), SIG_DTYPE)
    nout = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_fd_fixed(int(fd), ctypes.byref(stamp) if stamp is not None else None, block_size,
                                  out.ctypes.data_as(ctypes.POINTER(BlockSig)), n, ctypes.byref(nout), bh),
          "sf_index_fd_fixed")
    return out[:nout.value], bytes(bh)


def release_cache() -> None:
    """Free the streams and buffers the host entry points keep between calls
    (sf_release_host_cache)."""
    check(lib().sf_release_host_cache(), "sf_release_host_cache")


def index_file(path, block_size: int) -> Tuple[np.ndarray, bytes]:
    """Signatures of a file on disk + its blocks_hash.  A regular file that
    grows between the sizing stat and the call (SF_ENOSPC with the new need)
    is indexed again with room for it, as index_files does.  Anything else
    that opens (a FIFO, a character device) is read to EOF through index_fd:
    sized by a stat, its bytes would be consumed by a call whose rows did
    not fit."""
    st = os.stat(path)
    if not stat.S_ISREG(st.st_mode):
        fd = os.open(path, os.O_RDONLY)
        try:
            return index_fd(fd, block_size)
        finally:
            os.close(fd)
    size = st.st_size
    n = (size + block_size - 1) // block_size if size else 0
    nout = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    for _attempt in range(4):
        out = np.zeros(max(n, 1), SIG_DTYPE)
        rc = lib().sf_index_file(os.fsencode(path), block_size, out.ctypes.data_as(ctypes.POINTER(BlockSig)),
                                 n, ctypes.byref(nout), bh)
        if rc == SF_ENOSPC and nout.value > n:
            n = nout.value
            continue
        break
    check(rc, "sf_index_file")
    return out[:nout.value], bytes(bh)


def index_file_range(path, start: int, length: int, block_size: int) -> np.ndarray:
    """Rows of bytes [start, start+length) of a file (one shard of it; start a
    multiple of block_size), offsets relative to the file (sf_index_file_range)."""
    n = (length + block_size - 1) // block_size if length else 0
    out = np.zeros(max(n, 1), SIG_DTYPE)
    nout = ctypes.c_uint64(0)
    check(lib().sf_index_file_range(os.fsencode(path), start, length, block_size,
                                    out.ctypes.data_as(ctypes.POINTER(BlockSig)), n, ctypes.byref(nout)),
          "sf_index_file_range")
    return out[:nout.value]


def index_fd(fd: int, block_size: int) -> Tuple[np.ndarray, bytes]:
    """Signatures of everything readable from an open descriptor (a pipe, a
    FIFO, ...) to EOF + its blocks_hash (sf_index_fd: sequential route, rows
    in a library-grown buffer)."""
    rows = ctypes.POINTER(BlockSig)()
    nout = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_fd(int(fd), block_size, ctypes.byref(rows), ctypes.byref(nout), bh), "sf_index_fd")
    try:
        n = nout.value
        out = np.zeros(n, SIG_DTYPE)
        if n:
            ctypes.memmove(out.ctypes.data, rows, n * SIG_DTYPE.itemsize)
    finally:
        lib().sf_free_rows(rows)
    return out, bytes(bh)


def index_files(paths: Sequence, block_size: int, stage_bytes: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Many files through one pipeline (sf_index_files): what index_path does
    with one index_file per file (src/index.rs:685-715, 610-659).

    Returns (rows, first_row, blocks_hashes): file k's rows are
    rows[first_row[k]:first_row[k+1]] (offsets relative to the file), its
    blocks_hash is blocks_hashes[k] (uint8[20]).  stage_bytes = 0 uses the
    library default (256 MiB).  An unreadable file raises SfError naming it."""
    n = len(paths)
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(n, 1))(*enc)
    first = np.zeros(n + 1, np.uint64)
    hashes = np.zeros((max(n, 1), 20), np.uint8)
    need, bad = ctypes.c_uint64(0), ctypes.c_uint32(0)
    cap = 0
    while True:  # a file may grow between the sizing call and the real one
        out = np.zeros(max(cap, 1), SIG_DTYPE)
        rc = lib().sf_index_files(arr, n, block_size, stage_bytes, out.ctypes.data_as(ctypes.POINTER(BlockSig)),
                                  cap, first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), hashes.ctypes.data,
                                  ctypes.byref(need), ctypes.byref(bad))
        if rc == SF_ENOSPC and need.value > cap:
            cap = need.value
            continue
        where = f"sf_index_files: {os.fsdecode(enc[bad.value])}" if rc in (SF_EIO, SF_EINVAL) and bad.value < n \
            else "sf_index_files"
        check(rc, where)
        return out[:need.value], first, hashes[:n]


def index_fds_blocks(fds: Sequence[int], lists: Sequence[Tuple[object, object]], stamps: Sequence = None,
                     stage_bytes: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Many files in the reference's default mode through one pipeline
    (sf_index_fds_blocks): file k is the regular file open on fds[k], cut by
    the caller's chunker into lists[k] = (offsets, sizes); stamps[k]
    (file_stamp before chunking, or None for all) is checked when the call
    starts and after the file's last window is read.

    Returns (rows, first_row, blocks_hashes, status): file k's rows are
    rows[first_row[k]:first_row[k+1]], its blocks_hash blocks_hashes[k], and
    status[k] its own result (SF_OK, or SF_EAGAIN / SF_ERANGE / SF_EINVAL /
    SF_EIO for that file alone: its rows are not valid, it must be cut
    again).  A per-file failure does not raise; a call-level one (device,
    arguments) does."""
    n = len(fds)
    if len(lists) != n or (stamps is not None and len(stamps) != n):
        raise ValueError("fds, lists and stamps differ in length")
    offs, szs = [], []
    for o, z in lists:
        o = np.ascontiguousarray(o, dtype=np.uint64).reshape(-1)
        z = np.ascontiguousarray(z, dtype=np.uint32).reshape(-1)
        if o.size != z.size:
            raise ValueError("offsets and sizes differ in length")
        offs.append(o)
        szs.append(z)
    nb = np.array([o.size for o in offs] or [0], np.uint64)
    po = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data if o.size else None for o in offs])
    pz = (ctypes.c_void_p * max(n, 1))(*[z.ctypes.data if z.size else None for z in szs])
    fda = np.array(list(fds) or [0], np.int32)
    st = None
    if stamps is not None:
        st = (FileStamp * max(n, 1))(*stamps)
    total = int(nb[:n].sum()) if n else 0
    out = np.zeros(max(total, 1), SIG_DTYPE)
    first = np.zeros(n + 1, np.uint64)
    hashes = np.zeros((max(n, 1), 20), np.uint8)
    status = np.zeros(max(n, 1), np.int32)
    bad = ctypes.c_uint32(0)
    rc = lib().sf_index_fds_blocks(fda.ctypes.data, st, n, po, pz, nb.ctypes.data, stage_bytes,
                                   out.ctypes.data_as(ctypes.POINTER(BlockSig)), total,
                                   first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), hashes.ctypes.data,
                                   status.ctypes.data, ctypes.byref(bad))
    if rc != 0 and not (n and bad.value < n and status[bad.value] == rc):
        check(rc, "sf_index_fds_blocks")
    return out[:total], first, hashes[:n], status[:n]


def cut_fd(fd: int, ops, threads: int = 0, stamp: FileStamp = None) -> Tuple[np.ndarray, np.ndarray]:
    """The caller's chunker over the regular file open on fd (sf_cut_fd):
    ``ops`` is the address of an sf_chunker_ops (a native chunker; see
    examples/zpaq_standin_ops.c).  Split over ``threads`` threads (0: the
    library's reader count) and joined so that the boundaries are exactly the
    sequential ones.  Returns (offsets uint64, sizes uint32); raises
    SfError(SF_EAGAIN) if the file changed (against ``stamp`` if given, and
    while it was cut)."""
    po, pz = ctypes.c_void_p(), ctypes.c_void_p()
    n = ctypes.c_uint64(0)
    check(lib().sf_cut_fd(fd, ctypes.byref(stamp) if stamp is not None else None, ops, threads,
                          ctypes.byref(po), ctypes.byref(pz), ctypes.byref(n)), "sf_cut_fd")
    try:
        k = n.value
        offs = np.ctypeslib.as_array(ctypes.cast(po, ctypes.POINTER(ctypes.c_uint64)), (k,)).copy() if k else \
            np.zeros(0, np.uint64)
        sizes = np.ctypeslib.as_array(ctypes.cast(pz, ctypes.POINTER(ctypes.c_uint32)), (k,)).copy() if k else \
            np.zeros(0, np.uint32)
    finally:
        lib().sf_free_cuts(po)
        lib().sf_free_cuts(pz)
    return offs, sizes


def index_fd_cut(fd: int, ops, threads: int = 0, stamp: FileStamp = None) -> Tuple[np.ndarray, bytes]:
    """index_file in the default mode for the regular file open on fd, the
    caller's chunker (``ops``: the address of an sf_chunker_ops) on
    ``threads`` threads, the file read once (sf_index_fd_cut).  Returns
    (rows, blocks_hash); SfError(SF_EAGAIN) if the file changed."""
    p = ctypes.POINTER(BlockSig)()
    n = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_fd_cut(fd, ctypes.byref(stamp) if stamp is not None else None, ops, threads,
                                ctypes.byref(p), ctypes.byref(n), bh), "sf_index_fd_cut")
    try:
        rows = np.zeros(n.value, SIG_DTYPE)
        if n.value:
            ctypes.memmove(rows.ctypes.data, p, n.value * SIG_DTYPE.itemsize)
    finally:
        lib().sf_free_rows(p)
    return rows, bytes(bh)


def shard_range(file_len: int, block_size: int, n_shards: int, shard: int) -> Tuple[int, int]:
    """sf_shard_range: (start, length) of shard `shard` of n_shards (the
    partition of the multi-device forms)."""
    s, n = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().sf_shard_range(file_len, block_size, n_shards, shard, ctypes.byref(s), ctypes.byref(n)),
          "sf_shard_range")
    return s.value, n.value


def index_file_multi(path, block_size: int, n_devices: int = 0) -> Tuple[np.ndarray, bytes]:
    """One regular file on N devices of this process (sf_index_file_multi):
    shard r read and hashed on device r by a host thread of its own, rows in
    file order, blocks_hash over all digests.  n_devices = 0: every visible
    device."""
    size = os.stat(path).st_size
    n = (size + block_size - 1) // block_size if size else 0
    need = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    for _attempt in range(4):  # the file may grow between the stat and the call
        out = np.zeros(max(n, 1), SIG_DTYPE)
        rc = lib().sf_index_file_multi(os.fsencode(path), block_size, n_devices,
                                       out.ctypes.data_as(ctypes.POINTER(BlockSig)), n, ctypes.byref(need), bh)
        if rc == SF_ENOSPC and need.value > n:
            n = need.value
            continue
        break
    check(rc, f"sf_index_file_multi({os.fsdecode(path)})")
    return out[:need.value], bytes(bh)


def blocks_hash(digests) -> bytes:
    """compute_blocks_hash: SHA-1 over the 20-byte digests in order."""
    d = _u8(digests)
    if d.size % 20:
        raise ValueError("digest buffer length is not a multiple of 20")
    out = (ctypes.c_uint8 * 20)()
    check(lib().sf_blocks_hash(d.ctypes.data if d.size else None, d.size // 20, out), "sf_blocks_hash")
    return bytes(out)


def sha1(data) -> bytes:
    a = _u8(data)
    out = (ctypes.c_uint8 * 20)()
    check(lib().sf_sha1_host(a.ctypes.data if a.size else None, a.size, out), "sf_sha1_host")
    return bytes(out)


def rows_to_tuples(rows: np.ndarray) -> List[Tuple[int, int, bytes]]:
    return [(int(r["offset"]), int(r["size"]), bytes(r["sha1"])) for r in rows]
