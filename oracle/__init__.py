"""CPU oracle for syncfast's block-signature indexing path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this package, and only as the
checker (or the timed CPU baseline) -- never as the product path.  The
product (``syncfast_amd``) does not import it and has no CPU fallback.

Two restatements live here:

* ``libsf_oracle.so`` (``sf_oracle.c``, plain C): SHA-1 per block, the
  ``index_file`` loop over a fixed tiling or an explicit boundary list,
  ``compute_blocks_hash`` and the splitmix64 generator.  Cites
  /root/reference/src/index.rs:621-682 and src/lib.rs:72-90.
* pure-Python helpers built on ``hashlib`` (small cases and golden-vector
  generation).  ``hashlib.sha1`` is the same function as the reference's
  ``sha1 0.6.0`` crate: the reference's own KATs (src/index.rs:765-792,
  src/lib.rs:184-195) are reproduced bit for bit in tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsf_oracle.so")
_BASE_PATH = os.path.join(_HERE, "build", "libsf_baseline.so")
_lib = None
_base = None

GAMMA = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1


def build(force: bool = False) -> str:
    """Compile sf_oracle.c with gcc (no reference sources involved)."""
    src = os.path.join(_HERE, "sf_oracle.c")
    if (force or not os.path.exists(_LIB_PATH) or not os.path.exists(_BASE_PATH)
            or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.sfo_sha1.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.sfo_num_blocks.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.sfo_num_blocks.restype = ctypes.c_uint64
        L.sfo_index_fixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, u8p, u8p]
        L.sfo_index_fixed.restype = ctypes.c_uint64
        L.sfo_index_blocks.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, u8p]
        L.sfo_blocks_hash.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.sfo_index_fixed_mt.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_int]
        L.sfo_index_fixed_mt.restype = ctypes.c_uint64
        L.sfo_fill_splitmix.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.sfo_adler32.argtypes = [u8p, ctypes.c_uint64]
        L.sfo_adler32.restype = ctypes.c_uint32
        L.sfo_adler_fixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, u8p]
        L.sfo_adler_blocks.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, u8p]
        _lib = L
    return _lib


def baseline_lib() -> ctypes.CDLL:
    """libsf_baseline.so: the SHA-NI CPU baseline (bench.py only)."""
    global _base
    if _base is None:
        if not os.path.exists(_BASE_PATH):
            build()
        L = ctypes.CDLL(_BASE_PATH)
        L.sfb_has_shani.argtypes = []
        L.sfb_has_shani.restype = ctypes.c_int
        L.sfb_index_fixed_shani.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_int]
        L.sfb_index_fixed_shani.restype = ctypes.c_uint64
        L.sfb_zpaq_cut.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.sfb_zpaq_cut.restype = ctypes.c_uint64
        L.sfb_zpaq_index.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_int]
        L.sfb_zpaq_index.restype = ctypes.c_uint64
        _base = L
    return _base


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(bytes(data), dtype=np.uint8)


# ------------------------------------------------------------------ C oracle

def sha1(data) -> bytes:
    a = _as_u8(data)
    out = np.zeros(20, np.uint8)
    lib().sfo_sha1(_ptr(a), a.size, _ptr(out))
    return out.tobytes()


def index_fixed(data, block_size: int):
    """(offsets u64[n], sizes u32[n], digests u8[n,20]) for a fixed tiling."""
    a = _as_u8(data)
    n = lib().sfo_num_blocks(a.size, block_size)
    offs = np.zeros(n, np.uint64)
    sizes = np.zeros(n, np.uint32)
    dig = np.zeros((n, 20), np.uint8)
    lib().sfo_index_fixed(_ptr(a), a.size, block_size, _ptr(offs), _ptr(sizes), _ptr(dig))
    return offs, sizes, dig


def index_fixed_mt(data, block_size: int, threads: int) -> np.ndarray:
    a = _as_u8(data)
    n = lib().sfo_num_blocks(a.size, block_size)
    dig = np.zeros((n, 20), np.uint8)
    lib().sfo_index_fixed_mt(_ptr(a), a.size, block_size, _ptr(dig), threads)
    return dig


def index_fixed_shani(data, block_size: int, threads: int = 1) -> np.ndarray:
    """Fixed tiling with the product's host SHA-1 (SHA-NI): the strongest CPU
    baseline for bench.py, not a checker."""
    a = _as_u8(data)
    n = lib().sfo_num_blocks(a.size, block_size)
    dig = np.zeros((n, 20), np.uint8)
    baseline_lib().sfb_index_fixed_shani(_ptr(a), a.size, block_size, _ptr(dig), threads)
    return dig


def zpaq_standin_sizes(data) -> np.ndarray:
    """Block sizes of the ZPAQ-form STAND-IN chunker (examples/zpaq_standin.h,
    13 bits, 32 KiB cap): the crate's per-byte work for the configs[0]
    baseline, not the reference's boundaries."""
    a = _as_u8(data)
    cap = a.size // 1024 + 16
    out = np.zeros(cap, np.uint32)
    n = int(baseline_lib().sfb_zpaq_cut(_ptr(a), a.size, _ptr(out), cap))
    if n > cap:  # more than one block per KiB: cut again into a list that fits
        out = np.zeros(n, np.uint32)
        baseline_lib().sfb_zpaq_cut(_ptr(a), a.size, _ptr(out), n)
    return out[:n]


def zpaq_standin_index(data, shani: bool) -> np.ndarray:
    """The stand-in chunker with each block SHA-1'd as it is cut, in one pass
    (the reference's default index_file loop, src/index.rs:629-647), on the
    calling thread: digests u8[n, 20]."""
    a = _as_u8(data)
    cap = a.size // 1024 + 16
    dig = np.zeros((cap, 20), np.uint8)
    n = int(baseline_lib().sfb_zpaq_index(_ptr(a), a.size, _ptr(dig), cap, int(shani)))
    if n > cap:
        dig = np.zeros((n, 20), np.uint8)
        baseline_lib().sfb_zpaq_index(_ptr(a), a.size, _ptr(dig), n, int(shani))
    return dig[:n]


def has_shani() -> bool:
    return bool(baseline_lib().sfb_has_shani())


def index_blocks(data, offsets, sizes) -> np.ndarray:
    a = _as_u8(data)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    sz = np.ascontiguousarray(sizes, dtype=np.uint32)
    assert offs.shape == sz.shape
    if offs.size:
        assert int((offs + sz.astype(np.uint64)).max()) <= a.size
    dig = np.zeros((offs.size, 20), np.uint8)
    lib().sfo_index_blocks(_ptr(a), _ptr(offs), _ptr(sz), offs.size, _ptr(dig))
    return dig


def blocks_hash(digests) -> bytes:
    d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
    assert d.size % 20 == 0
    out = np.zeros(20, np.uint8)
    lib().sfo_blocks_hash(_ptr(d), d.size // 20, _ptr(out))
    return out.tobytes()


def adler32(data) -> int:
    """zlib Adler-32 of a byte range (checker for the opt-in weak sum)."""
    a = _as_u8(data)
    return int(lib().sfo_adler32(_ptr(a), a.size))


def adler_fixed(data, block_size: int) -> np.ndarray:
    a = _as_u8(data)
    n = lib().sfo_num_blocks(a.size, block_size)
    out = np.zeros(n, np.uint32)
    lib().sfo_adler_fixed(_ptr(a), a.size, block_size, _ptr(out))
    return out


def adler_blocks(data, offsets, sizes) -> np.ndarray:
    a = _as_u8(data)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    sz = np.ascontiguousarray(sizes, dtype=np.uint32)
    out = np.zeros(offs.size, np.uint32)
    lib().sfo_adler_blocks(_ptr(a), _ptr(offs), _ptr(sz), offs.size, _ptr(out))
    return out


def block_lookup(table, present, queries) -> np.ndarray:
    """Index::get_block (src/index.rs:77-103) for many digests at once: for
    each query the first row (rowid order) whose digest equals it and whose
    present flag is set, or -1 -- the row SQLite returns first from
    idx_blocks_hash, (hash, rowid) order.  ``table`` uint8[n, 20] in rowid
    order, ``present`` bool[n] or None (all present), ``queries`` uint8[m, 20].
    Sort-based (numpy), so it handles millions of rows."""
    t = np.ascontiguousarray(np.asarray(table, np.uint8).reshape(-1, 20))
    q = np.ascontiguousarray(np.asarray(queries, np.uint8).reshape(-1, 20))
    rows = np.arange(t.shape[0], dtype=np.int64)
    if present is not None:
        keep = np.asarray(present).astype(bool).reshape(-1)
        t, rows = t[keep], rows[keep]
    out = np.full(q.shape[0], -1, np.int64)
    if t.shape[0] == 0 or q.shape[0] == 0:
        return out
    key = np.dtype((np.void, 20))
    tk = t.view(key).reshape(-1)
    uniq, first = np.unique(tk, return_index=True)  # first occurrence = smallest row among kept rows
    qk = q.view(key).reshape(-1)
    pos = np.searchsorted(uniq, qk)
    pos_c = np.minimum(pos, uniq.shape[0] - 1)
    hit = (pos < uniq.shape[0]) & (uniq[pos_c] == qk)
    out[hit] = rows[first[pos_c[hit]]]
    return out


def splitmix_bytes(length: int, seed: int, start: int = 0) -> np.ndarray:
    out = np.empty(length, np.uint8)
    lib().sfo_fill_splitmix(_ptr(out), length, seed & MASK64, start)
    return out


# ------------------------------------------------------- pure-Python oracle

def py_index_blocks(data: bytes, offsets, sizes) -> list:
    """hashlib restatement of src/index.rs:629-646 for an explicit boundary list."""
    return [hashlib.sha1(data[o:o + s]).digest() for o, s in zip(offsets, sizes)]


def py_index_fixed(data: bytes, block_size: int):
    n = (len(data) + block_size - 1) // block_size if block_size else 0
    offs = [i * block_size for i in range(n)]
    sizes = [min(block_size, len(data) - o) for o in offs]
    return offs, sizes, py_index_blocks(data, offs, sizes)


def py_blocks_hash(digests) -> bytes:
    """src/index.rs:661-682."""
    h = hashlib.sha1()
    for d in digests:
        h.update(bytes(d))
    return h.digest()


def py_splitmix_bytes(length: int, seed: int, start: int = 0) -> bytes:
    """Pure-Python splitmix64 stream (cross-checks the C generator)."""
    out = bytearray()
    w0 = start >> 3
    nw = ((start + length + 7) >> 3) - w0
    for i in range(w0, w0 + nw):
        z = (seed + (i + 1) * GAMMA) & MASK64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    skip = start - (w0 << 3)
    return bytes(out[skip:skip + length])


def kat_input() -> bytes:
    """The reference KAT file, src/index.rs:749-755."""
    return b"".join(b"Line %d\n" % (i + 1) for i in range(2000)) + b"Test content\n" * 2000
