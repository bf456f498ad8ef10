"""Host-memory entry points (bytes in host RAM or on disk -> signature rows).

These are the end-to-end forms of the path (the reference reads files,
src/index.rs:615): the C-ABI stages the bytes through pinned buffers, runs the
HIP kernel, and copies the rows back.  ``blocks_hash`` is the host stage of
compute_blocks_hash (src/index.rs:661-682).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Tuple

import numpy as np

from ._lib import BlockSig, check, lib

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


def index_file(path, block_size: int) -> Tuple[np.ndarray, bytes]:
    """Signatures of a file on disk + its blocks_hash."""
    size = os.path.getsize(path)
    n = (size + block_size - 1) // block_size if size else 0
    out = np.zeros(max(n, 1), SIG_DTYPE)
    nout = ctypes.c_uint64(0)
    bh = (ctypes.c_uint8 * 20)()
    check(lib().sf_index_file(os.fsencode(path), block_size, out.ctypes.data_as(ctypes.POINTER(BlockSig)),
                              n, ctypes.byref(nout), bh),
          "sf_index_file")
    return out[:nout.value], bytes(bh)


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
