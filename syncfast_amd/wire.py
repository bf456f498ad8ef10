"""The reference's wire messages for signature tables (src/sync/ssh/proto.rs).

``write_message`` mirrors proto.rs:139-187 byte for byte for the messages a
source sends about indexed files: FILE_ENTRY (name, size, blocks_hash),
END_FILES, FILE_START, FILE_BLOCK (digest, size), FILE_END, plus GET_FILE,
GET_BLOCK, BLOCK_DATA and COMPLETE.  ``file_blocks_device`` produces a whole
file's FILE_BLOCK run on the GPU straight from the HBM digest table
(C-ABI sf_wire_file_blocks_device), as FsSource streams it after FILE_START
(src/sync/fs.rs:217-233)."""
from __future__ import annotations

import ctypes
from typing import Optional

from ._lib import check, lib
from .digest import HashDigest


def _d(d) -> bytes:
    return d.bytes if isinstance(d, HashDigest) else bytes(d)


def write_message(kind: str, *args) -> bytes:
    """One message, exactly as proto.rs:139-187 writes it."""
    if kind == "FileEntry":
        name, size, digest = args
        return b"FILE_ENTRY\n" + bytes(name) + b"\n%d\n" % size + _d(digest) + b"\n"
    if kind == "EndFiles":
        return b"END_FILES\n"
    if kind == "GetFile":
        return b"GET_FILE\n" + bytes(args[0]) + b"\n"
    if kind == "FileStart":
        return b"FILE_START\n" + bytes(args[0]) + b"\n"
    if kind == "FileBlock":
        digest, size = args
        return b"FILE_BLOCK\n" + _d(digest) + b"\n%d\n" % size
    if kind == "FileEnd":
        return b"FILE_END\n"
    if kind == "GetBlock":
        return b"GET_BLOCK\n" + _d(args[0]) + b"\n"
    if kind == "BlockData":
        digest, data = args
        return b"BLOCK_DATA\n" + _d(digest) + b"\n%d\n" % len(data) + bytes(data) + b"\n"
    if kind == "Complete":
        return b"COMPLETE\n"
    raise ValueError(kind)


def file_blocks_device(digests, block_size: int, file_len: int, stream=None):
    """FILE_BLOCK messages for every block of a fixed-tiled file, built on the
    device from a uint8[n, 20] HBM digest table -> uint8 HBM tensor."""
    import torch
    n = digests.shape[0]
    need = ctypes.c_uint64(0)
    s = (stream or torch.cuda.current_stream(digests.device)).cuda_stream
    rc = lib().sf_wire_file_blocks_device(None, n, block_size, file_len, None, 0, ctypes.byref(need), s)
    if rc not in (0, -28):
        check(rc, "sf_wire_file_blocks_device")
    out = torch.empty(need.value, dtype=torch.uint8, device=digests.device)
    if need.value:
        check(lib().sf_wire_file_blocks_device(digests.data_ptr(), n, block_size, file_len, out.data_ptr(),
                                               out.numel(), ctypes.byref(need), s), "sf_wire_file_blocks_device")
    return out


def file_blocks_to_fd(digests, block_size: int, file_len: int, fd: int, stream=None) -> int:
    """The FILE_BLOCK run of a fixed-tiled file written to a file descriptor
    (an SSH pipe or a file): built on the device in chunks, streamed back by
    DMA and written while the next chunk is built (sf_wire_file_blocks_fd).
    Returns the bytes written."""
    import torch
    n = digests.shape[0]
    s = (stream or torch.cuda.current_stream(digests.device)).cuda_stream
    out = ctypes.c_uint64(0)
    with torch.cuda.device(digests.device):
        check(lib().sf_wire_file_blocks_fd(digests.data_ptr() if n else None, n, block_size, file_len, fd,
                                           ctypes.byref(out), s), "sf_wire_file_blocks_fd")
    return out.value
