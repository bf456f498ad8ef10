"""The reference's wire messages for signature tables (src/sync/ssh/proto.rs).

``write_message`` mirrors proto.rs:139-187 byte for byte for the messages a
source sends about indexed files: FILE_ENTRY (name, size, blocks_hash),
END_FILES, FILE_START, FILE_BLOCK (digest, size), FILE_END, plus GET_FILE,
GET_BLOCK, BLOCK_DATA and COMPLETE.  ``file_blocks_device`` produces a whole
file's FILE_BLOCK run on the GPU straight from the HBM digest table
(C-ABI sf_wire_file_blocks_device), as FsSource streams it after FILE_START
(src/sync/fs.rs:217-233).  ``Parser`` is the receiving side (proto.rs:189-477):
the incremental framing parser a destination runs over the same bytes."""
from __future__ import annotations

import ctypes
import re
from typing import List, Optional, Tuple

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


class ProtocolError(ValueError):
    """proto::Error: the byte stream is not a valid message sequence."""


# Framing limits of the reference parser (proto.rs:249-251).
COMMAND_MAX, FILENAME_MAX, SIZE_MAX = 20, 100, 15
_USIZE = re.compile(rb"\+?[0-9]+")  # what Rust's usize::from_str accepts


class Parser:
    """Incremental message parser, the receiving side of write_message
    (proto.rs:189-477).  ``receive(data)`` appends bytes and returns every
    message now complete, as (kind, *fields) tuples in write_message's
    argument order; an incomplete tail is kept for the next call.  Malformed
    input raises ProtocolError with the reference's message: a line longer
    than its limit (command 20, filename 100, size 15 bytes), a digest or
    data field not followed by a newline, a size that is not a usize, an
    unknown command."""

    def __init__(self):
        self._buf = bytearray()

    def receive(self, data) -> List[Tuple]:
        self._buf += bytes(data)
        out, pos = [], 0
        while True:
            r = self._one(pos)
            if r is None:
                break
            msg, pos = r
            out.append(msg)
        del self._buf[:pos]
        return out

    def _line(self, p, limit, err):
        i = self._buf.find(b"\n", p, min(len(self._buf), p + limit + 1))
        if i >= 0:
            return bytes(self._buf[p:i]), i + 1
        if len(self._buf) - p >= limit:
            raise ProtocolError(err)
        return None

    def _exact(self, p, n, err):
        if len(self._buf) - p < n + 1:
            return None
        if self._buf[p + n] != 0x0A:
            raise ProtocolError(err)
        return bytes(self._buf[p:p + n]), p + n + 1

    @staticmethod
    def _usize(b, err):
        if not _USIZE.fullmatch(b) or int(b) >= 1 << 64:
            raise ProtocolError(err)
        return int(b)

    def _one(self, p):
        if p >= len(self._buf):
            return None
        r = self._line(p, COMMAND_MAX, "Unterminated command")
        if r is None:
            return None
        cmd, p = r
        if cmd in (b"END_FILES", b"FILE_END", b"COMPLETE"):
            return ({b"END_FILES": ("EndFiles",), b"FILE_END": ("FileEnd",), b"COMPLETE": ("Complete",)}[cmd], p)
        if cmd in (b"GET_FILE", b"FILE_START"):
            r = self._line(p, FILENAME_MAX, "Unterminated filename")
            if r is None:
                return None
            return ("GetFile" if cmd == b"GET_FILE" else "FileStart", r[0]), r[1]
        if cmd == b"FILE_ENTRY":
            r = self._line(p, FILENAME_MAX, "Unterminated filename")
            if r is None:
                return None
            name, p = r
            r = self._line(p, SIZE_MAX, "Unterminated size")
            if r is None:
                return None
            size = self._usize(r[0], "Invalid file size")
            r = self._exact(r[1], 20, "Unterminated digest")
            if r is None:
                return None
            return ("FileEntry", name, size, HashDigest(r[0])), r[1]
        if cmd in (b"FILE_BLOCK", b"GET_BLOCK", b"BLOCK_DATA"):
            r = self._exact(p, 20, "Unterminated digest")
            if r is None:
                return None
            digest, p = HashDigest(r[0]), r[1]
            if cmd == b"GET_BLOCK":
                return ("GetBlock", digest), p
            r = self._line(p, SIZE_MAX, "Unterminated size" if cmd == b"FILE_BLOCK" else "Unterminated length")
            if r is None:
                return None
            size = self._usize(r[0], "Invalid block size" if cmd == b"FILE_BLOCK" else "Invalid block length")
            if cmd == b"FILE_BLOCK":
                return ("FileBlock", digest, size), r[1]
            r = self._exact(r[1], size, "Invalid data end byte")
            if r is None:
                return None
            return ("BlockData", digest, r[0]), r[1]
        raise ProtocolError("Unknown command")


def file_blocks_device(digests, block_size: int, file_len: int, stream=None):
    """FILE_BLOCK messages for every block of a fixed-tiled file, built on the
    device from a uint8[n, 20] HBM digest table -> uint8 HBM tensor."""
    from .device import _on, _require_device
    import torch
    _require_device(digests, "digests", torch.uint8)
    n = digests.shape[0]
    need = ctypes.c_uint64(0)
    with _on(digests.device, stream):
        s = torch.cuda.current_stream(digests.device).cuda_stream
        rc = lib().sf_wire_file_blocks_device(None, n, block_size, file_len, None, 0, ctypes.byref(need), s)
        if rc not in (0, -28):
            check(rc, "sf_wire_file_blocks_device")
        out = torch.empty(need.value, dtype=torch.uint8, device=digests.device)
        if need.value:
            check(lib().sf_wire_file_blocks_device(digests.data_ptr(), n, block_size, file_len, out.data_ptr(),
                                                   out.numel(), ctypes.byref(need), s), "sf_wire_file_blocks_device")
    return out


def _check_sizes(torch, sizes, digests):
    if (not isinstance(sizes, torch.Tensor) or sizes.numel() != digests.shape[0]
            or sizes.dtype not in (torch.int32, torch.uint32) or sizes.device != digests.device):
        raise ValueError("sizes must be one 32-bit size per digest, on the digests' device")


def blocks_device(digests, sizes, stream=None):
    """FILE_BLOCK messages for an explicit block list (content-defined
    blocks, each with its own size), built on the device from a uint8[n, 20]
    HBM digest table and an int32/uint32[n] HBM size array (bit pattern taken
    as uint32) -> uint8 HBM tensor (sf_wire_blocks_device)."""
    from .device import _on, _require_device
    import torch
    _require_device(digests, "digests", torch.uint8)
    n = digests.shape[0]
    _check_sizes(torch, sizes, digests)
    need = ctypes.c_uint64(0)
    with _on(digests.device, stream):
        sizes = sizes.contiguous()  # on the stream the kernels run on
        s = torch.cuda.current_stream(digests.device).cuda_stream
        rc = lib().sf_wire_blocks_device(None, sizes.data_ptr() if n else None, n, None, 0, ctypes.byref(need), s)
        if rc not in (0, -28):
            check(rc, "sf_wire_blocks_device")
        out = torch.empty(need.value, dtype=torch.uint8, device=digests.device)
        if need.value:
            check(lib().sf_wire_blocks_device(digests.data_ptr(), sizes.data_ptr(), n, out.data_ptr(), out.numel(),
                                              ctypes.byref(need), s), "sf_wire_blocks_device")
    return out


def blocks_to_fd(digests, sizes, fd: int, stream=None) -> int:
    """The explicit list's FILE_BLOCK run written to a file descriptor, built
    on the device in chunks and streamed back (sf_wire_blocks_fd).  Returns
    the bytes written."""
    from .device import _on, _require_device
    import torch
    _require_device(digests, "digests", torch.uint8)  # an HBM table: the kernels read it on its device
    n = digests.shape[0]
    _check_sizes(torch, sizes, digests)
    out = ctypes.c_uint64(0)
    # the library's streams and chunk buffers are the current device's
    # (HostLease keys on hipGetDevice): enter the digests' device
    with _on(digests.device, stream):
        sizes = sizes.contiguous()  # on the stream the chunks are built after
        s = torch.cuda.current_stream(digests.device).cuda_stream
        check(lib().sf_wire_blocks_fd(digests.data_ptr() if n else None, sizes.data_ptr() if n else None, n,
                                      int(fd), ctypes.byref(out), s), "sf_wire_blocks_fd")
    return out.value


def file_blocks_to_fd(digests, block_size: int, file_len: int, fd: int, stream=None) -> int:
    """The FILE_BLOCK run of a fixed-tiled file written to a file descriptor
    (an SSH pipe or a file): built on the device in chunks, streamed back by
    DMA and written while the next chunk is built (sf_wire_file_blocks_fd).
    Returns the bytes written."""
    from .device import _on, _require_device
    import torch
    _require_device(digests, "digests", torch.uint8)
    n = digests.shape[0]
    out = ctypes.c_uint64(0)
    with _on(digests.device, stream):
        s = torch.cuda.current_stream(digests.device).cuda_stream
        check(lib().sf_wire_file_blocks_fd(digests.data_ptr() if n else None, n, block_size, file_len, fd,
                                           ctypes.byref(out), s), "sf_wire_file_blocks_fd")
    return out.value
