"""GPU: the sequential route for inputs that cannot seek.

The reference's index_file streams whatever File::open accepts -- a FIFO, a
character device (src/index.rs:615,625).  sf_index_file takes such a path
directly (rows within cap), and sf_index_fd reads any descriptor to EOF into
a library-grown row buffer.  Rows and blocks_hash must equal the oracle's
for the same bytes, across stage boundaries (SF_TEST_STREAM_STAGE_MIB=1 makes the
stages small so a few MiB cross several)."""
import ctypes
import os
import threading

import numpy as np
import pytest

import oracle
from syncfast_amd import host
from syncfast_amd._lib import SF_ENOSPC, BlockSig, lib

pytestmark = pytest.mark.gpu


def _writer(path_or_fd, payload, chunk=1 << 16):
    def run():
        if isinstance(path_or_fd, int):
            w = os.fdopen(path_or_fd, "wb")
        else:
            w = open(path_or_fd, "wb")
        with w:
            for i in range(0, len(payload), chunk):  # many small writes: short reads on the other side
                w.write(payload[i:i + chunk])
    th = threading.Thread(target=run)
    th.start()
    return th


def _check(rows, bh, data, bs):
    offs, sizes, want = oracle.index_fixed(data, bs)
    assert len(rows) == len(want)
    if len(want):
        assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
        assert np.array_equal(np.stack([r["sha1"] for r in rows]), want)
    assert bh == oracle.blocks_hash(want)


@pytest.mark.parametrize("n,bs,stage_mib", [(0, 4096, ""), (1, 4096, ""), (3 * 4096 + 1234, 4096, ""),
                                           ((5 << 20) + 777, 4096, "1"), ((3 << 20) + 1, 65536, "1"),
                                           ((2 << 20), 1000, "1"), (40 << 20, 4096, "")])
def test_index_fd_pipe(gpu, n, bs, stage_mib, knobs):
    if stage_mib:
        knobs.set("SF_TEST_STREAM_STAGE_MIB", int(stage_mib))
    data = oracle.splitmix_bytes(n, 700 + n % 97)
    r, w = os.pipe()
    th = _writer(w, data.tobytes())
    try:
        rows, bh = host.index_fd(r, bs)
    finally:
        th.join(timeout=60)
        os.close(r)
    _check(rows, bh, data, bs)


def test_sf_index_file_on_fifo(gpu, tmp_path, knobs):
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)
    fifo = tmp_path / "fifo"
    os.mkfifo(fifo)
    bs = 4096
    data = oracle.splitmix_bytes((3 << 20) + 99, 711)
    nb = (data.size + bs - 1) // bs
    th = _writer(fifo, data.tobytes())
    out = np.zeros(nb, host.SIG_DTYPE)
    nout = ctypes.c_uint64()
    bh = (ctypes.c_uint8 * 20)()
    rc = lib().sf_index_file(os.fsencode(fifo), bs, out.ctypes.data_as(ctypes.POINTER(BlockSig)), nb,
                             ctypes.byref(nout), bh)
    th.join(timeout=60)
    assert rc == 0 and nout.value == nb
    _check(out, bytes(bh), data, bs)


def test_sf_index_file_on_fifo_reports_need(gpu, tmp_path):
    fifo = tmp_path / "fifo2"
    os.mkfifo(fifo)
    data = oracle.splitmix_bytes(10 * 4096, 712)
    th = _writer(fifo, data.tobytes())
    out = np.zeros(1, host.SIG_DTYPE)
    nout = ctypes.c_uint64()
    rc = lib().sf_index_file(os.fsencode(fifo), 4096, out.ctypes.data_as(ctypes.POINTER(BlockSig)), 1,
                             ctypes.byref(nout), None)
    th.join(timeout=60)
    assert rc == SF_ENOSPC and nout.value == 10


def test_host_index_file_on_fifo(gpu, tmp_path):
    # host.index_file on a FIFO: read once to EOF (a stat says 0 bytes; a
    # sized call would consume the stream and then ask for room)
    fifo = tmp_path / "fifo3"
    os.mkfifo(fifo)
    data = oracle.splitmix_bytes(7 * 4096 + 3, 714)
    th = _writer(fifo, data.tobytes())
    rows, bh = host.index_file(fifo, 4096)
    th.join(timeout=60)
    _check(rows, bh, data, 4096)


def test_index_fd_regular_file_from_offset(gpu, tmp_path):
    # a regular file's descriptor is read from its current position
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(9 * 4096 + 5, 713)
    data.tofile(p)
    fd = os.open(p, os.O_RDONLY)
    try:
        os.lseek(fd, 4096, os.SEEK_SET)
        rows, bh = host.index_fd(fd, 4096)
    finally:
        os.close(fd)
    _check(rows, bh, data[4096:], 4096)


def test_index_fd_bad_descriptor(gpu):
    from syncfast_amd._lib import SfError
    r, w = os.pipe()
    os.close(r)
    os.close(w)
    with pytest.raises(SfError):
        host.index_fd(r, 4096)
