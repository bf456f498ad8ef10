"""sf_cut_fd: the caller's content-defined chunker over one file on several
threads, joined so that the boundaries are exactly the sequential ones
(src/index.rs:622-647: one cdchunking stream per file).  Host only, so these
run on the CPU.

The chunker here is the stand-in of examples/zpaq_standin.h (the crate's
per-byte work, not its boundaries; the crate is not in this image), through
examples/build/libzpaq_standin.so, checked against the oracle's sequential
run of the same stand-in over the whole file in memory; and a Python chunker
(ctypes callbacks from the library's threads) with other parameters, checked
against a plain Python loop."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
from syncfast_amd import SfError, host
from syncfast_amd._lib import SF_EAGAIN, SF_EINVAL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "examples", "build", "libzpaq_standin.so")


class ChunkerOps(ctypes.Structure):
    _fields_ = [("create", ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)),
                ("next", ctypes.CFUNCTYPE(ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8),
                                          ctypes.c_size_t)),
                ("destroy", ctypes.CFUNCTYPE(None, ctypes.c_void_p)),
                ("ctx", ctypes.c_void_p)]


@pytest.fixture(scope="module")
def standin():
    if not os.path.exists(SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "examples"), "build/libzpaq_standin.so"])
    lib = ctypes.CDLL(SO)
    lib.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    lib.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    lib.sf_zpaq_standin_ops_free.argtypes = [ctypes.c_void_p]
    ops = lib.sf_zpaq_standin_ops(13, 32768)  # ZPAQ_BITS, MAX_BLOCK_SIZE (src/index.rs:40-41)
    yield lib, ops
    lib.sf_zpaq_standin_ops_free(ops)


def _cut(path, ops, threads, stamp=None):
    with open(path, "rb") as f:
        return host.cut_fd(f.fileno(), ops, threads, stamp)


def _check(path, data, ops, threads_list):
    want = oracle.zpaq_standin_sizes(data).astype(np.uint32)
    woffs = np.zeros(want.size, np.uint64)
    if want.size > 1:
        woffs[1:] = np.cumsum(want.astype(np.uint64))[:-1]
    for t in threads_list:
        offs, sizes = _cut(path, ops, t)
        assert np.array_equal(sizes, want) and np.array_equal(offs, woffs), t


@pytest.mark.parametrize("n", [0, 1, 100, 32768, 32769, (5 << 20) + 7, (41 << 20) + 12345])
def test_random_bytes_equal_the_sequential_cut(tmp_path, standin, n):
    _lib, ops = standin
    data = oracle.splitmix_bytes(n, 60 + n % 1000)
    p = tmp_path / "r.bin"
    data.tofile(p)
    _check(p, data, ops, [1, 2, 7, 16, 0])


def test_structured_bytes_equal_the_sequential_cut(tmp_path, standin):
    """Inputs on which speculative chains meet the true one late or only by
    the size cap: zeros, a short period, text (the reference KAT repeated),
    and all of them spliced together across the segment edges."""
    _lib, ops = standin
    kat = np.frombuffer(oracle.kat_input(), np.uint8)
    parts = [np.zeros(9 << 20, np.uint8), np.tile(np.arange(7, dtype=np.uint8), (6 << 20) // 7),
             np.tile(kat, (10 << 20) // kat.size), oracle.splitmix_bytes(5 << 20, 61)]
    for k, data in enumerate(parts + [np.concatenate(parts)]):
        p = tmp_path / f"s{k}.bin"
        data.tofile(p)
        _check(p, data, ops, [1, 3, 16])


def _py_standin(bits, max_size):
    """The stand-in's recurrence as a Python chunker (sf_chunker_ops through
    ctypes callbacks), and its sequential cut for checking."""
    limit = 1 << (32 - bits)
    states = {}

    def fresh():
        return {"h": 0, "c1": 0, "run": 0, "o1": bytearray(256)}

    def create(_ctx):
        key = len(states) + 1
        while key in states:
            key += 1
        states[key] = fresh()
        return key

    def nxt(ch, p, n):
        s = states[ch]
        h, c1, o1 = s["h"], s["c1"], s["o1"]
        m = min(n, max_size - s["run"])
        buf = ctypes.string_at(p, m)
        for i, c in enumerate(buf):
            h = ((h + c + 1) * (314159265 if c == o1[c1] else 271828182)) & 0xFFFFFFFF
            o1[c1] = c
            c1 = c
            if h < limit:
                states[ch] = fresh()
                return i + 1
        if m == max_size - s["run"]:
            states[ch] = fresh()
            return m
        s["h"], s["c1"], s["run"] = h, c1, s["run"] + m
        return 0

    def destroy(ch):
        states.pop(ch, None)

    def sequential(data):
        sizes, start, st = [], 0, fresh()
        h, c1, o1 = 0, 0, st["o1"]
        for i, c in enumerate(bytes(data)):
            h = ((h + c + 1) * (314159265 if c == o1[c1] else 271828182)) & 0xFFFFFFFF
            o1[c1] = c
            c1 = c
            if h < limit or i + 1 - start == max_size:
                sizes.append(i + 1 - start)
                start, h, c1, o1 = i + 1, 0, 0, bytearray(256)
        if start < len(data):
            sizes.append(len(data) - start)
        return sizes

    ops = ChunkerOps(ChunkerOps._fields_[0][1](create), ChunkerOps._fields_[1][1](nxt),
                     ChunkerOps._fields_[2][1](destroy), None)
    return ops, sequential


def test_python_chunker_other_parameters(tmp_path):
    """A chunker of the caller's in Python (callbacks from the library's
    threads), 8-bit boundaries and a 3000-byte cap: the joined cut equals a
    plain sequential loop, on several threads."""
    ops, sequential = _py_standin(8, 3000)
    data = oracle.splitmix_bytes((9 << 20) + 17, 62)
    p = tmp_path / "py.bin"
    data.tofile(p)
    want = np.asarray(sequential(data), np.uint32)
    for t in (1, 2):
        offs, sizes = _cut(p, ctypes.addressof(ops), t)
        assert np.array_equal(sizes, want), t


def test_errors(tmp_path, standin):
    _lib, ops = standin
    p = tmp_path / "e.bin"
    oracle.splitmix_bytes(100_000, 63).tofile(p)
    with open(p, "rb") as f:
        st = host.file_stamp(f.fileno())
    with open(p, "r+b") as g:  # a stale stamp: the file was written after it
        g.write(b"x")
    os.utime(p, ns=(st.mtime_sec * 10**9 + st.mtime_nsec, st.mtime_sec * 10**9 + st.mtime_nsec + 1))
    with pytest.raises(SfError) as e:
        _cut(p, ops, 4, st)
    assert e.value.code == SF_EAGAIN
    r, w = os.pipe()
    try:
        with pytest.raises(SfError) as e:
            host.cut_fd(r, ops, 4)
        assert e.value.code == SF_EINVAL
    finally:
        os.close(r)
        os.close(w)
    bad = ChunkerOps()  # no functions
    with pytest.raises(SfError) as e:
        _cut(p, ctypes.addressof(bad), 1)
    assert e.value.code == SF_EINVAL
