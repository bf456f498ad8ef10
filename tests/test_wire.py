"""Wire emission of signature tables (src/sync/ssh/proto.rs)."""
import ctypes
import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, wire
from syncfast_amd.digest import HashDigest


def test_reference_test_write_bytes():
    # proto::tests::test_write, src/sync/ssh/proto.rs:512-528
    out = wire.write_message("FileEntry", b"filename", 12, HashDigest(b"12345678901234567890"))
    out += wire.write_message("EndFiles")
    assert out == b"FILE_ENTRY\nfilename\n12\n12345678901234567890\nEND_FILES\n"


def test_other_messages():
    d = HashDigest(bytes(range(20)))
    assert wire.write_message("FileBlock", d, 4096) == b"FILE_BLOCK\n" + bytes(range(20)) + b"\n4096\n"
    assert wire.write_message("BlockData", d, b"xyz") == b"BLOCK_DATA\n" + bytes(range(20)) + b"\n3\nxyz\n"
    assert wire.write_message("FileStart", b"a/b") == b"FILE_START\na/b\n"
    assert wire.write_message("FileEnd") + wire.write_message("Complete") == b"FILE_END\nCOMPLETE\n"



def test_reference_test_parse():
    # proto::tests::test_parse, src/sync/ssh/proto.rs:483-510: the same byte
    # pieces, the same messages after each piece
    inputs = [b"FILE_ENTR", b"Y", b"\n", b"filename\n12", b"\n12345678901234567890\nCOMPLETE", b"\n"]
    expected = [[], [], [], [], [("FileEntry", b"filename", 12, HashDigest(b"12345678901234567890"))], [("Complete",)]]
    p = wire.Parser()
    for piece, want in zip(inputs, expected):
        assert p.receive(piece) == want


def test_parse_round_trips_every_message_bytewise():
    d = HashDigest(bytes(range(20)))
    msgs = [("FileEntry", b"dir/f", 123456789, d), ("EndFiles",), ("GetFile", b"dir/f"), ("FileStart", b"x"),
            ("FileBlock", d, 4096), ("FileBlock", HashDigest(b"\n" * 20), 7), ("FileEnd",), ("GetBlock", d),
            ("BlockData", d, b"a\nb\n"), ("BlockData", d, b""), ("Complete",)]
    stream = b"".join(wire.write_message(*m) for m in msgs)
    p = wire.Parser()
    got = []
    for i in range(len(stream)):  # one byte at a time: every split point
        got += p.receive(stream[i:i + 1])
    assert got == msgs
    assert wire.Parser().receive(stream) == msgs


@pytest.mark.parametrize("data,err", [
    (b"X" * 20, "Unterminated command"),
    (b"NOPE\n", "Unknown command"),
    (b"GET_FILE\n" + b"f" * 100, "Unterminated filename"),
    (b"FILE_BLOCK\n" + b"d" * 20 + b"x", "Unterminated digest"),
    (b"FILE_BLOCK\n" + b"d" * 20 + b"\n-1\n", "Invalid block size"),
    (b"FILE_BLOCK\n" + b"d" * 20 + b"\n1 \n", "Invalid block size"),
    (b"FILE_BLOCK\n" + b"d" * 20 + b"\n" + b"1" * 15, "Unterminated size"),
    (b"FILE_ENTRY\nf\n1a\n", "Invalid file size"),
    (b"FILE_ENTRY\nf\n" + b"1" * 16 + b"\n", "Unterminated size"),
    (b"BLOCK_DATA\n" + b"d" * 20 + b"\n2\nabc", "Invalid data end byte"),
])
def test_parse_errors(data, err):
    with pytest.raises(wire.ProtocolError, match=err):
        wire.Parser().receive(data)


def test_parse_limits_and_usize_forms():
    # a line of exactly its limit is accepted; Rust's usize::from_str takes a leading '+'
    p = wire.Parser()
    assert p.receive(b"GET_FILE\n" + b"f" * 100 + b"\n") == [("GetFile", b"f" * 100)]
    d = b"d" * 20
    assert p.receive(b"FILE_BLOCK\n" + d + b"\n+12\n") == [("FileBlock", HashDigest(d), 12)]
    assert p.receive(b"FILE_BLOCK\n" + d + b"\n" + b"9" * 15 + b"\n") == [("FileBlock", HashDigest(d), 10 ** 15 - 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,bs", [(4096 * 10 + 7, 4096), (65536 * 3, 65536), (999, 100), (5, 4096)])
def test_file_blocks_device_matches_write_message(gpu, n, bs):
    data = oracle.splitmix_bytes(n, n)
    t = torch.from_numpy(data.copy()).to(gpu)
    dig = device.index_device(t, bs)
    got = wire.file_blocks_device(dig, bs, n).cpu().numpy().tobytes()
    _, sizes, want_d = oracle.index_fixed(data, bs)
    want = b"".join(wire.write_message("FileBlock", bytes(dd), int(sz)) for dd, sz in zip(want_d, sizes))
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", ["1", "7", "1000", "0"])
@pytest.mark.parametrize("n,bs", [(4096 * 2500 + 7, 4096), (999, 100), (4096, 4096)])
def test_file_blocks_to_fd_streams_the_same_bytes(gpu, tmp_path, n, bs, chunk, knobs):
    # the streamed writer (chunks of SF_TEST_WIRE_CHUNK messages, double-buffered
    # D2H, in-order writes) produces exactly the device-built run
    if chunk != "0":
        knobs.set("SF_TEST_WIRE_CHUNK", int(chunk))
    data = oracle.splitmix_bytes(n, n + 1)
    t = torch.from_numpy(data.copy()).to(gpu)
    dig = device.index_device(t, bs)
    want = wire.file_blocks_device(dig, bs, n).cpu().numpy().tobytes()
    p = tmp_path / "wire.bin"
    with open(p, "wb") as f:
        got_n = wire.file_blocks_to_fd(dig, bs, n, f.fileno())
    assert got_n == len(want) and p.read_bytes() == want
    if n < 10_000:
        _, sizes, want_d = oracle.index_fixed(data, bs)
        assert want == b"".join(wire.write_message("FileBlock", bytes(dd), int(sz)) for dd, sz in zip(want_d, sizes))



@pytest.mark.gpu
@pytest.mark.parametrize("n,bs", [(4096 * 2500 + 7, 4096), (999, 100), (65536 * 8, 65536)])
def test_device_run_parses_back_to_the_rows(gpu, n, bs):
    # a destination's parser over the device-built FILE_BLOCK run gets the
    # file's rows back: every digest and every block size, in order
    data = oracle.splitmix_bytes(n, n + 2)
    dig = device.index_device(torch.from_numpy(data.copy()).to(gpu), bs)
    run = wire.file_blocks_device(dig, bs, n).cpu().numpy().tobytes()
    msgs = wire.Parser().receive(run)
    _, sizes, want = oracle.index_fixed(data, bs)
    assert [m[0] for m in msgs] == ["FileBlock"] * len(want)
    assert [m[1].bytes for m in msgs] == [bytes(w) for w in want]
    assert [m[2] for m in msgs] == [int(x) for x in sizes]


def test_blocks_device_validation_without_device():
    from syncfast_amd import _lib
    L = _lib.lib()
    n = ctypes.c_uint64(7)
    assert L.sf_wire_blocks_device(None, None, 0, None, 0, ctypes.byref(n), None) == 0 and n.value == 0
    assert L.sf_wire_blocks_device(None, None, 3, None, 0, ctypes.byref(n), None) == _lib.SF_EINVAL
    assert L.sf_wire_blocks_fd(None, None, 0, 1, ctypes.byref(n), None) == 0 and n.value == 0
    assert L.sf_wire_blocks_fd(None, None, 3, 1, ctypes.byref(n), None) == _lib.SF_EINVAL


@pytest.mark.gpu
def test_blocks_device_reference_kat_blocks(gpu):
    """The KAT file's three content-defined blocks (src/index.rs:765-792) as
    the FILE_BLOCK run a source would send: sizes 11579, 32768, 546."""
    digs = ["fb5ef7ebadd82c8085c5ff63823622bae0e263f6", "570d8b30fcfd585e4127b561f5ecd376ff4d0101",
            "b9a8c2641af2cf8fd8f36a2456a3eaa95c029127"]
    sizes = [11579, 32768, 546]
    d = torch.tensor(np.frombuffer(bytes.fromhex("".join(digs)), np.uint8).reshape(3, 20).copy(), device=gpu)
    got = wire.blocks_device(d, torch.tensor(sizes, dtype=torch.int32, device=gpu)).cpu().numpy().tobytes()
    want = b"".join(wire.write_message("FileBlock", bytes.fromhex(h), s) for h, s in zip(digs, sizes))
    assert got == want
    assert [m[2] for m in wire.Parser().receive(got)] == sizes


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 100_003])
def test_blocks_device_matches_write_message(gpu, n):
    rng = np.random.default_rng(n)
    dig = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    # every digit count from 1 to 10 (u32 up to 4294967295), zero included
    sizes = (rng.integers(0, 10, n) * 0 + 10 ** rng.integers(0, 10, n) * rng.integers(1, 10, n)).astype(np.uint64)
    sizes = np.minimum(sizes, 4294967295).astype(np.uint32)
    sizes[rng.random(n) < 0.05] = 0
    if n > 1:
        sizes[-1] = 4294967295
    got = wire.blocks_device(torch.from_numpy(dig).to(gpu),
                             torch.from_numpy(sizes.view(np.int32)).to(gpu)).cpu().numpy().tobytes()
    want = b"".join(wire.write_message("FileBlock", bytes(d), int(s)) for d, s in zip(dig, sizes))
    assert got == want


@pytest.mark.gpu
def test_blocks_device_equals_fixed_form_and_parses_back(gpu):
    n, bs = 4096 * 3000 + 77, 4096
    data = oracle.splitmix_bytes(n, 5)
    t = torch.from_numpy(data.copy()).to(gpu)
    dig = device.index_device(t, bs)
    nb = dig.shape[0]
    sizes = torch.full((nb,), bs, dtype=torch.int32, device=gpu)
    sizes[-1] = n - (nb - 1) * bs
    run = wire.blocks_device(dig, sizes)
    assert torch.equal(run, wire.file_blocks_device(dig, bs, n))
    # a content-defined-like list: rows back through the parser
    rng = np.random.default_rng(6)
    cut = np.minimum(rng.geometric(1 / 8192, 4000), 32768).astype(np.uint64)
    ends = np.cumsum(cut)
    ends = ends[ends < n]
    b = np.concatenate([[0], ends, [n]]).astype(np.uint64)
    offs, szs = b[:-1], np.diff(b).astype(np.uint32)
    d2 = device.index_device_blocks(t, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                                    torch.from_numpy(szs.astype(np.int32)).to(gpu))
    run2 = wire.blocks_device(d2, torch.from_numpy(szs.view(np.int32)).to(gpu)).cpu().numpy().tobytes()
    msgs = wire.Parser().receive(run2)
    assert [m[2] for m in msgs] == szs.tolist()
    assert [m[1].bytes for m in msgs] == [bytes(x) for x in oracle.index_blocks(data, offs, szs)]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", ["1", "7", "1000", "0"])
def test_blocks_to_fd_streams_the_device_run(gpu, tmp_path, chunk, knobs):
    if chunk != "0":
        knobs.set("SF_TEST_WIRE_CHUNK", int(chunk))
    rng = np.random.default_rng(int(chunk) + 3)
    n = 20_000 if chunk != "1" else 700
    dig = torch.from_numpy(rng.integers(0, 256, (n, 20), dtype=np.uint8)).to(gpu)
    sizes = torch.from_numpy(np.minimum(rng.geometric(1 / 8192, n), 32768).astype(np.int32)).to(gpu)
    want = wire.blocks_device(dig, sizes).cpu().numpy().tobytes()
    p = tmp_path / "run.bin"
    with open(p, "wb") as f:
        got = wire.blocks_to_fd(dig, sizes, f.fileno())
    assert got == len(want) and p.read_bytes() == want
