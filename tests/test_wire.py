"""Wire emission of signature tables (src/sync/ssh/proto.rs)."""
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
def test_file_blocks_to_fd_streams_the_same_bytes(gpu, tmp_path, monkeypatch, n, bs, chunk):
    # the streamed writer (chunks of SF_WIRE_CHUNK messages, double-buffered
    # D2H, in-order writes) produces exactly the device-built run
    if chunk != "0":
        monkeypatch.setenv("SF_WIRE_CHUNK", chunk)
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
