"""The C-ABI from plain C (examples/sf_index.c): no Python, no PyTorch in the
process -- what a Rust extern "C" binding amounts to.

CPU: the binary builds, links only libsyncfast_amd (+ the HIP runtime) and
fails loudly without a device.  GPU: a regular file, a FIFO and stdin give
the oracle's rows and blocks_hash (src/index.rs:621-682)."""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "build", "sf_index")


def _built(make: bool):
    """The example binary; built here on the CPU side (make is a no-op when it
    is up to date), only looked up on a GPU box (built by build())."""
    if make:
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "examples")])
    assert os.path.exists(BIN), f"{BIN} not built: run __graft_entry__.build()"
    return BIN


def _parse(out):
    files, cur = {}, None
    for ln in out.splitlines():
        f = ln.split()
        if f[0] == "file":
            cur = files.setdefault(f[1], {"rows": []})
        elif f[0] == "blocks_hash":
            cur["bh"] = f[1]
        else:
            cur["rows"].append((int(f[0]), int(f[1]), f[2]))
    return files


def _want(data, bs):
    offs, sizes, dig = oracle.index_fixed(data, bs)
    return [(int(o), int(s), bytes(d).hex()) for o, s, d in zip(offs, sizes, dig)], oracle.blocks_hash(dig).hex()


def test_c_consumer_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    r = subprocess.run([_built(True), "/dev/null"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_c_consumer_file_fifo_stdin(gpu, tmp_path):
    exe = _built(False)
    bs = 4096
    a = oracle.splitmix_bytes((3 << 20) + 77, 31)
    b = oracle.splitmix_bytes(10_000, 32)
    pa, fifo = tmp_path / "a.bin", tmp_path / "pipe"
    a.tofile(pa)
    os.mkfifo(fifo)

    def feed():
        with open(fifo, "wb") as w:
            w.write(b.tobytes())
    th = threading.Thread(target=feed)
    th.start()
    r = subprocess.run([exe, "-b", str(bs), str(pa), str(fifo), "-"], input=a[:5000].tobytes(),
                       capture_output=True, timeout=120)
    th.join(timeout=30)
    assert r.returncode == 0, r.stderr.decode()
    got = _parse(r.stdout.decode())
    for name, data in ((str(pa), a), (str(fifo), b), ("-", a[:5000])):
        rows, bh = _want(data, bs)
        assert got[name]["rows"] == rows and got[name]["bh"] == bh, name
    r = subprocess.run([exe, str(tmp_path / "missing")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "I/O error" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,bs", [(3 * 4096 + 5, 4096), (1 << 20, 65536), (0, 4096), (2_000_003, 1000)])
def test_c_consumer_device_path_and_wire(gpu, n, bs):
    # -w: bytes generated in HBM, hashed there and the FILE_BLOCK run streamed
    # to stdout, all from C -- equal to write_message over the oracle's digests
    from syncfast_amd import wire
    from syncfast_amd.digest import HashDigest
    r = subprocess.run([_built(False), "-w", str(n), "-b", str(bs)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    offs, sizes, dig = oracle.index_fixed(oracle.splitmix_bytes(n, 0x5EED0000), bs)
    want = b"".join(wire.write_message("FileBlock", HashDigest(bytes(d)), int(s)) for d, s in zip(dig, sizes))
    assert r.stdout == want


@pytest.mark.gpu
def test_c_consumer_block_lookup(gpu, tmp_path):
    # -L dst src: src's blocks looked up among dst's rows through
    # sf_block_set_* from C; the answers equal the oracle's first-row lookup
    bs = 4096
    rng = np.random.default_rng(5)
    a = oracle.splitmix_bytes(300 * bs, 41).reshape(300, bs)
    a[250:260] = a[10:20]  # repeated blocks inside dst: the first row wins
    fresh = oracle.splitmix_bytes(50 * bs, 42).reshape(50, bs)
    b = np.concatenate([a[rng.integers(0, 300, 150)], fresh])
    rng.shuffle(b)
    pa, pb = tmp_path / "dst", tmp_path / "src"
    a.tofile(pa)
    b.tofile(pb)
    r = subprocess.run([_built(False), "-L", "-b", str(bs), str(pa), str(pb)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got = [int(ln.split()[1]) for ln in r.stdout.decode().splitlines()]
    want = oracle.block_lookup(oracle.index_fixed(a.reshape(-1), bs)[2], None, oracle.index_fixed(b.reshape(-1), bs)[2])
    assert got == want.tolist() and sum(g >= 0 for g in got) == 150


def _cdc_cuts(data: np.ndarray):
    """The C consumer's stand-in chunker (-C), restated: a block ends after
    byte i when the little-endian word of bytes i-3..i times 2654435761
    (mod 2^32) is below 2^19, or at 32 KiB, or at the end of the data."""
    n = data.size
    trig = np.zeros(n, bool)
    if n >= 4:
        w = (data[:-3].astype(np.uint64) | data[1:-2].astype(np.uint64) << 8 |
             data[2:-1].astype(np.uint64) << 16 | data[3:].astype(np.uint64) << 24)
        trig[3:] = ((w * 2654435761) & 0xFFFFFFFF) < (1 << 19)
    offs, sizes, start = [], [], 0
    hits = np.flatnonzero(trig).tolist() + [n - 1]
    k = 0
    while start < n:
        while hits[k] < start:
            k += 1
        end = min(hits[k], start + 32767, n - 1) + 1
        offs.append(start)
        sizes.append(end - start)
        start = end
    return offs, sizes


@pytest.mark.gpu
def test_c_consumer_content_defined_blocks(gpu, tmp_path):
    # -C: a host chunker cuts each file, sf_index_buffer_blocks hashes its
    # blocks -- the reference's default mode as a C/Rust caller drops it in
    exe = _built(False)
    files = {}
    for i, n in enumerate([0, 1, 3, 4, 5000, 100_000, (3 << 20) + 11]):
        data = oracle.splitmix_bytes(n, 900 + i)
        p = tmp_path / f"c{i}"
        data.tofile(p)
        files[str(p)] = data
    ones = np.full(100_000, 0xFF, np.uint8)  # no trigger at all: 32 KiB blocks
    zeros = np.zeros(50_000, np.uint8)  # a trigger at every byte from the 4th: 1-byte blocks, the list grows
    for nm, data in (("ones", ones), ("zeros", zeros)):
        data.tofile(tmp_path / nm)
        files[str(tmp_path / nm)] = data
    r = subprocess.run([exe, "-C"] + list(files), capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got = _parse(r.stdout.decode())
    for name, data in files.items():
        offs, sizes = _cdc_cuts(data)
        dig = oracle.index_blocks(data, np.asarray(offs, np.uint64), np.asarray(sizes, np.uint32))
        rows = [(o, s, bytes(d).hex()) for o, s, d in zip(offs, sizes, dig)]
        assert got[name]["rows"] == rows and got[name]["bh"] == oracle.blocks_hash(dig).hex(), name
    assert [r[1] for r in got[str(tmp_path / "ones")]["rows"]] == [32768, 32768, 32768, 100_000 - 3 * 32768]
    assert len(got[str(tmp_path / "zeros")]["rows"]) == 50_000 - 3


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 5, 100_000, (3 << 20) + 17])
def test_c_consumer_content_defined_wire_run(gpu, n):
    # -v: bytes generated in HBM, cut by the host chunker, hashed as a list
    # on the device and the list's FILE_BLOCK run streamed to stdout, from C
    # -- equal to write_message over the oracle's digests and sizes
    from syncfast_amd import wire
    r = subprocess.run([_built(False), "-v", str(n)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    data = oracle.splitmix_bytes(n, 0x5EED0000)
    offs, sizes = _cdc_cuts(data)
    dig = oracle.index_blocks(data, np.asarray(offs, np.uint64), np.asarray(sizes, np.uint32))
    want = b"".join(wire.write_message("FileBlock", bytes(d), int(s)) for d, s in zip(dig, sizes))
    assert r.stdout == want


@pytest.mark.gpu
@pytest.mark.parametrize("threads,large_mib", [(1, 64), (4, 64), (4, 2)])
def test_c_consumer_default_mode_many_files(gpu, tmp_path, threads, large_mib):
    """examples/sf_index -Z -M: the default mode over many files from C --
    files cut by the stand-in chunker on `threads` threads over their open
    descriptors, batches hashed by sf_index_fds_blocks, two passes in one
    process; with -K 2 the files of 2 MiB and more are indexed alone, in
    their place, through sf_index_fd_cut on the threads.  Every row = the
    stand-in chunker's boundaries (the oracle's copy of it) with the oracle's
    digests; every blocks_hash = the oracle's; files in command-line order."""
    exe = _built(False)
    rng = np.random.default_rng(threads)
    paths, datas = [], []
    for k, n in enumerate([0, 1, 100_000, 32768, 3 << 20, 777, (9 << 20) + 3] +
                          [int(x) for x in rng.integers(0, 300_000, 40)] + [2 << 20]):
        p = tmp_path / f"f{k:03d}"
        d = oracle.splitmix_bytes(n, 900 + k)
        d.tofile(p)
        paths.append(str(p))
        datas.append(d)
    r = subprocess.run([exe, "-Z", "-M", "-P", "2", "-S", "1", "-K", str(large_mib), "-j", str(threads)] + paths,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = _parse(r.stdout)
    assert list(got) == paths
    for p, d in zip(paths, datas):
        sizes = oracle.zpaq_standin_sizes(d) if d.size else np.zeros(0, np.uint32)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) if sizes.size else sizes
        dig = oracle.index_blocks(d, offs, sizes) if sizes.size else np.zeros((0, 20), np.uint8)
        assert got[p]["rows"] == [(int(o), int(s), bytes(h).hex()) for o, s, h in zip(offs, sizes, dig)], p
        assert got[p]["bh"] == oracle.blocks_hash(dig).hex(), p


@pytest.mark.gpu
@pytest.mark.parametrize("n,bs", [((5 << 20) + 123, 4096), (1, 4096), (0, 4096), (777_777, 1000)])
def test_c_consumer_one_file_on_every_device(gpu, tmp_path, n, bs):
    # -X 0: sf_index_file_multi on every visible device (one here): the
    # oracle's rows and blocks_hash, from plain C
    exe = _built(False)
    data = oracle.splitmix_bytes(n, 41)
    p = tmp_path / "m.bin"
    data.tofile(p)
    r = subprocess.run([exe, "-X", "0", "-b", str(bs), str(p)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = _parse(r.stdout)[str(p)]
    rows, bh = _want(data, bs)
    assert got["rows"] == rows and got["bh"] == bh


@pytest.mark.gpu
@pytest.mark.parametrize("threads,two_calls", [(2, False), (16, False), (16, True)])
def test_c_consumer_parallel_cut(gpu, tmp_path, threads, two_calls):
    # -Z -p N: the stand-in chunker over each file on N threads, the file read
    # once and hashed from HBM (sf_index_fd_cut); -W: sf_cut_fd, then
    # sf_index_fd_blocks from the descriptor.  Every row equals the
    # one-stream cut's (the oracle's stand-in over the whole file) with the
    # oracle's digests
    exe = _built(False)
    files = {}
    for i, n in enumerate([0, 1, 70_000, (9 << 20) + 5, (33 << 20) + 77]):
        data = oracle.splitmix_bytes(n, 950 + i)
        p = tmp_path / f"p{i}"
        data.tofile(p)
        files[str(p)] = data
    z = np.zeros(12 << 20, np.uint8)  # the size cap and a degenerate hash across segment edges
    z.tofile(tmp_path / "zeros")
    files[str(tmp_path / "zeros")] = z
    r = subprocess.run([exe, "-Z", "-p", str(threads)] + (["-W"] if two_calls else []) + list(files),
                       capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    got = _parse(r.stdout.decode())
    for name, data in files.items():
        sizes = oracle.zpaq_standin_sizes(data).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) if sizes.size else sizes
        dig = oracle.index_blocks(data, offs, sizes.astype(np.uint32)) if sizes.size else np.zeros((0, 20), np.uint8)
        rows = [(int(o), int(s), bytes(d).hex()) for o, s, d in zip(offs, sizes, dig)]
        assert got[name]["rows"] == rows and got[name]["bh"] == oracle.blocks_hash(dig).hex(), name
