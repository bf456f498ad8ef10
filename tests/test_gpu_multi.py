"""GPU: one process, N devices (sf_index_file_multi, sf_index_device_multi)
with n_devices = 1 on the one-GPU box -- the multi-device plumbing (host
thread per device, shard rows at their row offsets, the RCCL communicator and
the grouped send/recv of the gather, forced through a self send/recv by the
SF_TEST_MULTI_SELF_GATHER hook) against the oracle.  N > 1 needs a node with
several GPUs and is unmeasured here."""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import _lib, device, host

pytestmark = pytest.mark.gpu

MIB = 1 << 20


@pytest.mark.parametrize("size,bs", [(0, 4096), (1, 4096), (5 * MIB + 123, 4096), (3 * MIB, 65536), (777, 100)])
def test_file_multi_equals_oracle(gpu, tmp_path, knobs, size, bs):
    knobs.set("SF_TEST_STREAM_STAGE_MIB", 1)  # several stages per shard
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(size, 8000 + size)
    data.tofile(p)
    for n in (0, 1):  # 0: every visible device
        rows, bh = host.index_file_multi(p, bs, n)
        offs, sizes, want = oracle.index_fixed(data, bs)
        assert np.array_equal(rows["sha1"], want) and bh == oracle.blocks_hash(want)
        assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    host.release_cache()


def test_file_multi_errors(gpu, tmp_path):
    p = tmp_path / "f"
    oracle.splitmix_bytes(100_000, 8100).tofile(p)
    L = _lib.lib()
    out = np.zeros(4, host.SIG_DTYPE)
    need = ctypes.c_uint64()
    bh = (ctypes.c_uint8 * 20)()
    sig = out.ctypes.data_as(ctypes.POINTER(_lib.BlockSig))
    assert L.sf_index_file_multi(os.fsencode(p), 4096, 1, sig, 4, ctypes.byref(need), bh) == _lib.SF_ENOSPC
    assert need.value == 25
    n = torch.cuda.device_count()
    assert L.sf_index_file_multi(os.fsencode(p), 4096, n + 1, sig, 25, ctypes.byref(need), bh) == _lib.SF_EINVAL
    assert L.sf_index_file_multi(os.fsencode(tmp_path / "missing"), 4096, 1, sig, 4, ctypes.byref(need),
                                 bh) == _lib.SF_EIO
    r, w = os.pipe()
    try:
        assert L.sf_index_file_multi(f"/proc/self/fd/{r}".encode(), 4096, 1, sig, 4, ctypes.byref(need),
                                     bh) == _lib.SF_EINVAL
    finally:
        os.close(r)
        os.close(w)


@pytest.mark.parametrize("self_gather", [0, 1])
@pytest.mark.parametrize("size,bs", [(64 * MIB + 4097, 4096), (32 * MIB, 65536), (1, 4096)])
def test_device_multi_equals_oracle(gpu, knobs, self_gather, size, bs):
    """The device-resident form with one device: straight into the table, or
    (self_gather) through RCCL's communicator and a grouped self send/recv."""
    knobs.set("SF_TEST_MULTI_SELF_GATHER", self_gather)
    data = device.splitmix_tensor(size, 8200, device=gpu)
    s = torch.cuda.Stream(gpu)
    table = torch.full(((size + bs - 1) // bs, 20), 0xEE, dtype=torch.uint8, device=gpu)
    with torch.cuda.stream(s):
        got = device.index_device_multi([data], size, bs, table=table, streams=[s])
    s.synchronize()
    _o, _s, want = oracle.index_fixed(data.cpu().numpy(), bs)
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("self_gather", [0, 1])
def test_device_multi_gather_streams(gpu, knobs, self_gather):
    """sf_index_device_multi_ex: hashing on one stream, the exchange on
    another that waits for it (the library's event); five files in a row with
    the exchange of file i still queued while file i+1 is hashed, each into a
    table of its own, every table the oracle's; the library-allocated scratch
    and table survive the caching allocator (record_stream on the streams the
    library used)."""
    knobs.set("SF_TEST_MULTI_SELF_GATHER", self_gather)
    bs = 4096
    hs, gs = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    sizes = [8 * MIB + 1, 3 * bs, 8 * MIB, 1, 5 * MIB + 4095]
    datas = [device.splitmix_tensor(n, 8300 + i, device=gpu) for i, n in enumerate(sizes)]
    torch.cuda.synchronize(gpu)
    tables = []
    for d, n in zip(datas, sizes):
        tables.append(device.index_device_multi([d], n, bs, streams=[hs], gather_streams=[gs]))
        junk = torch.full((1 << 20,), 0x55, dtype=torch.uint8, device=gpu)  # reuses freed blocks if unsafe
        del junk
    gs.synchronize()
    hs.synchronize()
    for d, n, t in zip(datas, sizes, tables):
        _o, _s, want = oracle.index_fixed(d.cpu().numpy(), bs)
        assert np.array_equal(t.cpu().numpy(), want), n


@pytest.mark.parametrize("self_gather", ["1", "0"])
def test_bench_library_path_one_device(gpu, self_gather):
    """bench.py's single-process multi-GPU path (--multi-path library, the
    default at N > 1) on the one device of the box: every step through
    sf_index_device_multi_ex with hash and gather streams, with the
    SF_TEST_MULTI_SELF_GATHER hook sending the table through RCCL (a self
    send/recv) -- the same code the driver's N-GPU run takes, at N = 1 -- plus
    the e2e_file_multi leg (sf_index_file_multi).  The bench checks the
    gathered table itself (every shard's first and last digest against the
    product's host SHA-1); here the line's shape."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SF_TEST_MULTI_SELF_GATHER"] = self_gather
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--multi-path", "library",
                        "--shard-gib", "0.25", "--steps", "6", "--warmup", "2", "--ramp-s", "0.05",
                        "--e2e-multi-gib", "0.125"], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["config"]["total_bytes"] == 1 << 28
    m = line["multi"]
    assert m["path"] == "library" and m["world"] == 1 and m["self_gather"] == (self_gather == "1")
    assert m["steps_as_root"] == [6]
    assert line["roofline"]["kernel"] == "sha1_fixed_kernel<128>" and line["roofline"]["kernel_ms"] > 0
    e2e = line["e2e_file_multi"]
    assert e2e["devices"] == 1 and e2e["bytes"] == 1 << 27 and e2e["GB/s"] > 0
