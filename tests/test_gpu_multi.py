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
