"""GPU parity at BASELINE sizes.

configs[1]: 8 GiB in 4 KiB blocks -- every one of the 2^21 digests compared
with the multi-threaded C oracle on the host (bit-exact, plus blocks_hash).
configs[4]: 32 GiB in 64 KiB blocks -- size-independent properties: a
random sample of blocks vs the oracle, the last block, idempotence of a second
launch, and the chunked-vs-whole checksum of checksums."""
import os

import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import device, host

pytestmark = pytest.mark.gpu
GiB = 1 << 30


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def test_config2_8gib_4k_every_digest(gpu):
    n, bs = 8 * GiB, 4096
    data = device.splitmix_tensor(n, 0x5EED0000, gpu)
    dig = device.index_device(data, bs).cpu().numpy()
    host_bytes = data.cpu().numpy()
    del data
    torch.cuda.empty_cache()
    want = oracle.index_fixed_mt(host_bytes, bs, _threads())
    assert dig.shape == (n // bs, 20)
    bad = np.nonzero((dig != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} digests differ, first at block {bad[:5]}"
    assert host.blocks_hash(dig) == oracle.blocks_hash(want)
    # explicit blocks scattered over the whole 8 GiB: most waves span more
    # than 4 GiB and take the per-lane path; some are 16-B aligned
    rng = np.random.default_rng(8)
    m = 3000
    sizes = rng.integers(0, 70_000, m)
    offs = np.array([int(rng.integers(0, n - s)) for s in sizes], np.int64)
    offs[::3] = offs[::3] // 16 * 16
    data_t = torch.from_numpy(host_bytes).to(gpu)
    dt = device.index_device_blocks(data_t, torch.from_numpy(offs).to(gpu),
                                    torch.from_numpy(sizes.astype(np.int32)).to(gpu)).cpu().numpy()
    assert np.array_equal(dt, oracle.index_blocks(host_bytes, offs, sizes))


def test_config5_32gib_64k_properties(gpu):
    n, bs = 32 * GiB, 65536
    data = device.splitmix_tensor(n, 0x5EED0004, gpu)
    d1 = device.index_device(data, bs)
    d2 = device.index_device(data, bs)
    assert torch.equal(d1, d2)  # idempotent
    dig = d1.cpu().numpy()
    rng = np.random.default_rng(4)
    sample = np.unique(np.concatenate([rng.integers(0, n // bs, 600), [0, 63, 64, n // bs - 1]]))
    for i in sample:
        blk = data[i * bs:(i + 1) * bs].cpu().numpy()
        assert bytes(dig[i]) == oracle.sha1(blk), i
    # checksum of checksums: indexing the halves separately gives the same table
    half = n // 2
    h1 = device.index_device(data[:half], bs)
    h2 = device.index_device(data[half:], bs)
    assert host.blocks_hash(torch.cat([h1, h2]).cpu().numpy()) == host.blocks_hash(dig)


@pytest.mark.parametrize("mode", ["stream", "staged"])
def test_config3_1024x8mib_every_digest_and_blocks_hash(gpu, mode):
    # configs[2] at full size: 1024 files x 8 MiB, every digest and every
    # file's blocks_hash vs the multi-threaded C oracle
    nf, flen, bs = 1024, 8 << 20, 4096
    data = device.splitmix_tensor(nf * flen, 0x5EED0002, gpu)
    if mode == "stream":
        st = device.BatchStream(nf, flen, bs)
        dig = torch.empty((nf * flen // bs, 20), dtype=torch.uint8, device=gpu)
        assert st.push(data, dig) is None
        (fh,) = st.finish()
    else:
        dig, _, fh = device.index_device_batch(data, [(i * flen, flen) for i in range(nf)], bs)
    dig, fh = dig.cpu().numpy(), fh.cpu().numpy()
    host_bytes = data.cpu().numpy()
    del data
    torch.cuda.empty_cache()
    want = oracle.index_fixed_mt(host_bytes, bs, _threads())
    bad = np.nonzero((dig != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} digests differ, first at block {bad[:5]}"
    per_file = want.reshape(nf, -1, 20)
    wrong = [f for f in range(nf) if bytes(fh[f]) != host.blocks_hash(per_file[f])]
    assert not wrong, f"{len(wrong)} blocks_hash differ, first files {wrong[:5]}"
