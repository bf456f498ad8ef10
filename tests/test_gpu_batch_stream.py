"""GPU: equal-size many-file batches as a stream (sf_index_device_batch_chained
through device.BatchStream): each launch hashes one batch's blocks and the
previous batch's per-file blocks_hash (src/index.rs:661-682).  Every digest
and every blocks_hash is compared with the oracle."""
import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import SfError, device
from syncfast_amd._lib import SF_EINVAL

pytestmark = pytest.mark.gpu


def _batch(nf, flen, seed, dev):
    host = np.concatenate([oracle.splitmix_bytes(flen, seed + i) for i in range(nf)])
    return host, torch.from_numpy(host).to(dev)


@pytest.mark.parametrize("last", ["finish", "push_last"])
@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("nf,flen,bs", [(64, 4096 * 16, 4096), (300, 4096 * 8, 4096), (5, 65536 * 4, 65536),
                                         (70, 1000 * 4, 1000), (40, 4096 * 128, 4096), (9, 1024 * 192, 1024)])
def test_stream_every_digest_and_hash(gpu, nf, flen, bs, split, last):
    # the last two shapes (128 and 192 blocks per file) take push_last's
    # column halves; the others fall back to push + finish
    st = device.BatchStream(nf, flen, bs, split=split)
    hosts, digs, hashes = [], [], []
    for k in range(4):
        host, t = _batch(nf, flen, 0x5EED0000 + 1000 * k, gpu)
        d = torch.empty((nf * flen // bs, 20), dtype=torch.uint8, device=gpu)
        if last == "push_last" and k == 3:
            hashes += st.push_last(t, d)
        else:
            h = st.push(t, d)
            if h is not None:
                hashes.append(h)
        hosts.append(host)
        digs.append(d)
    hashes += st.finish()
    assert st.finish() == [] and len(hashes) == 4
    for host, d, h in zip(hosts, digs, hashes):
        want = np.concatenate([oracle.index_fixed(host[i * flen:(i + 1) * flen], bs)[2] for i in range(nf)])
        assert np.array_equal(d.cpu().numpy(), want)
        per_file = want.reshape(nf, -1, 20)
        assert [bytes(x) for x in h.cpu().numpy()] == [oracle.blocks_hash(per_file[i]) for i in range(nf)]


def test_stream_rejects_unaligned_runs(gpu):
    # 6 digests per file = 120-B runs: not 16-B aligned, the chained form refuses
    nf, flen, bs = 4, 4096 * 6, 4096
    st = device.BatchStream(nf, flen, bs)
    _, t = _batch(nf, flen, 1, gpu)
    d = torch.empty((nf * 6, 20), dtype=torch.uint8, device=gpu)
    st.push(t, d)
    with pytest.raises(SfError):
        st.push(t, torch.empty_like(d))  # its launch would chain the first batch


def test_push_last_single_batch(gpu):
    # a stream of one batch: push_last alone runs both halves and the chains
    nf, flen, bs = 33, 4096 * 256, 4096
    host, t = _batch(nf, flen, 77, gpu)
    st = device.BatchStream(nf, flen, bs)
    assert st._half_cols() == 128
    d = torch.empty((nf * flen // bs, 20), dtype=torch.uint8, device=gpu)
    (h,) = st.push_last(t, d)
    want = np.concatenate([oracle.index_fixed(host[i * flen:(i + 1) * flen], bs)[2] for i in range(nf)])
    assert np.array_equal(d.cpu().numpy(), want)
    per_file = want.reshape(nf, -1, 20)
    assert [bytes(x) for x in h.cpu().numpy()] == [oracle.blocks_hash(per_file[i]) for i in range(nf)]


def _cols(t, nf, flen, bs, lo, hi, d):
    from syncfast_amd._lib import ChainJob, lib
    arr = (ChainJob * 1)()
    return lib().sf_index_device_batch_chained_cols(t.data_ptr(), nf, flen, bs, lo, hi, d.data_ptr(), arr, 0,
                                                    torch.cuda.current_stream(t.device).cuda_stream)


def test_column_range_writes_only_its_rows(gpu):
    nf, flen, bs = 7, 4096 * 256, 4096  # 256 blocks per file
    host, t = _batch(nf, flen, 5, gpu)
    want = np.concatenate([oracle.index_fixed(host[i * flen:(i + 1) * flen], bs)[2] for i in range(nf)])
    want = want.reshape(nf, 256, 20)
    for lo, hi in [(0, 64), (64, 192), (192, 256), (0, 256)]:
        d = torch.full((nf * 256, 20), 0xA5, dtype=torch.uint8, device=gpu)
        assert _cols(t, nf, flen, bs, lo, hi, d) == 0
        got = d.cpu().numpy().reshape(nf, 256, 20)
        assert np.array_equal(got[:, lo:hi], want[:, lo:hi]), (lo, hi)
        assert (got[:, :lo] == 0xA5).all() and (got[:, hi:] == 0xA5).all(), (lo, hi)
    d = torch.empty((nf * 256, 20), dtype=torch.uint8, device=gpu)
    for lo, hi in [(0, 100), (32, 256), (64, 64), (128, 64), (0, 320)]:
        assert _cols(t, nf, flen, bs, lo, hi, d) == SF_EINVAL, (lo, hi)
    # a partial range of files that are not whole block waves is refused
    _, t2 = _batch(3, 4096 * 96, 6, gpu)
    d2 = torch.empty((3 * 96, 20), dtype=torch.uint8, device=gpu)
    assert _cols(t2, 3, 4096 * 96, 4096, 0, 64, d2) == SF_EINVAL
    assert _cols(t2, 3, 4096 * 96, 4096, 0, 96, d2) == 0  # whole files: any shape
