"""GPU: equal-size many-file batches as a stream (sf_index_device_batch_chained
through device.BatchStream): each launch hashes one batch's blocks and the
previous batch's per-file blocks_hash (src/index.rs:661-682).  Every digest
and every blocks_hash is compared with the oracle."""
import numpy as np
import pytest
import torch

import oracle
from syncfast_amd import SfError, device

pytestmark = pytest.mark.gpu


def _batch(nf, flen, seed, dev):
    host = np.concatenate([oracle.splitmix_bytes(flen, seed + i) for i in range(nf)])
    return host, torch.from_numpy(host).to(dev)


@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("nf,flen,bs", [(64, 4096 * 16, 4096), (300, 4096 * 8, 4096), (5, 65536 * 4, 65536),
                                         (70, 1000 * 4, 1000)])
def test_stream_every_digest_and_hash(gpu, nf, flen, bs, split):
    st = device.BatchStream(nf, flen, bs, split=split)
    hosts, digs, hashes = [], [], []
    for k in range(4):
        host, t = _batch(nf, flen, 0x5EED0000 + 1000 * k, gpu)
        d = torch.empty((nf * flen // bs, 20), dtype=torch.uint8, device=gpu)
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
