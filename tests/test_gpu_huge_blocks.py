"""GPU: explicit blocks of 2 GiB and more, and the u32 edges of the block
kernels' arithmetic.

* Blocks of 2^32 - 8 ... 2^32 - 1 bytes: (size + 8) wraps in 32 bits, so the
  explicit-list paths count compressions without the wrap (n_chunks_wide);
  the reference hashes a block of any length (src/index.rs:629-646).  One
  launch holds a wave of such blocks (span >= 4 GiB: the per-lane path) and a
  wave of blocks of 2^31 + 13, 2^31 + 1 and 2^31 bytes at byte offsets (the
  144-B slot path), while another thread hashes a 2^31 + 13-byte block from
  host memory through sf_index_buffer_blocks (a block larger than a stage).
  Every digest is checked against hashlib over the same bytes.  One lane
  hashes a 4 GiB block alone: ~2^26 sequential compressions, over a minute.
* A blocks_hash chain job whose 64 files' digest runs span more than 4 GiB in
  one wave (3.4 M blocks per file): the block launch's chain wave addresses
  a wave's runs with 32-bit offsets, so such a job runs on the 64-bit helper
  kernel instead; every file's blocks_hash vs hashlib over its digest run."""
import concurrent.futures as cf
import hashlib

import numpy as np
import pytest
import torch

from syncfast_amd import device, host

pytestmark = pytest.mark.gpu


def _sha1(buf, off, size):
    return hashlib.sha1(memoryview(buf)[off:off + size]).digest()


@pytest.mark.timeout(600)
def test_blocks_of_2gib_and_past_the_u32_chunk_count_wrap(gpu):
    n = (1 << 32) + 64
    data = device.splitmix_tensor(n, 0x5EED0900, gpu)
    rng = np.random.default_rng(900)
    # wave 0 (list positions 0..63): blocks of 2^32 - 9 .. 2^32 - 1 bytes, span >= 4 GiB
    w0 = [(0, 0xFFFFFFFF), (1, 0xFFFFFFF8), (6, 0xFFFFFFFB), (13, 0xFFFFFFF7)]
    w0 += [(int(rng.integers(0, n - 400)), int(rng.integers(0, 300))) for _ in range(64 - len(w0))]
    # wave 1 (64..127): blocks of >= 2^31 bytes at byte offsets, span < 3.75 GiB
    big = (1 << 31) + 13
    w1 = [(7, big), (3, (1 << 31) + 1), (64, 1 << 31), (12345, 777)]
    w1 += [(int(rng.integers(0, (1 << 31) - 400)), int(rng.integers(0, 300))) for _ in range(64 - len(w1))]
    blocks = w0 + w1
    offs = torch.tensor([o for o, _s in blocks], dtype=torch.int64, device=gpu)
    sizes = torch.from_numpy(np.array([s for _o, s in blocks], np.uint32).view(np.int32)).to(gpu)
    host_copy = data.cpu().numpy()
    torch.cuda.synchronize()
    # the host route in parallel: a 2^31 + 13-byte block between two small ones
    hb = host_copy[: big + 64]
    hl = ([0, 5, 5 + big], [5, big, 20])

    def host_route():
        return host.index_buffer_blocks(hb, *hl)

    with cf.ThreadPoolExecutor(8) as pool:
        out = device.index_device_blocks(data, offs, sizes, check_range=False)  # async on the stream
        h_fut = pool.submit(host_route)
        want = list(pool.map(lambda b: _sha1(host_copy, *b), blocks))
        h_want = [_sha1(hb, o, s) for o, s in zip(*hl)]
        h_rows, h_bh = h_fut.result()
        torch.cuda.synchronize()
    got = out.cpu().numpy()
    bad = [i for i in range(len(blocks)) if bytes(got[i]) != want[i]]
    assert not bad, [(i, blocks[i]) for i in bad]
    assert [bytes(r) for r in h_rows["sha1"]] == h_want
    assert h_bh == hashlib.sha1(b"".join(h_want)).digest()


@pytest.mark.timeout(300)
def test_chain_job_whose_wave_spans_more_than_4gib(gpu):
    n_files, bs, nbf = 64, 16, 3_400_000  # run_len 68 MB: 64 runs pass 4 GiB
    file_len = nbf * bs
    data = device.splitmix_tensor(n_files * file_len, 0x5EED0901, gpu)
    dig = [torch.empty((n_files * nbf, 20), dtype=torch.uint8, device=gpu) for _ in range(3)]
    # split chains: launch 2 carries batch 0's first halves, launch 3 its second
    # halves and batch 1's first, beside block work; finish() the rest alone
    bs_stream = device.BatchStream(n_files, file_len, bs)
    done = [bs_stream.push(data, d) for d in dig]
    done += bs_stream.finish()
    hashes = [h for h in done if h is not None]
    assert len(hashes) == 3
    torch.cuda.synchronize()
    assert torch.equal(dig[0], dig[1]) and torch.equal(dig[0], dig[2])
    runs = dig[0].cpu().numpy().reshape(n_files, nbf * 20)
    with cf.ThreadPoolExecutor(8) as pool:
        want = list(pool.map(lambda f: hashlib.sha1(runs[f].data).digest(), range(n_files)))
    for h in hashes:
        got = h.cpu().numpy()
        assert [bytes(got[f]) for f in range(n_files)] == want
