"""CPU, world_size 2 and 3 over gloo: shard layout + digest-table gather.

Each rank plays one GPU: it takes its shard of one logical file, produces
that shard's digest table (here with the oracle, since there is no GPU), and
gathers to rank 0, which must hold exactly the whole-file table and
blocks_hash."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from syncfast_amd.shard import gather_digests, shard_blocks, shard_range


def test_shard_range_tiles_file():
    for total, bs, world in [(0, 4096, 2), (1, 4096, 3), (4096 * 10, 4096, 4), (4096 * 10 + 5, 4096, 3),
                             (12345678, 65536, 8), (100, 7, 5), (3 * 4096, 4096, 8)]:
        pos = 0
        for r in range(world):
            s, ln = shard_range(total, bs, world, r)
            assert s == pos and (s % bs == 0 or ln == 0)
            pos += ln
        assert pos == total
        assert sum(shard_blocks(total, bs, world)) == ((total + bs - 1) // bs if total else 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, bs, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, ln = shard_range(total, bs, world, rank)
        data = oracle.splitmix_bytes(ln, 0x5EED0000, start)  # this rank's shard of the file
        _, _, dig = oracle.index_fixed(data, bs)
        full = gather_digests(torch.from_numpy(dig), total, bs)
        work, finish = gather_digests(torch.from_numpy(dig), total, bs, async_op=True)
        work.wait()
        full2 = finish()
        if rank == 0:
            q.put((full.numpy().tobytes(), full2.numpy().tobytes()))
        else:
            assert full is None and full2 is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,bs", [(2, 4096 * 37 + 100, 4096), (3, 65536 * 5 + 1, 65536), (2, 1000, 4096)])
def test_gather_matches_whole_file(world, total, bs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, got_async = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole = oracle.splitmix_bytes(total, 0x5EED0000)
    _, _, want = oracle.index_fixed(whole, bs)
    assert got == want.tobytes() and got_async == want.tobytes()
    assert oracle.blocks_hash(np.frombuffer(got, np.uint8)) == oracle.blocks_hash(want)
