"""GPU: the multi-GPU composition HIP -> shard -> gather, on the one GPU of the box.

- Two rank processes (torch.multiprocessing spawn, gloo) each hash their
  shard_range piece of one logical file through the HIP kernel on cuda:0 and
  gather to rank 0, which must hold exactly the whole-file table (oracle) and
  blocks_hash -- the file -> shards -> table-in-order invariant of
  src/index.rs:629-656 with the real kernel in the loop.
- bench.py --gpus 2 without a launcher starts its two ranks itself and
  reports n_gpus = 2 (gloo rehearsal: both ranks share cuda:0; RCCL needs a
  GPU per rank, which the driver's 8-GPU run provides)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, total, bs, seed, q):
    import torch
    import torch.distributed as dist

    from syncfast_amd import device
    from syncfast_amd.shard import gather_digests, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        start, ln = shard_range(total, bs, world, rank)
        data = torch.empty(ln, dtype=torch.uint8, device=dev)
        device.fill_splitmix(data, seed, start)  # this rank's bytes of the one logical file
        dig = device.index_device(data, bs)
        torch.cuda.synchronize()
        full = gather_digests(dig, total, bs)
        if rank == 0:
            q.put(full.numpy().tobytes())
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,bs", [(2, (64 << 20) + 12345, 4096), (3, (48 << 20) + 1, 65536)])
def test_hip_shards_gathered_equal_whole_file(gpu, world, total, bs):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    seed = 0x5EED0003
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, total, bs, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = oracle.splitmix_bytes(total, seed)
    want = oracle.index_fixed_mt(whole, bs, 8)
    assert got == want.tobytes()
    assert oracle.blocks_hash(np.frombuffer(got, np.uint8)) == oracle.blocks_hash(want)


def test_bench_self_launches_two_ranks(gpu):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--shard-gib", "0.0625", "--steps", "3", "--warmup", "1", "--ramp-s", "0",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["total_bytes"] == 2 * (64 << 20)
    assert line["config"]["parallelism"].startswith("shard2+gloo_gather")
    assert line["value"] > 0
