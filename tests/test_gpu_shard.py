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


def test_index_file_range_shards_concatenate(gpu, tmp_path):
    # sf_index_file_range: every shard_range piece of a file on disk, rows
    # with FILE offsets; concatenated in rank order = sf_index_file's rows
    from syncfast_amd import host
    from syncfast_amd._lib import SF_EINVAL, SF_ERANGE, SfError
    from syncfast_amd.shard import shard_range
    bs = 4096
    data = oracle.splitmix_bytes((40 << 20) + 777, 0x5EED0005)
    p = tmp_path / "f.bin"
    data.tofile(p)
    whole, bh = host.index_file(p, bs)
    for world in (1, 2, 3, 8):
        parts = [host.index_file_range(p, *shard_range(data.size, bs, world, r), bs) for r in range(world)]
        assert np.concatenate(parts).tobytes() == whole.tobytes(), world
    assert host.index_file_range(p, data.size, 0, bs).size == 0  # an empty shard at EOF (unaligned start)
    small = tmp_path / "small.bin"
    data[:10].tofile(small)
    pieces = [host.index_file_range(small, *shard_range(10, bs, 3, r), bs) for r in range(3)]
    assert [x.size for x in pieces] == [1, 0, 0]
    with pytest.raises(SfError) as e:
        host.index_file_range(p, 100, 4096, bs)  # start not block-aligned
    assert e.value.code == SF_EINVAL
    with pytest.raises(SfError) as e:
        host.index_file_range(p, 4096, data.size, bs)  # past the end
    assert e.value.code == SF_ERANGE


def _file_rank(rank, world, port, path, bs, q):
    import torch.distributed as dist

    from syncfast_amd.shard import index_file_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = index_file_sharded(path, bs)
        if rank == 0:
            rows, bh = res
            q.put((rows.tobytes(), bh))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


def test_index_file_sharded_two_ranks(gpu, tmp_path):
    # one file on disk, two ranks (sharing the box's GPU, gloo gather): rank 0
    # holds the whole file's rows and blocks_hash, equal to the oracle's
    import torch.multiprocessing as mp

    from syncfast_amd import host
    bs = 65536
    data = oracle.splitmix_bytes((24 << 20) + 12345, 0x5EED0006)
    p = tmp_path / "g.bin"
    data.tofile(p)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_file_rank, args=(r, 2, port, str(p), bs, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    rows_b, bh = q.get(timeout=100)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    rows = np.frombuffer(rows_b, host.SIG_DTYPE)
    offs, sizes, want = oracle.index_fixed(data, bs)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    assert np.array_equal(np.stack([r["sha1"] for r in rows]), want)
    assert bh == oracle.blocks_hash(want)


def _rccl_world1(port, q):
    import torch
    import torch.distributed as dist

    from syncfast_amd import device
    from syncfast_amd.shard import gather_digests
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        n, bs = (16 << 20) + 5, 4096
        data = device.splitmix_tensor(n, 0x5EED0008, dev)
        dig = device.index_device(data, bs)
        full = gather_digests(dig, n, bs)  # RCCL gather (to itself), synchronous form
        work, finish = gather_digests(dig, n, bs, async_op=True)
        work.wait()
        full2 = finish()
        torch.cuda.synchronize()
        ok = full.device.type == "cuda" and torch.equal(full, dig) and torch.equal(full2, dig)
        q.put((ok, dig.cpu().numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def test_rccl_gather_path_world1(gpu):
    # the bench's RCCL code path (backend "nccl" = RCCL on ROCm, device
    # tensors, sync and async gathers) on the one GPU of this box
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_world1, args=(_free_port(), q))
    p.start()
    ok, got = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0 and ok
    n, bs = (16 << 20) + 5, 4096
    assert got == oracle.index_fixed(oracle.splitmix_bytes(n, 0x5EED0008), bs)[2].tobytes()


def _list_rank(rank, world, port, path, offs, sizes, q, stale=False):
    import time

    import torch.distributed as dist

    from syncfast_amd import _lib, host
    from syncfast_amd.shard import index_file_blocks_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stamp = None
        if rank == 0:  # the chunking rank: its stamp, taken before the chunker read the file
            with open(path, "rb") as f:
                stamp = host.file_stamp(f.fileno())
            if stale:  # written after the chunker's stamp: no rank may hash it under that list
                time.sleep(0.02)
                with open(path, "r+b") as g:
                    g.seek(12345)
                    g.write(b"\x77" * 100)
        dist.barrier()
        try:
            res = index_file_blocks_sharded(path, offs, sizes, stamp=stamp)
        except _lib.SfError as e:
            q.put(("error", e.code, rank))
            return
        if rank == 0:
            rows, bh = res
            q.put((rows.tobytes(), bh))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


def test_hip_list_shards_stale_stamp_fails_every_rank(gpu, tmp_path):
    """the chunking rank's stamp is broadcast; a file written after
    it is SF_EAGAIN on every rank (the caller cuts it again), never a gathered
    table that mixes two versions."""
    import torch.multiprocessing as mp
    n = (8 << 20) + 3
    path = tmp_path / "cdc.bin"
    oracle.splitmix_bytes(n, 0x5EED0300).tofile(path)
    b = np.arange(0, n, 8000, dtype=np.uint64)
    offs, szs = b, np.diff(np.concatenate([b, [n]])).astype(np.uint32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_list_rank, args=(r, 2, port, str(path), offs, szs, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from syncfast_amd import _lib
    assert sorted(g[2] for g in got) == [0, 1] and all(g[0] == "error" and g[1] == _lib.SF_EAGAIN for g in got)


@pytest.mark.parametrize("world", [2, 3])
def test_hip_list_shards_gathered_equal_whole_list(gpu, tmp_path, world):
    """The default (content-defined) mode on N ranks: the host chunker's list
    split by list_shards, each rank hashing its blocks from the file through
    the HIP path (sf_index_file_blocks), gathered to rank 0 = the whole list's
    rows and blocks_hash (oracle)."""
    import torch.multiprocessing as mp

    from syncfast_amd import host
    rng = np.random.default_rng(world)
    n = (24 << 20) + 999
    data = oracle.splitmix_bytes(n, 0x5EED0200)
    path = tmp_path / "cdc.bin"
    data.tofile(path)
    sizes = np.minimum(rng.geometric(1 / 8192, n // 2000), 32768).astype(np.uint64)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    b = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    offs, szs = b[:-1], np.diff(b).astype(np.uint32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_list_rank, args=(r, world, port, str(path), offs, szs, q)) for r in range(world)]
    for p in procs:
        p.start()
    rows_b, bh = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = np.frombuffer(rows_b, host.SIG_DTYPE)
    want = oracle.index_blocks(data, offs, szs)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], szs)
    assert np.array_equal(rows["sha1"], want)
    assert bh == oracle.blocks_hash(want)
