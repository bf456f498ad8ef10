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


def _fake_index_file_range(path, start, length, bs):
    """CPU stand-in for sf_index_file_range (no GPU here): the oracle's rows of
    the byte range, file offsets -- only the shard/gather/rebuild logic of
    index_file_sharded is under test."""
    from syncfast_amd.host import SIG_DTYPE
    data = np.fromfile(path, np.uint8)[start:start + length]
    offs, sizes, dig = oracle.index_fixed(data, bs)
    out = np.zeros(offs.size, SIG_DTYPE)
    out["offset"], out["size"], out["sha1"] = offs + start, sizes, dig
    return out


def _file_worker(rank, world, port, path, bs, q):
    import syncfast_amd.host as h
    from syncfast_amd.shard import index_file_sharded
    h.index_file_range = _fake_index_file_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = index_file_sharded(path, bs)
        if rank == 0:
            q.put((res[0].tobytes(), res[1]))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,bs", [(2, 4096 * 37 + 100, 4096), (3, 65536 * 5 + 1, 65536), (3, 10, 4096)])
def test_index_file_sharded_rebuilds_rows(tmp_path, world, total, bs):
    from syncfast_amd.host import SIG_DTYPE
    p = tmp_path / "f"
    data = oracle.splitmix_bytes(total, 0x5EED0007)
    data.tofile(p)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_file_worker, args=(r, world, port, str(p), bs, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    rows_b, bh = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    rows = np.frombuffer(rows_b, SIG_DTYPE)
    offs, sizes, want = oracle.index_fixed(data, bs)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    assert np.array_equal(rows["sha1"], want)
    assert bh == oracle.blocks_hash(want)


def _failing_worker(rank, world, port, path, bs, q):
    import syncfast_amd.host as h
    from syncfast_amd._lib import SF_EIO, SfError
    from syncfast_amd.shard import index_file_sharded

    def fake(path, start, length, bs_):
        if rank == world - 1:  # this rank's read fails (e.g. the file shrank under it)
            raise SfError(SF_EIO, "sf_index_file_range")
        return _fake_index_file_range(path, start, length, bs_)
    h.index_file_range = fake
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        index_file_sharded(path, bs)
        q.put((rank, "returned"))
    except SfError as e:
        q.put((rank, "SfError" if e.code == SF_EIO else f"code {e.code}"))
    finally:
        dist.destroy_process_group()


def test_index_file_sharded_one_rank_fails_all_raise(tmp_path):
    # no rank is left waiting in the gather: every rank raises
    p = tmp_path / "f"
    oracle.splitmix_bytes(4096 * 10, 1).tofile(p)
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, str(p), 4096, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert got == {r: "SfError" for r in range(world)}


def _missing_on_dst_worker(rank, world, port, path, bs, q):
    import syncfast_amd.host as h
    from syncfast_amd._lib import SfError
    from syncfast_amd.shard import index_file_sharded
    h.index_file_range = _fake_index_file_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        index_file_sharded(path, bs)
        q.put((rank, "returned"))
    except FileNotFoundError:
        q.put((rank, "FileNotFoundError"))
    except SfError:
        q.put((rank, "SfError"))
    finally:
        dist.destroy_process_group()


def test_index_file_sharded_missing_on_dst_all_raise(tmp_path):
    """dst cannot stat the file: it broadcasts -1 instead of raising before
    the broadcast, so no rank waits in a collective dst never joins; dst
    raises the OSError, the others SfError."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_missing_on_dst_worker, args=(r, world, port, str(tmp_path / "gone"), 4096, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert got == {0: "FileNotFoundError", 1: "SfError", 2: "SfError"}


def _subgroup_worker(rank, world, port, path, bs, q):
    import syncfast_amd.host as h
    from syncfast_amd.shard import index_file_sharded
    h.index_file_range = _fake_index_file_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sub = dist.new_group([1, 2])  # every rank takes part in new_group
        if rank in (1, 2):
            # dst is a GLOBAL rank (2), which is rank 1 inside the subgroup
            res = index_file_sharded(path, bs, group=sub, dst=2)
            q.put((rank, None if res is None else (res[0].tobytes(), res[1])))
    finally:
        dist.destroy_process_group()


def test_index_file_sharded_subgroup_global_dst(tmp_path):
    from syncfast_amd.host import SIG_DTYPE
    p = tmp_path / "f"
    total, bs = 4096 * 21 + 7, 4096
    data = oracle.splitmix_bytes(total, 0x5EED0009)
    data.tofile(p)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, str(p), bs, q)) for r in range(3)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert got[1] is None
    rows = np.frombuffer(got[2][0], SIG_DTYPE)
    offs, sizes, want = oracle.index_fixed(data, bs)
    assert np.array_equal(rows["offset"], offs) and np.array_equal(rows["size"], sizes)
    assert np.array_equal(rows["sha1"], want) and got[2][1] == oracle.blocks_hash(want)


def test_list_shards_partition_a_block_list():
    from syncfast_amd.shard import list_shards
    rng = np.random.default_rng(4)
    for n_blocks, world in [(0, 3), (1, 4), (10, 2), (5000, 8), (777, 3)]:
        sizes = np.minimum(rng.geometric(1 / 8192, n_blocks), 32768).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) if n_blocks else np.zeros(0, np.uint64)
        cuts = list_shards(offs, sizes, world)
        assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == n_blocks
        assert all(a <= b for a, b in zip(cuts, cuts[1:]))
        if n_blocks > 100 * world:  # tiling list: every rank's bytes within one block (32 KiB) of an even share
            total = int(sizes.sum())
            for r in range(world):
                share = int(sizes[cuts[r]:cuts[r + 1]].sum())
                assert abs(share - total / world) <= 2 * 32768


def _list_worker(rank, world, port, data, offs, sizes, q):
    from syncfast_amd.shard import gather_digests_counts, list_shards
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cuts = list_shards(offs, sizes, world)
        mine = oracle.index_blocks(data, offs[cuts[rank]:cuts[rank + 1]], sizes[cuts[rank]:cuts[rank + 1]])
        counts = [cuts[r + 1] - cuts[r] for r in range(world)]
        full = gather_digests_counts(torch.from_numpy(mine), counts)
        if rank == 0:
            q.put(full.numpy().tobytes())
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_of_list_shards_is_the_list_table(world):
    """An explicit (content-defined-like) list split by list_shards, each
    rank's digests gathered with uneven counts: rank 0 holds the list's table
    in list order (digests by the oracle here: no GPU on this machine)."""
    rng = np.random.default_rng(world)
    n = 600_000
    data = oracle.splitmix_bytes(n, 0x5EED0100)
    sizes = np.minimum(rng.geometric(1 / 8192, n // 1000), 32768).astype(np.uint64)
    cuts = np.cumsum(sizes)
    cuts = cuts[cuts < n]
    b = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    offs, szs = b[:-1], np.diff(b).astype(np.uint32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_list_worker, args=(r, world, port, data, offs, szs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == oracle.index_blocks(data, offs, szs).tobytes()
