"""Multi-GPU sharding of one logical file + RCCL gather of the signature table.

The reference indexes one file on one thread (src/index.rs:610-659).  Blocks
are independent, so a file splits into contiguous, block-aligned shards, one
per rank (one process per GPU, torch.distributed over RCCL/xGMI); each rank
hashes its shard with no communication.  The only exchange is the one the
single-file ``blocks_hash`` needs (src/index.rs:661-682 hashes ALL of a
file's digests in order): every shard's 20-byte digest table is gathered to
rank 0, which then owns the full (offset, size, SHA-1) table.

Everything here is backend-agnostic torch.distributed, so the same code runs
over RCCL on MI355X and over gloo in the CPU tests.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(total_len: int, block_size: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, block-aligned byte range [start, start+len) of `rank`.

    Blocks are dealt as evenly as possible (the first `nblocks % world` ranks
    get one extra); a rank may get an empty range.  Block i of the file is
    block (i - first_block) of the shard that holds it, so the concatenation
    of the shards' digest tables in rank order is the file's table."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    nblocks = (total_len + block_size - 1) // block_size if total_len else 0
    per, extra = divmod(nblocks, world)
    first = rank * per + min(rank, extra)
    count = per + (1 if rank < extra else 0)
    start = min(total_len, first * block_size)
    end = min(total_len, (first + count) * block_size)
    return start, max(0, end - start)


def shard_blocks(total_len: int, block_size: int, world: int) -> List[int]:
    """Number of blocks of every rank's shard."""
    out = []
    for r in range(world):
        _, ln = shard_range(total_len, block_size, world, r)
        out.append((ln + block_size - 1) // block_size if ln else 0)
    return out


def list_shards(offsets, sizes, world: int) -> List[int]:
    """Block-index cuts [c_0 = 0, c_1, ..., c_world = n] of an offset-ordered
    block list (a chunker's output): rank r takes blocks [c_r, c_{r+1}), the
    first block starting at or after r/world of the list's byte span, so
    the ranks' byte shares are about even (to within one block for a
    tiling list).  Content-defined
    boundaries need no fix-up between ranks here: the host chunker cut the
    whole file before the list was split."""
    import numpy as np
    offs = np.asarray(offsets, dtype=np.uint64).reshape(-1)
    n = offs.size
    if world < 1:
        raise ValueError("bad world")
    if n == 0:
        return [0] * (world + 1)
    lo = int(offs[0])
    hi = int((offs + np.asarray(sizes, dtype=np.uint64).reshape(-1)).max())
    cuts = [0]
    for r in range(1, world):
        target = lo + (hi - lo) * r // world
        cuts.append(max(cuts[-1], int(np.searchsorted(offs, np.uint64(target), side="left"))))
    cuts.append(n)
    return cuts


def gather_digests(local: torch.Tensor, total_len: int, block_size: int,
                   group: Optional[dist.ProcessGroup] = None, dst: int = 0,
                   async_op: bool = False):
    """Gather every rank's uint8[n_r, 20] digest table to `dst`.

    Ranks may hold different block counts (uneven last shard): tables are
    padded to the largest shard for the collective and trimmed on `dst`.
    Returns the full uint8[n, 20] table on `dst` (None elsewhere); with
    async_op, returns (work, finish) where finish() -> table after
    work.wait()."""
    counts = shard_blocks(total_len, block_size, dist.get_world_size(group))
    return gather_digests_counts(local, counts, group, dst, async_op)


def gather_digests_counts(local: torch.Tensor, counts: List[int], group: Optional[dist.ProcessGroup] = None,
                          dst: int = 0, async_op: bool = False):
    """gather_digests with every rank's row count given (an explicit block
    list's shards, list_shards)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)  # shard index: the rank within `group`
    is_dst = dist.get_rank() == dst  # `dst` is a global rank, as dist.gather takes it
    if len(counts) != world:
        raise ValueError("one count per rank")
    if local.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} digests, shard has {counts[rank]}")
    m = max(counts) if counts else 0
    if dist.get_backend(group) == "gloo" and local.device.type != "cpu":
        local = local.cpu()  # gloo gathers host tensors (rehearsal / CPU tests only)
    if local.shape[0] != m:
        padded = torch.zeros((m, 20), dtype=torch.uint8, device=local.device)
        padded[:local.shape[0]] = local
    else:
        padded = local
    bufs = [torch.empty_like(padded) for _ in range(world)] if is_dst else None
    work = dist.gather(padded, bufs, dst=dst, group=group, async_op=async_op)

    def finish():
        if not is_dst:
            return None
        return torch.cat([b[:c] for b, c in zip(bufs, counts)])

    if async_op:
        return work, finish
    return finish()


def index_file_sharded(path, block_size: int, group: Optional[dist.ProcessGroup] = None, dst: int = 0,
                       device: Optional[torch.device] = None):
    """One file on disk indexed by every rank of the group, each on its own
    GPU: rank r reads and hashes its shard_range of the file
    (sf_index_file_range, pread pipeline on the rank's current device), the
    shards' digest tables are gathered to `dst`, which rebuilds the file's rows
    and computes its blocks_hash (src/index.rs:661-682 chains over every
    digest, so it runs once, after the gather).

    The file's length is `dst`'s stat of it, broadcast, so every rank cuts the
    same shards even if the file changes meanwhile.  Before the gather the
    ranks agree on success: a rank whose read fails (the file shrank under
    it, an I/O error) raises its SfError and every other rank raises too,
    instead of waiting in a gather that rank never joins.

    Returns (rows SIG_DTYPE[n], blocks_hash bytes) on `dst`, None elsewhere.
    `device`: where the collectives' tensors live (the rank's GPU for RCCL;
    None = host tensors, for gloo).  `dst` is a rank of the default group."""
    import os

    import numpy as np

    from . import host
    from ._lib import SF_EIO, SfError
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)  # shard index: the rank within `group`
    is_dst = dist.get_rank() == dst  # `dst` is a global rank, as the collectives take it
    where = device if device is not None else torch.device("cpu")
    # dst's stat, broadcast; a stat that fails on dst is broadcast as -1 so
    # every rank raises after the broadcast instead of waiting in it
    stat_err: Optional[BaseException] = None
    size = 0
    if is_dst:
        try:
            size = os.path.getsize(path)
        except OSError as e:
            stat_err, size = e, -1
    size_t = torch.tensor([size], dtype=torch.int64, device=where)
    dist.broadcast(size_t, src=dst, group=group)
    size = int(size_t.item())
    if size < 0:
        if stat_err is not None:
            raise stat_err
        raise SfError(SF_EIO, f"index_file_sharded: rank {dst} could not stat {os.fsdecode(path)}")
    start, ln = shard_range(size, block_size, world, rank)
    failure: Optional[BaseException] = None
    try:
        rows = host.index_file_range(path, start, ln, block_size)
    except (SfError, OSError) as e:
        failure = e
    failed = torch.tensor([1 if failure is not None else 0], dtype=torch.int32, device=where)
    dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=group)
    if failure is not None:
        raise failure
    if int(failed.item()):
        raise SfError(SF_EIO, f"index_file_sharded: another rank failed to index its shard of {os.fsdecode(path)}")
    dig = torch.from_numpy(np.ascontiguousarray(rows["sha1"]).reshape(-1, 20))
    if device is not None:
        dig = dig.to(device)
    table = gather_digests(dig, size, block_size, group=group, dst=dst)
    if not is_dst:
        return None
    table = table.cpu().numpy()
    n = table.shape[0]
    out = np.zeros(n, host.SIG_DTYPE)
    out["offset"] = np.arange(n, dtype=np.uint64) * block_size
    out["size"] = block_size
    if n:
        out["size"][-1] = size - (n - 1) * block_size
    out["sha1"] = table
    return out, host.blocks_hash(table)


def index_file_blocks_sharded(path, offsets, sizes, group: Optional[dist.ProcessGroup] = None, dst: int = 0,
                              device: Optional[torch.device] = None, stamp=None):
    """The reference's default (content-defined) blocks of one file on N
    ranks: every rank holds the same offset-ordered list (the host chunker's
    output over the file, src/index.rs:622-625), takes its list_shards range
    and hashes those blocks from the file on its own GPU; the digests are
    gathered to `dst`, which returns the file's rows in list order and its
    blocks_hash (src/index.rs:661-682).

    One version of the file: `stamp` (on `dst`, host.file_stamp of the
    descriptor the chunker read, taken before it read) is broadcast, and
    every rank hashes its blocks from its own open of the path through
    sf_index_fd_blocks with that stamp as the expected one -- a file renamed
    over the path or written after the chunker's stamp gives SF_EAGAIN on the
    rank that sees it, and then on every rank, so the caller cuts the file
    again; the gathered table never mixes two versions.  Without a stamp each
    rank stamps its own open (the call still fails on a change during it).
    The ranks agree on success before the gather, as index_file_sharded does.
    Returns (rows, blocks_hash) on `dst`, None elsewhere."""
    import os

    import numpy as np

    from . import host
    from ._lib import SF_EAGAIN, SF_EIO, FileStamp, SfError
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    is_dst = dist.get_rank() == dst
    where = device if device is not None else torch.device("cpu")
    offs = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    szs = np.ascontiguousarray(sizes, dtype=np.uint32).reshape(-1)
    # dst's stamp to every rank (dev, ino, size, nlink, mtime, ctime; all -1: none)
    fields = [f for f, _t in FileStamp._fields_]
    st_t = torch.full((len(fields),), -1, dtype=torch.int64, device=where)
    if is_dst and stamp is not None:
        st_t = torch.tensor([ctypes.c_int64(int(getattr(stamp, f))).value for f in fields], dtype=torch.int64,
                            device=where)  # uint64 fields carried bit for bit
    dist.broadcast(st_t, src=dst, group=group)
    vals = st_t.cpu().tolist()
    expect = None
    if any(v != -1 for v in vals):
        expect = FileStamp(*[v & 0xFFFFFFFFFFFFFFFF if t is not ctypes.c_int64 else v
                             for v, (_f, t) in zip(vals, FileStamp._fields_)])
    cuts = list_shards(offs, szs, world)
    b0, b1 = cuts[rank], cuts[rank + 1]
    failure: Optional[BaseException] = None
    try:
        fd = os.open(path, os.O_RDONLY | os.O_NONBLOCK)
        try:
            rows, _ = host.index_fd_blocks(fd, offs[b0:b1], szs[b0:b1], expect)
        finally:
            os.close(fd)
    except (SfError, OSError, ValueError) as e:
        failure = e
    code = 0 if failure is None else (2 if isinstance(failure, SfError) and failure.code == SF_EAGAIN else 1)
    failed = torch.tensor([code], dtype=torch.int32, device=where)
    dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=group)
    if failure is not None:
        raise failure
    if int(failed.item()) == 2:
        raise SfError(SF_EAGAIN, f"index_file_blocks_sharded: {os.fsdecode(path)} changed under another rank")
    if int(failed.item()):
        raise SfError(SF_EIO, f"index_file_blocks_sharded: another rank failed on {os.fsdecode(path)}")
    dig = torch.from_numpy(np.ascontiguousarray(rows["sha1"]).reshape(-1, 20))
    if device is not None:
        dig = dig.to(device)
    counts = [cuts[r + 1] - cuts[r] for r in range(world)]
    table = gather_digests_counts(dig, counts, group=group, dst=dst)
    if not is_dst:
        return None
    table = table.cpu().numpy()
    out = np.zeros(offs.size, host.SIG_DTYPE)
    out["offset"] = offs
    out["size"] = szs
    out["sha1"] = table
    return out, host.blocks_hash(table)
