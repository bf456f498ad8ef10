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


def gather_digests(local: torch.Tensor, total_len: int, block_size: int,
                   group: Optional[dist.ProcessGroup] = None, dst: int = 0,
                   async_op: bool = False):
    """Gather every rank's uint8[n_r, 20] digest table to `dst`.

    Ranks may hold different block counts (uneven last shard): tables are
    padded to the largest shard for the collective and trimmed on `dst`.
    Returns the full uint8[n, 20] table on `dst` (None elsewhere); with
    async_op, returns (work, finish) where finish() -> table after
    work.wait()."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)  # shard index: the rank within `group`
    is_dst = dist.get_rank() == dst  # `dst` is a global rank, as dist.gather takes it
    counts = shard_blocks(total_len, block_size, world)
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
    size_t = torch.tensor([os.path.getsize(path) if is_dst else 0], dtype=torch.int64, device=where)
    dist.broadcast(size_t, src=dst, group=group)
    size = int(size_t.item())
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
