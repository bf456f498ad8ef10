"""CPU: the gather plan of the single-process multi-device path.

sf_index_device_multi / _ex (syncfast_amd/csrc/sf_multi.cpp) hash shard r of
one file on device r and gather every shard's digest table to the root with
grouped RCCL send/recv (the table a file's blocks_hash needs,
src/index.rs:661-682).  The plan -- which device's rows land where in the
root's table, how many bytes each sender sends, which shard is hashed in
place and which is empty -- is exposed as sf_test_multi_plan and checked here
for N = 1..8 devices, every root, and file lengths with fewer blocks than
devices, a short last block and an exact multiple: the in-place and received
ranges tile the table exactly once, and every range agrees with
sf_shard_range and with syncfast_amd.shard.shard_range (the per-process
torch.distributed form's partition)."""
import ctypes
import random

import pytest

from syncfast_amd import host
from syncfast_amd._lib import lib
from syncfast_amd.shard import shard_range as torch_shard_range

NONE, IN_PLACE, SENT = 0, 1, 2


def plan(file_len, bs, n, root, self_gather=False):
    off = (ctypes.c_uint64 * n)()
    nbytes = (ctypes.c_uint64 * n)()
    route = (ctypes.c_int * n)()
    assert lib().sf_test_multi_plan(file_len, bs, n, root, int(self_gather), off, nbytes, route) == 0
    return list(off), list(nbytes), list(route)


def lengths(bs, n):
    rng = random.Random(bs * 31 + n)
    out = {0, 1, bs - 1, bs, bs + 1, n * bs, n * bs - 1, n * bs + 1, (n - 1) * bs + 5, 7 * n * bs,
           7 * n * bs + 13, (2 ** 20) * bs // 4096}
    out |= {rng.randrange(1, 200 * bs) for _ in range(6)}
    return sorted(x for x in out if x >= 0)


@pytest.mark.parametrize("bs", [4096, 1000, 65536])
@pytest.mark.parametrize("n", range(1, 9))
def test_plan_tiles_the_table_once(n, bs):
    for file_len in lengths(bs, n):
        nb = (file_len + bs - 1) // bs if file_len else 0
        for root in range(n):
            off, nbytes, route = plan(file_len, bs, n, root)
            covered = []
            for r in range(n):
                start, ln = host.shard_range(file_len, bs, n, r)
                assert (start, ln) == torch_shard_range(file_len, bs, n, r)
                rows = (ln + bs - 1) // bs if ln else 0
                assert nbytes[r] == 20 * rows, (file_len, n, root, r)
                if ln == 0:
                    assert route[r] == NONE, (file_len, n, root, r)
                    continue
                assert off[r] == (start // bs) * 20, (file_len, n, root, r)
                assert route[r] == (IN_PLACE if r == root else SENT), (file_len, n, root, r)
                covered.append((off[r], off[r] + nbytes[r]))
            # the root hashes in place or receives; every range exactly once
            covered.sort()
            pos = 0
            for a, b in covered:
                assert a == pos, (file_len, n, root, covered)
                pos = b
            assert pos == nb * 20, (file_len, n, root)
            # the root receives n_senders tables; no device sends to itself
            senders = [r for r in range(n) if route[r] == SENT]
            assert root not in senders
            assert len(senders) == sum(1 for r in range(n) if r != root and nbytes[r])


def test_fewer_blocks_than_devices():
    # 3 blocks over 8 devices: shards 3..7 are empty and take no part
    off, nbytes, route = plan(2 * 4096 + 5, 4096, 8, 6)
    assert route == [SENT, SENT, SENT, NONE, NONE, NONE, NONE, NONE]
    assert off[:3] == [0, 20, 40] and nbytes[:3] == [20, 20, 20]
    # root's own shard empty: it only receives
    assert route[6] == NONE


def test_self_gather_is_one_device_only():
    off, nbytes, route = plan(10 * 4096 + 1, 4096, 1, 0, self_gather=True)
    assert route == [SENT] and off == [0] and nbytes == [11 * 20]
    assert plan(10 * 4096 + 1, 4096, 1, 0)[2] == [IN_PLACE]
    # ignored with more than one device
    assert plan(10 * 4096, 4096, 2, 1, self_gather=True)[2] == [SENT, IN_PLACE]


def test_plan_rejects_bad_arguments():
    o, b, r = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), (ctypes.c_int * 2)()
    assert lib().sf_test_multi_plan(100, 0, 2, 0, 0, o, b, r) != 0
    assert lib().sf_test_multi_plan(100, 10, 0, 0, 0, o, b, r) != 0
    assert lib().sf_test_multi_plan(100, 10, 2, 2, 0, o, b, r) != 0
    assert lib().sf_test_multi_plan(100, 10, 2, 0, 0, None, b, r) != 0
