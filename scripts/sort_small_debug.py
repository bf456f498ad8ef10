#!/usr/bin/env python3
"""Debug (round 6): explicit lists sorted from 128 blocks gave one wrong
digest through sf_index_fd_cut in the C consumer.  Here the same 3 MiB file
(splitmix seed 904) and its stand-in boundaries through every route that
takes launch_table -- sf_index_fd_cut (1 and 4 threads), sf_index_fd_blocks,
sf_index_device_blocks from a torch tensor -- with the sort forced on and
off, each call twice, against the oracle; prints the wrong block indices."""
import ctypes
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import oracle
    from syncfast_amd import _lib, device, host
    Z = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "build", "libzpaq_standin.so"))
    Z.sf_zpaq_standin_ops.restype = ctypes.c_void_p
    Z.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]
    ops = Z.sf_zpaq_standin_ops(13, 32768)
    for n, seed in ((3 << 20, 904), (9 << 20, 906), (64 << 20, 5)):
        d = oracle.splitmix_bytes(n, seed)
        sizes = oracle.zpaq_standin_sizes(d).astype(np.uint32)
        offs = np.concatenate([[0], np.cumsum(sizes, dtype=np.uint64)[:-1]]).astype(np.uint64)
        want = oracle.index_blocks(d, offs, sizes)
        tmp = tempfile.mkdtemp()
        p = os.path.join(tmp, "f")
        d.tofile(p)
        fd = os.open(p, os.O_RDONLY)
        t = torch.from_numpy(d).cuda()
        for sort in (1, 0):
            _lib.set_knob("SF_TEST_TABLE_SORT", sort)
            for rep in range(2):
                res = {}
                for th in (1, 4):
                    rows, _bh = host.index_fd_cut(fd, ops, th)
                    res[f"fd_cut_t{th}"] = rows["sha1"]
                rows, _bh = host.index_fd_blocks(fd, offs, sizes)
                res["fd_blocks"] = rows["sha1"]
                res["device_blocks"] = device.index_device_blocks(
                    t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                    torch.from_numpy(sizes.view(np.int32)).cuda()).cpu().numpy()
                for k, v in res.items():
                    bad = np.nonzero(np.any(np.asarray(v).reshape(-1, 20) != want, axis=1))[0]
                    print(json.dumps({"bytes": n, "blocks": int(sizes.size), "sort": sort, "rep": rep, "route": k,
                                      "wrong": int(bad.size), "first_wrong": [int(x) for x in bad[:8]]}), flush=True)
        os.close(fd)
        os.unlink(p)
        os.rmdir(tmp)


if __name__ == "__main__":
    main()
