#!/usr/bin/env python3
"""Round 6: does the stream-ordered allocator explain round 5's one
SF_ETIMEDOUT?  Round 5's library (SF_LIB=build_ab/libsf_r5.so, built from its
commit) ran sf_index_device_batch with a status word as ONE fused launch
whose chain lanes polled per-stage counters taken from hipMallocAsync on the
device's default pool.  scripts/fused_two_stream_stress.py queued 2000 such
launches with no synchronisation between them and never saw a timeout; the
sort workspace went wrong only when calls synchronised in between (the pool
then gives its freed blocks back: DESIGN.md 3.4).  Here: ITERS calls, each
followed by a device synchronisation (SYNC=1, default) or not (SYNC=0), 32 x
8 MiB files, every status word and blocks_hash checked.  Raw ctypes (round
5's library lacks this round's symbols).  One JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FileDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("len", ctypes.c_uint64)]


def main():
    import numpy as np
    import torch
    import hashlib
    L = ctypes.CDLL(os.environ["SF_LIB"])
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    L.sf_index_device_batch.argtypes = [vp, u64, vp, u32, u32, vp, u64, vp, vp, vp, vp, vp]
    L.sf_fill_splitmix_device.argtypes = [vp, u64, u64, u64, vp]
    dev = torch.device("cuda", 0)
    nf, flen, bs = 32, 8 << 20, 4096
    data = torch.empty(nf * flen, dtype=torch.uint8, device=dev)
    assert L.sf_fill_splitmix_device(data.data_ptr(), data.numel(), 91, 0, None) == 0
    descs = (FileDesc * nf)(*[FileDesc(i * flen, flen) for i in range(nf)])
    nb = nf * flen // bs
    dig = torch.empty((nb, 20), dtype=torch.uint8, device=dev)
    fh = torch.empty((nf, 20), dtype=torch.uint8, device=dev)
    iters, sync = int(os.environ.get("ITERS", "200")), os.environ.get("SYNC", "1") != "0"
    status = torch.zeros(iters, dtype=torch.int32, device=dev)
    nout = ctypes.c_uint64()
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    want = None
    bad_hash, t0 = 0, time.perf_counter()
    for i in range(iters):
        rc = L.sf_index_device_batch(data.data_ptr(), data.numel(), descs, nf, bs, dig.data_ptr(), nb,
                                     fh.data_ptr(), None, ctypes.byref(nout), status[i:i + 1].data_ptr(), s)
        assert rc == 0, rc
        if sync:
            torch.cuda.synchronize()
            h = fh.cpu().numpy().tobytes()
            if want is None:
                d = dig.cpu().numpy().reshape(nf, -1, 20)
                want = b"".join(hashlib.sha1(d[f].tobytes()).digest() for f in range(nf))
            bad_hash += h != want
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    print(json.dumps({"lib": os.path.basename(os.environ["SF_LIB"]), "sync_each_call": sync, "iters": iters,
                      "timeouts": int(np.count_nonzero(st == -110)), "other_status": sorted(set(int(x) for x in st) - {0, -110}),
                      "first_timeout": [int(x) for x in np.nonzero(st)[0][:5]], "wrong_blocks_hash": bad_hash,
                      "s": round(time.perf_counter() - t0, 2),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("SF_") and k != "SF_LIB"}}), flush=True)


if __name__ == "__main__":
    main()
