#!/usr/bin/env python3
"""Fused many-file launches (sf_index_device_batch with a status word:
sha1_staged_kernel with its blocks_hash chains) alternating on
two streams with nothing between them -- the pattern of round 5's
sf_index_files stages when its one SF_ETIMEDOUT happened (run in
round 6 on the waiting form, 2000 launches without a timeout, and kept for the
no-wait form, whose status word is never written).
Each launch's counter words come from hipMallocAsync on its stream and go back with
hipFreeAsync behind the kernel, so this also exercises the stream-ordered
allocator handing one launch's freed counters to the other stream's next
launch.  Every status word must stay 0 and every blocks_hash equal the
product's host SHA-1 over the digests.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--files", type=int, default=32)
    ap.add_argument("--file-mib", type=int, default=8)
    a = ap.parse_args()
    import numpy as np
    import torch
    from syncfast_amd import device, host
    dev = torch.device("cuda", 0)
    flen = a.file_mib << 20
    data = [device.splitmix_tensor(a.files * flen, 4242 + k, device=dev) for k in range(2)]
    files = [(i * flen, flen) for i in range(a.files)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    nb = a.files * (flen // 4096)
    digs = [torch.empty((nb, 20), dtype=torch.uint8, device=dev) for _ in range(2)]
    fhs = [torch.empty((a.files, 20), dtype=torch.uint8, device=dev) for _ in range(2)]
    status = torch.zeros(a.launches, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.launches):
        k = i & 1
        with torch.cuda.stream(streams[k]):
            device.index_device_batch(data[k], files, 4096, out=digs[k], hashes_out=fhs[k], stream=streams[k],
                                      status=status[i:i + 1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = status.cpu().numpy()
    bad = int(np.count_nonzero(st))
    ok_hashes = True
    for k in range(2):
        d = digs[k].cpu().numpy().reshape(a.files, -1, 20)
        fh = fhs[k].cpu().numpy()
        for f in (0, a.files // 2, a.files - 1):
            ok_hashes &= bytes(fh[f]) == host.blocks_hash(d[f])
    print(json.dumps({"launches": a.launches, "files": a.files, "file_mib": a.file_mib,
                      "nonzero_status": bad, "first_bad": [int(x) for x in np.nonzero(st)[0][:10]],
                      "status_values": sorted(set(int(x) for x in st)), "last_hashes_ok": bool(ok_hashes),
                      "seconds": round(dt, 3)}), flush=True)
    sys.exit(1 if bad or not ok_hashes else 0)


if __name__ == "__main__":
    main()
