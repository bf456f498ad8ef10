"""Explicit-block-list throughput probe (not a test).

sf_index_device_blocks (sha1_table_kernel) over the same 4 GiB of HBM with
different block-size mixes, beside the fixed-tiling kernel on the same bytes:
  fixed4k   : sf_index_device_fixed, 4 KiB blocks (reference point)
  list4k    : the same 4 KiB tiling given as an explicit list
  cdc       : content-defined-like sizes -- geometric with mean 8 KiB, capped
              at 32 KiB, at least 1 B (the reference's default regime,
              ZPAQ 13 bits + max 32 KiB, src/index.rs:40-41)
  files     : ragged many-file batch: files of 0..200 KiB cut in 4 KiB blocks
              (each file's last block short), 16-B aligned file starts
Each list runs in list order (SF_TABLE_SORT=0) and sorted by block length
(SF_TABLE_SORT=1, the launcher's default from 2^17 blocks).  Every digest of each list run is compared with the fixed kernel where the
blocks coincide (list4k) and with a host SHA-1 spot check otherwise.
Usage: python scripts/ragged_probe.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syncfast_amd._lib import set_knob  # noqa: E402  (knobs are latched at load)
from syncfast_amd.device import fill_splitmix, index_device, index_device_blocks  # noqa: E402

GiB = 1 << 30


def cdc_sizes(total, rng):
    out, pos = [], 0
    while pos < total:
        s = int(min(32768, max(1, rng.geometric(1 / 8192))))
        s = min(s, total - pos)
        out.append(s)
        pos += s
    return np.array(out, np.int64)


def file_sizes(total, rng):
    offs, sizes, pos = [], [], 0
    while True:
        flen = int(rng.integers(0, 200 * 1024))
        if pos + flen > total:
            break
        nb = (flen + 4095) // 4096
        for b in range(nb):
            offs.append(pos + 4096 * b)
            sizes.append(min(4096, flen - 4096 * b))
        pos = (pos + flen + 15) & ~15
    return np.array(offs, np.int64), np.array(sizes, np.int64)


def timed(fn, s, reps=5):
    fn()
    s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    total = 4 * GiB
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    fill_splitmix(data, 0x5EED0000)
    rng = np.random.default_rng(7)
    s = torch.cuda.Stream(dev)
    t_end = time.perf_counter() + 0.5
    dig_fixed = torch.empty((total // 4096, 20), dtype=torch.uint8, device=dev)
    with torch.cuda.stream(s):
        while time.perf_counter() < t_end:
            index_device(data, 4096, out=dig_fixed, stream=s)
            s.synchronize()
    cases = {}
    offs4k = np.arange(total // 4096, dtype=np.int64) * 4096
    cases["list4k"] = (offs4k, np.full(offs4k.size, 4096, np.int64))
    sz = cdc_sizes(total, rng)
    cases["cdc"] = (np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.int64), sz)
    cases["files"] = file_sizes(total, rng)
    # diagnostic: the per-lane (unaligned) load path with no size imbalance
    cases["list4k_unaligned"] = (offs4k[:-1] + 1, np.full(offs4k.size - 1, 4096, np.int64))
    # diagnostic: the same unaligned 4 KiB blocks in a random order (every
    # wave's 64 blocks far apart in memory, as in a length-sorted CDC list)
    perm = rng.permutation(offs4k.size - 1)
    cases["list4k_unaligned_shuffled"] = (offs4k[:-1][perm] + 1, np.full(offs4k.size - 1, 4096, np.int64))
    if os.environ.get("PROBE_CLASS"):  # length-class width A/B on the CDC list (SF_TABLE_CLASS_BITS)
        cases = {"cdc": cases["cdc"], "files": cases["files"]}
    if os.environ.get("PROBE_ALIGN"):  # per-lane path at dword (+4) and 8-B (+8) alignment
        cases = {}
        for sh in (1, 4, 8):
            cases[f"list4k_plus{sh}"] = (offs4k[:-1] + sh, np.full(offs4k.size - 1, 4096, np.int64))
    out = {}
    for rep in range(2):
        ms = timed(lambda: index_device(data, 4096, out=dig_fixed, stream=s), s)
        out["fixed4k"] = {"ms": round(ms, 3), "GiB/s": round(total / GiB / (ms * 1e-3), 1)}
        modes = [("0", None), ("1", None)]
        if os.environ.get("PROBE_CLASS"):
            modes = [("1", b) for b in ("2", "3", "4", "5", "6")]
        for (name, (o, z)), (srt, cb) in [(c, m) for c in cases.items() for m in modes]:
            # SF_TABLE_SORT: 0 = list order, 1 = blocks sorted by length (the default from 2^17 blocks)
            set_knob("SF_TEST_TABLE_SORT", int(srt))
            if cb:
                set_knob("SF_TABLE_CLASS_BITS", int(cb))
            name = name + ("_sorted" if srt == "1" else "") + (f"_m{cb}" if cb else "")
            to = torch.from_numpy(o).to(dev)
            tz = torch.from_numpy(z.astype(np.int32)).to(dev)
            dig = torch.empty((o.size, 20), dtype=torch.uint8, device=dev)
            ms = timed(lambda: index_device_blocks(data, to, tz, out=dig, check_range=False, stream=s), s)
            nbytes = int(z.sum())
            out[name] = {"ms": round(ms, 3), "GiB/s": round(nbytes / GiB / (ms * 1e-3), 1), "blocks": int(o.size),
                         "mean_block": round(nbytes / o.size, 1)}
            if rep == 0:
                d = dig.cpu().numpy()
                if name in ("list4k", "list4k_sorted"):
                    assert np.array_equal(d, dig_fixed.cpu().numpy()), name
                for i in rng.integers(0, o.size, 64):
                    b = data[int(o[i]): int(o[i]) + int(z[i])].cpu().numpy().tobytes()
                    assert bytes(d[i]) == hashlib.sha1(b).digest(), (name, i)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
