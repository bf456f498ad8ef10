"""Content-defined block lists through sha1_table_kernel: timing + interleaved A/B.

usage: python scripts/cdc_ab.py [lib1.so lib2.so ...]
  (no libs: the in-tree library)

4 GiB of splitmix64 bytes in HBM, three lists over the same bytes:
  cdc      geometric sizes, mean 8 KiB, capped at 32 KiB, >= 1 B, byte offsets
           (the reference's default regime: ZPAQ 13 bits, max 32 KiB,
           src/index.rs:40-41), blocks sorted by length class (the launcher's
           default from 2^17 blocks)
  list4k   the 4 KiB tiling given as a list (16-B aligned, LDS path)
  fixed4k  sf_index_device_fixed on the same bytes (reference point)
Each library is loaded with ctypes; rounds are interleaved, every digest of
every library must agree with the first, and the cdc list is spot-checked
against hashlib.  CDC_ROUNDS (default 6) rounds of CDC_REPS (5) launches.
CDC_ONLY=1 runs only the cdc list (rocprof passes); CDC_LISTS=list4k (or
cdc,list4k) picks the lists, without the fixed-kernel reference point;
cdc16 = the cdc sizes with every block 16-B aligned (the aligned LDS path);
a8k / u8k = equal 8 KiB blocks at 16-B aligned / byte offsets (stride 8195);
files = a ragged many-file batch (files of 0..200 KiB in 4 KiB blocks, each
file's last block short, 16-B aligned file starts).
GiB/s are of the bytes each list covers.
"""
import ctypes
import hashlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402
from syncfast_amd._lib import LIB_PATH  # noqa: E402

GiB = 1 << 30


def cdc_sizes(total, rng):
    s = np.minimum(32768, np.maximum(1, rng.geometric(1 / 8192, size=total // 4096))).astype(np.int64)
    c = np.cumsum(s)
    n = int(np.searchsorted(c, total))
    s = s[: n + 1]
    s[-1] -= int(c[n] - total) if c[n] > total else 0
    s = s[s > 0]
    assert int(s.sum()) == total
    return s


def bind(path):
    L = ctypes.CDLL(os.path.abspath(path))
    fb = L.sf_index_device_blocks
    fb.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    fb.restype = ctypes.c_int
    ff = L.sf_index_device_fixed
    ff.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    ff.restype = ctypes.c_int
    return fb, ff


def main():
    libs = sys.argv[1:] or [LIB_PATH]
    total = int(float(os.environ.get("CDC_GIB", "4")) * GiB)
    rounds = int(os.environ.get("CDC_ROUNDS", "6"))
    reps = int(os.environ.get("CDC_REPS", "5"))
    only = os.environ.get("CDC_ONLY") == "1"
    pick = [x for x in os.environ.get("CDC_LISTS", "").split(",") if x]
    only = only or bool(pick)
    dev = torch.device("cuda:0")
    data = device.splitmix_tensor(total, 0x5EED0000, dev)
    rng = np.random.default_rng(7)
    sz = cdc_sizes(total, rng)
    offs = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.int64)
    lists = {"cdc": (offs, sz)}
    if "cdc16" in pick:  # the same sizes, every block 16-B aligned (gaps of < 16 B; blocks past 4 GiB dropped)
        o16 = np.zeros_like(offs)
        o16[1:] = (np.cumsum((sz[:-1] + 15) // 16 * 16))
        keep = o16 + sz <= total
        lists["cdc16"] = (o16[keep], sz[keep])
    for name, stride in (("a8k", 8192), ("u8k", 8195)):  # equal 8 KiB blocks: aligned / byte offsets
        if name in pick:
            o = np.arange((total - 8192) // stride + 1, dtype=np.int64) * stride
            lists[name] = (o, np.full(o.size, 8192, np.int64))
    if "files" in pick:  # a ragged many-file batch: files of 0..200 KiB in 4 KiB blocks, 16-B aligned starts
        fl = rng.integers(0, 200 * 1024, total // (100 * 1024) + 16)
        starts = np.concatenate([[0], np.cumsum((fl + 15) // 16 * 16)[:-1]])
        fl, starts = fl[starts + fl <= total], starts[starts + fl <= total]
        nb = (fl + 4095) // 4096
        fo = np.repeat(starts, nb) + 4096 * (np.arange(int(nb.sum())) - np.repeat(np.cumsum(nb) - nb, nb))
        fz = np.minimum(4096, np.repeat(starts + fl, nb) - fo)
        lists["files"] = (fo.astype(np.int64), fz.astype(np.int64))
    if not only or "list4k" in pick:
        o4 = np.arange(total // 4096, dtype=np.int64) * 4096
        lists["list4k"] = (o4, np.full(o4.size, 4096, np.int64))
    if pick:
        lists = {k: lists[k] for k in pick}
    dl = {k: (torch.from_numpy(o).to(dev), torch.from_numpy(z.astype(np.int32)).to(dev)) for k, (o, z) in lists.items()}
    B = [bind(p) for p in libs]
    s = torch.cuda.current_stream(dev)
    nfix = total // 4096
    outs = {(i, k): torch.empty((lists[k][0].size, 20), dtype=torch.uint8, device=dev)
            for i in range(len(libs)) for k in lists}
    fixed_out = torch.empty((nfix, 20), dtype=torch.uint8, device=dev)
    nb = ctypes.c_uint64()

    def run(i, k):
        if k == "fixed4k":
            assert B[i][1](data.data_ptr(), total, 4096, fixed_out.data_ptr(), nfix, ctypes.byref(nb),
                           s.cuda_stream) == 0
            return
        o, z = dl[k]
        assert B[i][0](data.data_ptr(), total, o.data_ptr(), z.data_ptr(), o.numel(), outs[(i, k)].data_ptr(),
                       None, s.cuda_stream) == 0

    for _ in range(int(0.5 * 3400 / (total / GiB))):  # clock ramp (~0.5 s of the fixed kernel)
        run(0, "fixed4k")
    torch.cuda.synchronize()
    names = list(lists) + ([] if only else ["fixed4k"])
    times = {(i, k): [] for i in range(len(libs)) for k in names}
    # the library measured first after another list runs ~3 % slow on the
    # 4 KiB list (profiles/r04/s20, s21): the order rotates every round
    # (CDC_ROTATE=0: fixed order, as before round 4's s22)
    rotate = os.environ.get("CDC_ROTATE", "1") == "1"
    for r in range(rounds):
        for k in names:
            for j in range(len(libs)):
                i = (j + r) % len(libs) if rotate else j
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    run(i, k)
                e1.record(s)
                torch.cuda.synchronize()
                times[(i, k)].append(e0.elapsed_time(e1) / reps)
        print(f"round {r} done", flush=True)
    # parity: every library = the first; cdc spot-checked with hashlib; list4k = fixed kernel
    for k in lists:
        for i in range(1, len(libs)):
            assert torch.equal(outs[(i, k)], outs[(0, k)]), (libs[i], k)
    if not only:
        run(0, "fixed4k")
        assert torch.equal(outs[(0, "list4k")], fixed_out), "list4k != fixed kernel"
    if "cdc" in lists:
        d = outs[(0, "cdc")].cpu().numpy()
        for j in list(rng.integers(0, offs.size, 200)) + [0, offs.size - 1]:
            b = data[int(offs[j]): int(offs[j]) + int(sz[j])].cpu().numpy().tobytes()
            assert bytes(d[j]) == hashlib.sha1(b).digest(), j
    res = {"blocks": {k: int(lists[k][0].size) for k in lists}, "bytes": total,
           "list_bytes": {k: int(lists[k][1].sum()) for k in lists},
           "mean_block": round(total / offs.size, 1)}
    for i, p in enumerate(libs):
        for k in names:
            med = statistics.median(times[(i, k)])
            nb = int(lists[k][1].sum()) if k in lists else total
            res[f"{os.path.basename(p)}:{k}"] = {"ms": round(med, 4), "min_ms": round(min(times[(i, k)]), 4),
                                                 "GiB/s": round(nb / GiB / (med * 1e-3), 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
