"""Per-wave timeline of sha1_table_kernel (diagnostic build, -DSF_WAVE_TRACE).

usage: python scripts/table_trace.py TRACE_LIB.so OUT.npz [lists]
  lists: comma list of cdc, list4k (default both)

Each wave of the traced kernel writes its start / end (s_memrealtime, 100 MHz),
HW_ID, XCC_ID, its longest block's compressions and its path (slot / aligned)
into a trace buffer.  The CDC-like 4 GiB list of scripts/cdc_ab.py (same
seed) and the 4 KiB list are run untraced (timing), then traced; the traced
digests must equal the untraced ones.  scripts/table_trace_report.py reads
the .npz: occupancy over time per SIMD, the tail, wave length vs duration.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cdc_ab import GiB, bind, cdc_sizes  # noqa: E402
from syncfast_amd import device  # noqa: E402


def main():
    lib, out = sys.argv[1], sys.argv[2]
    pick = (sys.argv[3] if len(sys.argv) > 3 else "cdc,list4k").split(",")
    total = int(float(os.environ.get("CDC_GIB", "4")) * GiB)
    dev = torch.device("cuda:0")
    data = device.splitmix_tensor(total, 0x5EED0000, dev)
    rng = np.random.default_rng(7)
    sz = cdc_sizes(total, rng)
    offs = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.int64)
    lists = {"cdc": (offs, sz)}
    o4 = np.arange(total // 4096, dtype=np.int64) * 4096
    lists["list4k"] = (o4, np.full(o4.size, 4096, np.int64))
    lists = {k: lists[k] for k in pick}
    L = ctypes.CDLL(os.path.abspath(lib))
    L.sf_trace_set.argtypes = [ctypes.c_void_p]
    fb, ff = bind(lib)
    s = torch.cuda.current_stream(dev)
    nfix = total // 4096
    fixed_out = torch.empty((nfix, 20), dtype=torch.uint8, device=dev)
    nb = ctypes.c_uint64()
    t_end = time.time() + 0.5
    while time.time() < t_end:  # clock ramp
        assert ff(data.data_ptr(), total, 4096, fixed_out.data_ptr(), nfix, ctypes.byref(nb), s.cuda_stream) == 0
        torch.cuda.synchronize()
    res = {}
    for k, (o, z) in lists.items():
        do = torch.from_numpy(o).to(dev)
        dz = torch.from_numpy(z.astype(np.int32)).to(dev)
        ref = torch.empty((o.size, 20), dtype=torch.uint8, device=dev)
        got = torch.empty_like(ref)
        nwaves = (o.size + 63) // 64
        tr = torch.zeros(nwaves * 8, dtype=torch.int32, device=dev)

        def run(outp):
            assert fb(data.data_ptr(), total, do.data_ptr(), dz.data_ptr(), o.size, outp.data_ptr(), None,
                      s.cuda_stream) == 0

        L.sf_trace_set(None)
        ms = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            run(ref)
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        L.sf_trace_set(tr.data_ptr())
        tms = []
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            run(got)
            e1.record(s)
            torch.cuda.synchronize()
            tms.append(e0.elapsed_time(e1))
        L.sf_trace_set(None)
        assert torch.equal(ref, got), f"{k}: traced digests differ"
        t = tr.cpu().numpy().view(np.uint32).reshape(nwaves, 8)
        res[k] = t
        res[k + "_ms"] = np.array(ms)
        res[k + "_traced_ms"] = np.array(tms)
        print(f"{k}: {o.size} blocks, untraced {np.median(ms):.4f} ms, traced {np.median(tms):.4f} ms, "
              f"{int(z.sum()) / GiB / (np.median(ms) * 1e-3):.1f} GiB/s", flush=True)
    np.savez_compressed(out, **res)
    print("saved", out)


if __name__ == "__main__":
    main()
