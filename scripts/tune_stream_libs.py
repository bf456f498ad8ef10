"""Interleaved A/B of library builds on config 3 as a batch stream (not a test).

usage: python scripts/tune_stream_libs.py lib1.so lib2.so ...
Each .so is loaded with ctypes and drives device.BatchStream's launches
(sf_index_device_batch_chained, split chains); per round and build: K pushes
+ finish over 1024 x 8 MiB files, ms per batch; the plain fixed kernel of the
first build is timed beside them as the reference point.  Every build's
digests and blocks_hash must agree."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402
from syncfast_amd._lib import ChainJob, check  # noqa: E402


def main():
    libs = sys.argv[1:]
    nf, flen, bs, K = 1024, 8 << 20, 4096, int(os.environ.get("K", "10"))
    data = device.splitmix_tensor(nf * flen, 0x5EED0000)
    n = nf * flen // bs
    d = [torch.empty((n, 20), dtype=torch.uint8, device="cuda") for _ in range(3)]
    s = torch.cuda.current_stream()
    fns = []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        f = L.sf_index_device_batch_chained
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                      ctypes.POINTER(ChainJob), ctypes.c_uint32, ctypes.c_void_p]
        f.restype = ctypes.c_int
        g = L.sf_index_device_fixed
        g.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
        g.restype = ctypes.c_int
        fns.append((f, g))

    class Stream(device.BatchStream):
        def __init__(self, f):
            super().__init__(nf, flen, bs)
            self.f = f

        def _launch(self, data_, digests, jobs, ref):
            arr = (ChainJob * max(len(jobs), 1))(*jobs)
            check(self.f(data_.data_ptr() if data_ is not None else None, nf if data_ is not None else 0, flen, bs,
                         digests.data_ptr() if digests is not None else None, arr, len(jobs), s.cuda_stream),
                  "sf_index_device_batch_chained")

    def run_stream(f):
        st = Stream(f)
        out = []
        for i in range(K):
            h = st.push(data, d[i % 3])
            if h is not None:
                out.append(h)
        out += st.finish()
        return out

    nb = ctypes.c_uint64()

    def plain():
        for i in range(K):
            fns[0][1](data.data_ptr(), nf * flen, bs, d[i % 3].data_ptr(), n, ctypes.byref(nb), s.cuda_stream)

    def blocks_only():  # the chained kernel with no chain jobs: its block part alone
        arr = (ChainJob * 1)()
        for i in range(K):
            check(fns[0][0](data.data_ptr(), nf, flen, bs, d[i % 3].data_ptr(), arr, 0, s.cuda_stream), "chained")

    for _ in range(30):
        plain()
    ref = None
    names = ["plain", "blocks_only"] + libs
    times = {name: [] for name in names}
    for _ in range(int(os.environ.get("ROUNDS", "6"))):
        for name in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if name == "plain":
                plain()
                hs = None
            elif name == "blocks_only":
                blocks_only()
                hs = None
            else:
                hs = run_stream(fns[libs.index(name)][0])
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / K)
            if hs is not None:
                got = torch.cat([h.cpu() for h in hs])
                if ref is None:
                    ref = got
                assert torch.equal(got, ref), f"{name}: blocks_hash differs"
    for name in names:
        print(f"{name}: median {statistics.median(times[name]):.4f} ms/batch  min {min(times[name]):.4f}", flush=True)


if __name__ == "__main__":
    main()
