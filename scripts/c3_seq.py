"""Config 3 launch-duration decomposition (not a test): back-to-back
segments of K launches with no host sync in between -- plain fixed kernel,
then per library the chained kernel with no chain jobs and a batch stream
(K-1 pushes + push_last) -- repeated ROUNDS times (EVENTS=1: a timing event
recorded after every launch, as bench.py does), so a kernel trace (scripts/c3_seq.sh)
gives every launch's duration under the same clock and power state.

usage: python scripts/c3_seq.py [lib.so ...]   (default: the in-tree library)
Each extra library adds its two segments.  scripts/c3_seq_report.py reads
the trace."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402
from syncfast_amd._lib import LIB_PATH, ChainJob, check  # noqa: E402


def main():
    libs = sys.argv[1:] or [LIB_PATH]
    nf, flen, bs = 1024, 8 << 20, 4096
    K, rounds = int(os.environ.get("K", "20")), int(os.environ.get("ROUNDS", "3"))
    data = device.splitmix_tensor(nf * flen, 0x5EED0000)
    n = nf * flen // bs
    d = [torch.empty((n, 20), dtype=torch.uint8, device="cuda") for _ in range(3)]
    s = torch.cuda.current_stream()
    fns = []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        f = L.sf_index_device_batch_chained_cols
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                      ctypes.c_uint64, ctypes.c_void_p, ctypes.POINTER(ChainJob), ctypes.c_uint32, ctypes.c_void_p]
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

        def _launch(self, data_, digests, jobs, ref, cols=None):
            arr = (ChainJob * max(len(jobs), 1))(*jobs)
            lo, hi = cols if cols is not None else (0, self.nbf)
            check(self.f(data_.data_ptr() if data_ is not None else None, nf if data_ is not None else 0, flen, bs,
                         lo, hi, digests.data_ptr() if digests is not None else None, arr, len(jobs), s.cuda_stream),
                  "chained_cols")
            mark()

    events = os.environ.get("EVENTS") == "1"  # a timing event after every launch, as bench.py's step mode
    evs = []

    def mark():
        if events:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            evs.append(e)

    nb = ctypes.c_uint64()
    keep = []
    for r in range(rounds + 1):  # round 0 warms up
        for i in range(K):
            fns[0][1](data.data_ptr(), nf * flen, bs, d[i % 3].data_ptr(), n, ctypes.byref(nb), s.cuda_stream)
            mark()
        arr = (ChainJob * 1)()
        for f, _ in fns:
            for i in range(K):
                check(f(data.data_ptr(), nf, flen, bs, 0, n // nf, d[i % 3].data_ptr(), arr, 0, s.cuda_stream),
                      "blocks_only")
                mark()
            st = Stream(f)
            for i in range(K - 1):
                h = st.push(data, d[i % 3])
                if h is not None:
                    keep.append(h)
            keep += st.push_last(data, d[(K - 1) % 3])
    torch.cuda.synchronize()
    print(f"done: {rounds} rounds of K={K}; {len(keep)} hash tables", flush=True)


if __name__ == "__main__":
    main()
