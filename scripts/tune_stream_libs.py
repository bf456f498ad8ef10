"""Interleaved A/B of library builds on config 3 as a batch stream (not a test).

usage: python scripts/tune_stream_libs.py lib1.so lib2.so ...
Each .so is loaded with ctypes and drives device.BatchStream's launches
(sf_index_device_batch_chained_cols, split chains); per round and build: K
pushes + finish over 1024 x 8 MiB files, ms per batch, and (":last", LAST=1
default) K-1 pushes + push_last; the plain fixed kernel of the
first build is timed beside them as the reference point.  Every build's
digests and blocks_hash must agree (checked after the timed rounds, so no
host work idles the GPU between them; builds whose file name contains
"exp" compute wrong hashes on purpose and are not checked).  The order of
the runs rotates from round to round."""
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
                  "sf_index_device_batch_chained_cols")

    def run_stream(f, emid, last):
        st = Stream(f)
        out = []
        for i in range(K - (1 if last else 0)):
            h = st.push(data, d[i % 3])
            if h is not None:
                out.append(h)
        if last:  # the last batch in two column halves (BatchStream.push_last)
            out += st.push_last(data, d[(K - 1) % 3])
            emid.record(s)
        else:
            emid.record(s)  # the pushes alone (without the finish)
            out += st.finish()
        return out

    nb = ctypes.c_uint64()

    def plain():
        for i in range(K):
            fns[0][1](data.data_ptr(), nf * flen, bs, d[i % 3].data_ptr(), n, ctypes.byref(nb), s.cuda_stream)

    def blocks_only():  # the chained kernel with no chain jobs: its block part alone
        arr = (ChainJob * 1)()
        for i in range(K):
            check(fns[0][0](data.data_ptr(), nf, flen, bs, 0, n // nf, d[i % 3].data_ptr(), arr, 0, s.cuda_stream),
                  "chained")

    for _ in range(30):
        plain()
    runs = libs + [p + ":last" for p in libs] if os.environ.get("LAST", "1") == "1" else libs
    names = ["plain", "blocks_only"] + runs
    times = {name: [] for name in names}
    pushes = {name: [] for name in runs}
    last = {}
    for r in range(int(os.environ.get("ROUNDS", "6"))):
        for name in names[r % len(names):] + names[:r % len(names)]:  # rotated: no name always runs first
            e0, e1, em = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(s)
            if name == "plain":
                plain()
            elif name == "blocks_only":
                blocks_only()
            else:
                lib_name = name.rsplit(":last", 1)[0]
                last[name] = run_stream(fns[libs.index(lib_name)][0], em, name.endswith(":last"))
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / K)
            if name in pushes:
                pushes[name].append(e0.elapsed_time(em) / K)
    ref = None
    for name, hs in last.items():
        if "exp" in os.path.basename(name):
            continue
        got = torch.cat([h.cpu() for h in hs])
        if ref is None:
            ref = got
        assert torch.equal(got, ref), f"{name}: blocks_hash differs"
    for name in names:
        extra = f"  (pushes alone {statistics.median(pushes[name]):.4f})" if name in pushes else ""
        print(f"{name}: median {statistics.median(times[name]):.4f} ms/batch  min {min(times[name]):.4f}{extra}",
              flush=True)


if __name__ == "__main__":
    main()
