"""Config 3 as a stream of batches: per-batch time of the plain fixed kernel
(no blocks_hash, reference point) vs the batch stream with whole chains and
with split chains (blocks_hash of every file included).  Each stream round =
10 pushes + finish; interleaved rounds in one process; medians in ms/batch."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402


def main():
    nf, flen, bs = 1024, 8 << 20, 4096
    data = device.splitmix_tensor(nf * flen, 0x5EED0000)
    n = nf * flen // bs
    d = [torch.empty((n, 20), dtype=torch.uint8, device="cuda") for _ in range(3)]
    s = torch.cuda.current_stream()
    K = 10

    def plain():
        for i in range(K):
            device.index_device(data, bs, out=d[i % 3])

    def stream(split):
        def run():
            st = device.BatchStream(nf, flen, bs, split=split)
            for i in range(K):
                st.push(data, d[i % 3])
            st.finish()
        return run

    cases = [("plain fixed (no blocks_hash)", plain), ("stream, whole chains", stream(False)),
             ("stream, split chains", stream(True))]
    for _ in range(3):
        plain()
    times = {k: [] for k, _ in cases}
    for _ in range(int(os.environ.get("ROUNDS", "6"))):
        for name, fn in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / K)
    for name, _ in cases:
        print(f"{name}: median {statistics.median(times[name]):.4f} ms/batch  min {min(times[name]):.4f}", flush=True)


if __name__ == "__main__":
    main()
