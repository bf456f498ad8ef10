"""Where the time of the chained batch-stream launch goes (config 3 shape):
plain fixed kernel over the same 8 GiB, the chained kernel with and without
the previous batch's chains, and the chains alone (finish on an idle GPU).
Interleaved rounds in one process; medians in ms."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

GiB = 1 << 30


def main():
    nf, flen, bs = 1024, 8 << 20, 4096
    data = device.splitmix_tensor(nf * flen, 0x5EED0000)
    n = nf * flen // bs
    d = [torch.empty((n, 20), dtype=torch.uint8, device="cuda") for _ in range(2)]
    fh = torch.empty((nf, 20), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def plain():
        device.index_device(data, bs, out=d[0])

    st = device.BatchStream(nf, flen, bs)
    st.push(data, d[1])  # d[1] = "previous batch" from here on

    def chained():
        st._prev = d[1]
        st._launch(data, d[0], fh)

    def chained_nochain():
        st._prev = None
        st._launch(data, d[0], None)

    def chains_only():
        st._prev = d[1]
        st._launch(None, None, fh)

    cases = [("plain fixed", plain), ("chained (blocks + prev chains)", chained),
             ("chained, no chains", chained_nochain), ("chains only", chains_only)]
    for _ in range(30):
        plain()
    times = {k: [] for k, _ in cases}
    for _ in range(int(os.environ.get("ROUNDS", "8"))):
        for name, fn in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 5)
    for name, _ in cases:
        print(f"{name}: median {statistics.median(times[name]):.4f} ms  min {min(times[name]):.4f}", flush=True)


if __name__ == "__main__":
    main()
