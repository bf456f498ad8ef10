"""FILE_BLOCK run build rate on the device (not a test): 2^21 messages of
config 2's fixed tiling (sf_wire_file_blocks_device) against the same count
of content-defined-like sizes (sf_wire_blocks_device: lengths, scan, scatter;
blocking read of the total).  Best of REPS, HIP events around each call."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syncfast_amd import wire  # noqa: E402


def best(fn, reps):
    out, ms = None, []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        out = fn()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return out, min(ms)


def main():
    n, bs, reps = 1 << 21, 4096, int(os.environ.get("REPS", "5"))
    dev = torch.device("cuda:0")
    dig = torch.randint(0, 256, (n, 20), dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(1)
    sizes = torch.from_numpy(np.minimum(rng.geometric(1 / 8192, n), 32768).astype(np.int32)).to(dev)
    fixed, ms_f = best(lambda: wire.file_blocks_device(dig, bs, n * bs), reps)
    var, ms_v = best(lambda: wire.blocks_device(dig, sizes), reps)
    for name, out, ms in (("fixed", fixed, ms_f), ("content-defined sizes", var, ms_v)):
        print(f"{name}: {n} messages, {out.numel() / 1e6:.1f} MB in {ms:.3f} ms = "
              f"{out.numel() / ms / 1e6:.1f} GB/s, {n / ms / 1e6:.2f} G messages/s", flush=True)


if __name__ == "__main__":
    main()
