"""Rank 0 of the N-GPU bench, simulated on one GPU: does the gather of step
i's digest table delay step i+2 when only two tables rotate?

Per step: the SHA-1 launch writes table i % nbuf on the main stream; a side
stream (standing in for RCCL's receive kernel on rank 0) waits for that
launch and then writes 7 x 40 MiB (what rank 0 receives per step at N = 8)
with a device copy -- a CU-based blit, like RCCL's kernels; before the launch
that reuses a table, the main stream waits for the side stream's work on it
(what work.wait() does in bench.py).  Reported: ms per step for nbuf = 2, 3,
4, no side work, and nbuf = 3 with the receive on one step in 8 (the root
rotating over 8 ranks, bench.py's default), interleaved."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

GiB = 1 << 30


def run(data, nbuf, steps, recv_bytes, side, every=1):
    """every = k: this rank is the receiving root on one step in k (a root
    that rotates over k ranks); every = 1: a fixed root."""
    bs = 4096
    nblk = data.numel() // bs
    digs = [torch.empty((nblk, 20), dtype=torch.uint8, device=data.device) for _ in range(nbuf)]
    src = torch.empty(recv_bytes, dtype=torch.uint8, device=data.device)
    dst = [torch.empty(recv_bytes, dtype=torch.uint8, device=data.device) for _ in range(nbuf)]
    main = torch.cuda.current_stream()
    sstream = torch.cuda.Stream()
    done = [None] * nbuf
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        b = i % nbuf
        if done[b] is not None:
            main.wait_event(done[b])
        device.index_device(data, bs, out=digs[b], stream=main)
        if side and i % every == 0:
            ev = torch.cuda.Event()
            ev.record(main)
            sstream.wait_event(ev)
            with torch.cuda.stream(sstream):
                dst[b].copy_(src)  # the receive into rank 0's buffers
            done[b] = torch.cuda.Event()
            done[b].record(sstream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    n = 8 * GiB
    data = device.splitmix_tensor(n, 0x5EED0000)
    recv = 7 * 40 << 20
    for _ in range(30):  # clock ramp
        device.index_device(data, 4096)
    torch.cuda.synchronize()
    res = {}
    reps, steps = int(os.environ.get("SIM_REPS", "6")), int(os.environ.get("SIM_STEPS", "40"))
    for rep in range(reps):
        for name, nbuf, side, every in (("no gather", 2, False, 1), ("nbuf=2", 2, True, 1), ("nbuf=3", 3, True, 1),
                                        ("nbuf=4", 4, True, 1), ("nbuf=3, root rotating over 8", 3, True, 8)):
            ms = run(data, nbuf, steps, recv, side, every)
            res.setdefault(name, []).append(ms)
            print(f"rep {rep} {name}: {ms:.3f} ms/step", flush=True)
    for k, v in res.items():
        print(f"{k}: median {sorted(v)[len(v) // 2]:.3f} ms/step over {len(v)} reps", flush=True)


if __name__ == "__main__":
    main()
