"""Rank 0 of the N-GPU bench, simulated on one GPU: does the gather of step
i's digest table delay step i+2 when only two tables rotate?

Per step: the SHA-1 launch writes table i % nbuf on the main stream; a side
stream (standing in for RCCL's receive kernel on rank 0) waits for that
launch and then writes 7 x 40 MiB (what rank 0 receives per step at N = 8)
with a device copy -- a CU-based blit, like RCCL's kernels; before the launch
that reuses a table, the main stream waits for the side stream's work on it
(what work.wait() does in bench.py).  Reported: ms per step for nbuf = 2, 3
and no side work, interleaved."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

GiB = 1 << 30


def run(data, nbuf, steps, recv_bytes, side):
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
        if side:
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
        for name, nbuf, side in (("no gather", 2, False), ("nbuf=2", 2, True), ("nbuf=3", 3, True),
                                 ("nbuf=4", 4, True)):
            ms = run(data, nbuf, steps, recv, side)
            res.setdefault(name, []).append(ms)
            print(f"rep {rep} {name}: {ms:.3f} ms/step", flush=True)
    for k, v in res.items():
        print(f"{k}: median {sorted(v)[len(v) // 2]:.3f} ms/step over {len(v)} reps", flush=True)


if __name__ == "__main__":
    main()
