"""Config 3 (1024 x 8 MiB files, 4 KiB blocks, every blocks_hash) as two
streams: the plain sha1_fixed_kernel hashes batch i on the launch stream while
batch i-1's chains run alone (sha1_chain_helper_kernel, via
sf_index_device_batch_chained with no blocks) on a HIGH-priority stream that
waits for batch i-1's launch.  Interleaved against the plain kernel (config 2's
work, no blocks_hash) and the shipped fused batch stream (device.BatchStream).
Every blocks_hash of the last batch is compared between the two forms.

usage: python scripts/c3_two_stream.py   (C3_STEPS=20 C3_ROUNDS=4)
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402
from syncfast_amd._lib import ChainJob, check, lib  # noqa: E402

GiB = 1 << 30


def main():
    K = int(os.environ.get("C3_STEPS", "20"))
    rounds = int(os.environ.get("C3_ROUNDS", "4"))
    prio = int(os.environ.get("C3_PRIO", "-1"))
    dev = torch.device("cuda:0")
    nf, flen, bs = 1024, 8 << 20, 4096
    nbf = flen // bs
    data = device.splitmix_tensor(nf * flen, 0x5EED0000, dev)
    digs = [torch.empty((nf * nbf, 20), dtype=torch.uint8, device=dev) for _ in range(3)]
    hashes = [torch.empty((nf, 20), dtype=torch.uint8, device=dev) for _ in range(3)]
    A = torch.cuda.current_stream(dev)
    B = torch.cuda.Stream(dev, priority=prio)
    print("stream priorities", torch.cuda.Stream.priority_range(), "B", B.priority, flush=True)

    def chains(b, stream):
        job = ChainJob(digs[b].data_ptr(), nf, 0, nbf, None, hashes[b].data_ptr())
        arr = (ChainJob * 1)(job)
        check(lib().sf_index_device_batch_chained(None, 0, flen, bs, None, arr, 1, stream.cuda_stream),
              "sf_index_device_batch_chained")

    def run_plain():
        for i in range(K):
            device.index_device(data, bs, out=digs[i % 3], stream=A)

    def run_fused():
        bstream = device.BatchStream(nf, flen, bs, stream=A)
        out = None
        for i in range(K):
            if i == K - 1:
                out = bstream.push_last(data, digs[i % 3])[-1]
            else:
                bstream.push(data, digs[i % 3])
        return out

    evA = [torch.cuda.Event() for _ in range(3)]
    evB = [torch.cuda.Event() for _ in range(3)]

    def run_two():
        used = [False] * 3
        for i in range(K):
            b = i % 3
            if used[b]:
                A.wait_event(evB[b])  # batch i-3's chains have read digs[b]
            device.index_device(data, bs, out=digs[b], stream=A)
            evA[b].record(A)
            B.wait_event(evA[b])
            chains(b, B)
            evB[b].record(B)
            used[b] = True
        A.wait_event(evB[(K - 1) % 3])
        return hashes[(K - 1) % 3]

    forms = {"plain": run_plain, "fused": run_fused, "two_stream": run_two}
    for _ in range(3):  # warm + clock ramp
        for f in forms.values():
            f()
    torch.cuda.synchronize()
    times = {k: [] for k in forms}
    for r in range(rounds):
        order = list(forms) if r % 2 == 0 else list(reversed(forms))
        for k in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(A)
            forms[k]()
            e1.record(A)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / K)
        print(f"round {r} done", flush=True)
    h_fused = run_fused().clone()
    h_two = run_two().clone()
    torch.cuda.synchronize()
    assert torch.equal(h_fused, h_two), "blocks_hash differs between the fused and two-stream forms"
    res = {"steps": K, "rounds": rounds, "B_priority": B.priority}
    for k, v in times.items():
        med = statistics.median(v)
        res[k] = {"ms_per_batch": round(med, 4), "all": [round(x, 4) for x in v],
                  "GiB/s": round(nf * flen / GiB / (med * 1e-3), 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
