"""Cost of the first call of each device path in a fresh process (what a
one-shot index run pays once): each entry point timed on a tiny input, first
call then second call, in a fixed order.

usage: python scripts/first_call_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(name, fn):
    out = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    print(f"{name}: first {out[0]:.2f} ms, second {out[1]:.2f} ms", flush=True)


def main():
    t0 = time.perf_counter()
    torch.zeros(1, device="cuda")
    print(f"torch CUDA init: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    t0 = time.perf_counter()
    from syncfast_amd import device, host, wire
    from syncfast_amd._lib import lib
    lib()
    print(f"import + load library: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    data = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    timed("fill_splitmix", lambda: device.fill_splitmix(data, 1))
    timed("index_device (fixed kernel)", lambda: device.index_device(data, 4096))
    offs = torch.arange(0, 1 << 20, 4096, dtype=torch.int64, device="cuda")
    sizes = torch.full((256,), 4096, dtype=torch.int32, device="cuda")
    timed("index_device_blocks (table kernel)", lambda: device.index_device_blocks(data, offs, sizes))
    eq = [(i * 65536, 65536) for i in range(16)]
    timed("index_device_batch equal, status (staged kernel)", lambda: device.index_device_batch(data, eq, 4096))
    rag = [(i * 65536, 65536 - 16 * i) for i in range(16)]
    timed("index_device_batch ragged (table + chains, hipMallocAsync)",
          lambda: device.index_device_batch(data, rag, 4096))
    dig = device.index_device(data, 4096)
    timed("wire.file_blocks_device", lambda: wire.file_blocks_device(dig, 4096, 1 << 20))
    buf = bytes(1 << 20)
    timed("host.index_buffer 1 MiB (in place)", lambda: host.index_buffer(buf, 4096))
    timed("host.index_buffer 64 KiB (staged)", lambda: host.index_buffer(buf[:65536], 4096))


if __name__ == "__main__":
    main()
