"""End-to-end rates (host memory / file -> H2D -> kernel -> D2H rows).

Not the headline metric (that is device-resident); recorded in DESIGN.md.
Inputs are random host bytes (numpy), sizes bounded to fit the box."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syncfast_amd import host  # noqa: E402

GiB = 1 << 30


def rate(n, t):
    return f"{n / GiB / t:.2f} GiB/s ({n / t / 1e9:.2f} GB/s)"


def main():
    n = int(float(os.environ.get("E2E_GIB", "4")) * GiB)
    rng = np.random.default_rng(0)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    # raw PCIe reference: pinned H2D copy with torch
    pin = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    dev.copy_(pin, non_blocking=True); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        dev.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    print("pinned H2D (torch, 4x1 GiB):", rate(4 << 30, time.perf_counter() - t0), flush=True)
    host.index_buffer(data[: 256 << 20], 4096)  # warm up
    for knob in ("0", "1"):
        os.environ["SF_NO_HOSTREG"] = knob
        t0 = time.perf_counter()
        rows = host.index_buffer(data, 4096)
        t = time.perf_counter() - t0
        print(f"sf_index_buffer {n / GiB:.0f} GiB, 4 KiB blocks, {'staged memcpy' if knob == '1' else 'hostRegister'}:",
              rate(n, t), flush=True)
    assert rows.shape[0] == n // 4096
    d = os.environ.get("E2E_DIR", "/tmp")
    with tempfile.NamedTemporaryFile(dir=d, delete=False) as f:
        f.write(data.tobytes())
        path = f.name
    try:
        for i in range(2):
            t0 = time.perf_counter()
            rows, bh = host.index_file(path, 4096)
            t = time.perf_counter() - t0
            print(f"sf_index_file {n / GiB:.0f} GiB ({'cold-ish' if i == 0 else 'page cache'}), incl. blocks_hash:",
                  rate(n, t), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
