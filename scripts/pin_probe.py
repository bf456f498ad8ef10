import time, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from syncfast_amd import host
n = 4 << 30
pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
a = pinned.numpy(); a[:] = 7
b = np.full(n, 7, np.uint8)
host.index_buffer(b[:256 << 20], 4096)
for rep in range(2):
    for name, buf in (("pinned", a), ("pageable", b)):
        t0 = time.perf_counter(); host.index_buffer(buf, 4096); t = time.perf_counter() - t0
        print(f"sf_index_buffer 4 GiB {name} (rep {rep}): {n / t / 1e9:.2f} GB/s", flush=True)
