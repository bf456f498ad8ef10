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
    # in place (regions locked one ahead, rows + blocks_hash overlapped), in
    # place serial (whole range locked first, rows after: the earlier form),
    # staged through pinned buffers
    routes = (("in place, overlapped", {}), ("in place, serial", {"SF_INPLACE_SERIAL": "1"}),
              ("staged memcpy", {"SF_NO_HOSTREG": "1"}))
    for rep in range(2):
        for name, env in routes:
            os.environ.update(env)
            t0 = time.perf_counter()
            rows = host.index_buffer(data, 4096)
            t = time.perf_counter() - t0
            for k in env:
                del os.environ[k]
            print(f"sf_index_buffer {n / GiB:.0f} GiB, 4 KiB blocks, {name} (rep {rep}):", rate(n, t), flush=True)
    assert rows.shape[0] == n // 4096
    d = os.environ.get("E2E_DIR", "/tmp")
    with tempfile.NamedTemporaryFile(dir=d, delete=False) as f:
        f.write(data.tobytes())
        path = f.name
    try:
        # the pread pipeline (stages read by 16 threads, rows + blocks_hash per
        # stage); the file is never mapped and page-locked
        for i in range(4):
            t0 = time.perf_counter()
            rows, bh = host.index_file(path, 4096)
            t = time.perf_counter() - t0
            what = "cold-ish" if i == 0 else "page cache, pread pipeline"
            print(f"sf_index_file {n / GiB:.0f} GiB ({what}), incl. blocks_hash:", rate(n, t), flush=True)
    finally:
        os.unlink(path)
    many_files(data, d)
    wire_rate()


def wire_rate():
    """FILE_BLOCK run of config 2's table (2^21 blocks) streamed to a file
    descriptor (/dev/null: device build + D2H + write syscalls)."""
    from syncfast_amd import device, wire
    from syncfast_amd._lib import set_knob
    n = 8 << 30
    t = device.splitmix_tensor(n, 0x5EED0000)
    dig = device.index_device(t, 4096)
    torch.cuda.synchronize()
    with open("/dev/null", "wb") as f:
        wire.file_blocks_to_fd(dig, 4096, n, f.fileno())  # warm up
        for rep in range(2):
            for chunk in ("65536", "262144", "1048576"):  # messages per chunk (SF_TEST_WIRE_CHUNK; default 262144)
                set_knob("SF_TEST_WIRE_CHUNK", int(chunk))
                t0 = time.perf_counter()
                nbytes = wire.file_blocks_to_fd(dig, 4096, n, f.fileno())
                dt = time.perf_counter() - t0
                print(f"wire: FILE_BLOCK run of 2^21 blocks ({nbytes / 1e6:.1f} MB) to an fd, chunk {chunk}: "
                      f"{nbytes / dt / 1e9:.2f} GB/s ({dig.shape[0] / dt / 1e6:.1f} M messages/s)", flush=True)
        set_knob("SF_TEST_WIRE_CHUNK", 0)


def many_files(data, d):
    """index_path's shape: many files from the page cache, (a) through the
    one native pipeline sf_index_files, (b) one sf_index_file per file (the
    reference's per-file structure), (c) Index.index_path incl. SQLite rows."""
    import shutil
    from syncfast_amd.index import FixedChunker, Index
    rng = np.random.default_rng(1)
    cases = [("config-3 shape, 8 MiB files", [8 << 20] * (data.size // (8 << 20))),
             ("mixed 0-200 KiB files", [])]
    left = data.size
    while left > 200 << 10:
        k = int(rng.integers(0, 200 << 10))
        cases[1][1].append(k)
        left -= k
    for name, sizes in cases:
        root = tempfile.mkdtemp(dir=d)
        try:
            paths, off = [], 0
            for i, k in enumerate(sizes):
                p = os.path.join(root, f"f{i:06d}")
                with open(p, "wb") as f:
                    f.write(data[off:off + k].tobytes())
                paths.append(p)
                off += k
            total = off
            host.index_files(paths[:8], 4096)  # warm up
            t0 = time.perf_counter()
            rows, first, fh = host.index_files(paths, 4096)
            ta = time.perf_counter() - t0
            print(f"sf_index_files {len(paths)} {name} ({total / GiB:.2f} GiB), rows + blocks_hash:",
                  rate(total, ta), flush=True)
            t0 = time.perf_counter()
            for k, p in enumerate(paths):
                r1, bh1 = host.index_file(p, 4096)
            tb = time.perf_counter() - t0
            assert r1.tobytes() == rows[int(first[-2]):].tobytes() and bh1 == bytes(fh[-1])
            print(f"  one sf_index_file per file: {rate(total, tb)}  -> pipeline x{tb / ta:.1f}", flush=True)
            idx = Index.open(os.path.join(root, ".syncfast.idx"), chunker=FixedChunker(4096))
            t0 = time.perf_counter()
            idx.index_path(root)
            idx.commit()
            tc = time.perf_counter() - t0
            print(f"  Index.index_path (walk + pipeline + SQLite rows): {rate(total, tc)}", flush=True)
        finally:
            shutil.rmtree(root)


if __name__ == "__main__":
    if os.environ.get("E2E_ONLY") == "wire":
        wire_rate()
    else:
        main()
