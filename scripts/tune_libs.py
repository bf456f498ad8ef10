"""Interleaved A/B of differently-compiled builds of the library in ONE process.

usage: python scripts/tune_libs.py lib1.so lib2.so ...
Each .so is loaded with ctypes; sf_index_device_fixed is timed on the same
8 GiB HBM buffer, rounds interleaved; digests must agree."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

GiB = 1 << 30


def main():
    libs = sys.argv[1:]
    size = int(float(os.environ.get("TUNE_GIB", "8")) * GiB)
    bs = int(os.environ.get("TUNE_BS", "4096"))
    data = device.splitmix_tensor(size, 0x5EED0000)
    n = size // bs
    Ls = []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        f = L.sf_index_device_fixed
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
        f.restype = ctypes.c_int
        Ls.append(f)
    s = torch.cuda.current_stream()
    outs = [torch.empty((n, 20), dtype=torch.uint8, device="cuda") for _ in libs]
    nb = ctypes.c_uint64()
    times = [[] for _ in libs]
    # clock ramp
    for _ in range(40):
        Ls[0](data.data_ptr(), size, bs, outs[0].data_ptr(), n, ctypes.byref(nb), s.cuda_stream)
    if os.environ.get("TUNE_MODE") == "batch":  # config 3: 1024 x 8 MiB + per-file blocks_hash
        return batch(libs, data, size, bs, s)
    for r in range(int(os.environ.get("TUNE_ROUNDS", "6"))):
        for i, f in enumerate(Ls):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                assert f(data.data_ptr(), size, bs, outs[i].data_ptr(), n, ctypes.byref(nb), s.cuda_stream) == 0
            e1.record(s)
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 5)
    for i, p in enumerate(libs):
        if "noload" not in p:
            assert torch.equal(outs[i], outs[0]), p
        med = statistics.median(times[i])
        print(f"{os.path.basename(p)}: median {med:.4f} ms min {min(times[i]):.4f} -> "
              f"{size / GiB / (med * 1e-3):.1f} GiB/s", flush=True)


def batch(libs, data, size, bs, s):
    from syncfast_amd._lib import FileDesc
    nf = int(os.environ.get("TUNE_FILES", "1024"))
    flen = size // nf
    files = (FileDesc * nf)(*[FileDesc(i * flen, flen) for i in range(nf)])
    n = size // bs
    fs, dig, fh = [], [], []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        f = L.sf_index_device_batch
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(FileDesc), ctypes.c_uint32, ctypes.c_uint32,
                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_void_p]
        f.restype = ctypes.c_int
        fs.append(f)
        dig.append(torch.empty((n, 20), dtype=torch.uint8, device="cuda"))
        fh.append(torch.empty((nf, 20), dtype=torch.uint8, device="cuda"))
    nb = ctypes.c_uint64()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")  # chain status (SF_ETIMEDOUT), checked at the end
    times = [[] for _ in libs]

    def call(i):
        assert fs[i](data.data_ptr(), size, files, nf, bs, dig[i].data_ptr(), n, fh[i].data_ptr(), None,
                     ctypes.byref(nb), st.data_ptr(), s.cuda_stream) == 0
    for _ in range(20):
        call(0)
    for r in range(int(os.environ.get("TUNE_ROUNDS", "6"))):
        for i in range(len(libs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                call(i)
            e1.record(s)
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 5)
    assert int(st.item()) == 0, "a blocks_hash chain timed out"
    for i, p in enumerate(libs):
        assert torch.equal(dig[i], dig[0]) and torch.equal(fh[i], fh[0]), p
        med = statistics.median(times[i])
        print(f"batch {nf} files {os.path.basename(p)}: median {med:.4f} ms min {min(times[i]):.4f} -> "
              f"{size / GiB / (med * 1e-3):.1f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
