"""How long it takes to get a page-locked staging buffer, and how fast H2D
runs from it: the one-time cost a fresh process pays before its first
pipelined stage (a one-shot `index` run pays it every time).

  A hipHostMalloc
  B anonymous mmap (4 KiB pages), touched, hipHostRegister
  C anonymous mmap, MADV_HUGEPAGE, touched, hipHostRegister

Each for 64 and 256 MiB, then 4 H2D copies of the whole buffer.

usage: python scripts/pin_alloc_probe.py"""
import ctypes
import mmap
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
H2D = 1


def ms(t0):
    return (time.perf_counter() - t0) * 1e3


def h2d_rate(ptr, n, dev):
    s = torch.cuda.current_stream()
    assert hip.hipMemcpyAsync(dev.data_ptr(), ptr, n, H2D, ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        assert hip.hipMemcpyAsync(dev.data_ptr(), ptr, n, H2D, ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    return 4 * n / (time.perf_counter() - t0) / 1e9


def main():
    torch.zeros(1, device="cuda")
    dev = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    for rep in range(2):
        for mib in (64, 256):
            n = mib << 20
            p = ctypes.c_void_p()
            t0 = time.perf_counter()
            assert hip.hipHostMalloc(ctypes.byref(p), n, 0) == 0
            ta = ms(t0)
            ra = h2d_rate(p.value, n, dev)
            t0 = time.perf_counter()
            hip.hipHostFree(p)
            fa = ms(t0)
            res = [f"hipHostMalloc {ta:.1f} ms (free {fa:.1f}), H2D {ra:.1f} GB/s"]
            for huge in (False, True):
                t0 = time.perf_counter()
                m = mmap.mmap(-1, n + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
                base = ctypes.addressof(ctypes.c_char.from_buffer(m))
                off = (-base) % (2 << 20)  # 2 MiB aligned start
                if huge:
                    m.madvise(mmap.MADV_HUGEPAGE, off, n)
                ctypes.memset(base + off, 1, n)
                tt = ms(t0)
                t0 = time.perf_counter()
                assert hip.hipHostRegister(base + off, n, 0) == 0
                tr = ms(t0)
                r = h2d_rate(base + off, n, dev)
                t0 = time.perf_counter()
                hip.hipHostUnregister(ctypes.c_void_p(base + off))
                fu = ms(t0)
                res.append(f"mmap{'+THP' if huge else ''} touch {tt:.1f} ms + register {tr:.1f} ms "
                           f"(unregister {fu:.1f}), H2D {r:.1f} GB/s")
                del base
                m.close()
            print(f"rep {rep} {mib} MiB: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
