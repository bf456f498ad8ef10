#!/usr/bin/env python3
"""Round 6: configs[0]'s folder (one 64 MiB file, page cache) indexed by a
FRESH process each time -- the way the reference's CLI runs (`syncfast index`,
src/main.rs:122) -- so the HIP runtime's start-up and the library's first
allocations are counted: the C consumer (`examples/build/sf_index -Z -p 16`,
no Python; its -T line gives the one sf_index_fd_cut call's own time), the
same binary finding the device and stopping (the runtime's start-up), and
`Index.index_path` from a fresh interpreter, 3 runs each, wall time of the
whole process.  One JSON line per run."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import oracle
    d = tempfile.mkdtemp(prefix="sf_cold_")
    folder = os.path.join(d, "folder")
    os.mkdir(folder)
    p = os.path.join(folder, "file64")
    oracle.splitmix_bytes(64 << 20, 0x5EED0000).tofile(p)
    with open(p, "rb") as f:  # into the page cache
        while f.read(1 << 24):
            pass
    exe = os.path.join(ROOT, "examples", "build", "sf_index")
    py = ("import sys, time; t0 = time.perf_counter(); sys.path.insert(0, %r); "
          "from syncfast_amd.index import Index, NativeChunker; import ctypes; "
          "Z = ctypes.CDLL(%r); Z.sf_zpaq_standin_ops.restype = ctypes.c_void_p; "
          "Z.sf_zpaq_standin_ops.argtypes = [ctypes.c_uint, ctypes.c_uint32]; "
          "ix = Index.open(%r, chunker=NativeChunker(Z.sf_zpaq_standin_ops(13, 32768), 16)); "
          "t1 = time.perf_counter(); ix.index_path(%r); ix.commit(); t2 = time.perf_counter(); "
          "print(round((t1 - t0) * 1e3, 1), round((t2 - t1) * 1e3, 1))"
          % (ROOT, os.path.join(ROOT, "examples", "build", "libzpaq_standin.so"), os.path.join(d, "idx.db"), folder))
    for r in range(3):  # the HIP runtime's start-up alone: a process that only finds the device
        t0 = time.perf_counter()
        out = subprocess.run([exe, os.path.join(d, "missing")], capture_output=True, text=True, timeout=120)
        print(json.dumps({"run": r, "route": "C consumer, device found, nothing indexed (a missing path)",
                          "process_ms": round((time.perf_counter() - t0) * 1e3, 1)}), flush=True)
    for r in range(3):
        t0 = time.perf_counter()
        out = subprocess.run([exe, "-Z", "-p", "16", "-T", p], capture_output=True, text=True, timeout=120,
                             env=dict(os.environ, SF_TRACE="1"))
        t = time.perf_counter() - t0
        call = [json.loads(ln) for ln in out.stderr.splitlines() if ln.startswith("{")]
        print(json.dumps({"run": r, "route": "C consumer -Z -p 16 (sf_index_fd_cut), fresh process", "rc": out.returncode,
                          "process_ms": round(t * 1e3, 1), "GB/s_of_process": round((64 << 20) / t / 1e9, 3),
                          "first_call_ms": round(call[0]["hash_s"] * 1e3, 2) if call else None,
                          "trace": [ln for ln in out.stderr.splitlines() if "trace" in ln]}), flush=True)
    for r in range(3):
        try:
            os.unlink(os.path.join(d, "idx.db"))
        except OSError:
            pass
        t0 = time.perf_counter()
        out = subprocess.run([sys.executable, "-c", py], capture_output=True, text=True, timeout=300)
        t = time.perf_counter() - t0
        parts = out.stdout.split()
        print(json.dumps({"run": r, "route": "Index.index_path(folder), fresh interpreter", "rc": out.returncode,
                          "process_ms": round(t * 1e3, 1), "import_and_open_ms": float(parts[0]) if parts else None,
                          "index_path_ms": float(parts[1]) if len(parts) > 1 else None,
                          "stderr": out.stderr[-300:] if out.returncode else ""}), flush=True)


if __name__ == "__main__":
    main()
