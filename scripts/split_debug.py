"""Which blocks of one wave a library build hashes wrongly (probe, not a
test): four 64-block explicit lists (16-B aligned, equal line offsets,
random byte offsets) through sf_index_device_blocks of the library given as
argv[1], each digest against hashlib; prints the bad blocks with off & 3,
the line offset and the size.  Used to find the divergent-shuffle bug of the
rejected last-touch layout (profiles/r03/cdc_prio/split_debug_*.log).

usage: python scripts/split_debug.py path/to/libsyncfast_amd.so
"""
import ctypes, os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from syncfast_amd import device
import hashlib
dev = torch.device("cuda:0")
def bind(p):
    L = ctypes.CDLL(os.path.abspath(p)); f = L.sf_index_device_blocks
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return f
f = bind(sys.argv[1])
rng = np.random.default_rng(3)
n = 1 << 20
data = device.splitmix_tensor(n, 99, dev)
hb = data.cpu().numpy().tobytes()
for trial in range(4):
    m = 64
    sizes = rng.integers(200, 3000, m).astype(np.int64)
    offs = np.sort(rng.integers(0, n - 4000, m)).astype(np.int64)
    if trial == 0: offs = offs & ~15  # aligned -> other path; make some unaligned
    if trial == 1: offs[:] = offs[0] + np.arange(m) * 4096 + 4  # all q equal
    to = torch.from_numpy(offs).to(dev); tz = torch.from_numpy(sizes.astype(np.int32)).to(dev)
    out = torch.zeros((m, 20), dtype=torch.uint8, device=dev)
    rc = f(data.data_ptr(), n, to.data_ptr(), tz.data_ptr(), m, out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    bad = [i for i in range(m) if bytes(o[i]) != hashlib.sha1(hb[offs[i]:offs[i]+sizes[i]]).digest()]
    q = (offs + data.data_ptr()) & 127
    print("trial", trial, "rc", rc, "bad", len(bad), [(i, int(offs[i] & 3), int(q[i]), int(sizes[i])) for i in bad[:12]], flush=True)
