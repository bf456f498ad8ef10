"""Debug probe (not a test): which waves of the CDC-like list's sorted launch
run at raised priority in a -DSF_DBG_PRIO build (lane 0 of each wave writes
its STATUS register and max_nch into its block's digest).
usage: python scripts/prio_dbg.py lib.so"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
L.sf_index_device_blocks.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
L.sf_test_table_order.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
total = 4 << 30
dev = torch.device("cuda:0")
data = device.splitmix_tensor(total, 0x5EED0000, dev)
rng = np.random.default_rng(7)
s = np.minimum(32768, np.maximum(1, rng.geometric(1 / 8192, size=total // 4096))).astype(np.int64)
c = np.cumsum(s)
n = int(np.searchsorted(c, total))
s = s[: n + 1]
s[-1] -= int(c[n] - total) if c[n] > total else 0
s = s[s > 0]
offs = np.concatenate([[0], np.cumsum(s)[:-1]]).astype(np.int64)
to, tz = torch.from_numpy(offs).to(dev), torch.from_numpy(s.astype(np.int32)).to(dev)
out = torch.zeros((offs.size, 20), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
assert L.sf_index_device_blocks(data.data_ptr(), total, to.data_ptr(), tz.data_ptr(), offs.size, out.data_ptr(), None, st) == 0
order = torch.empty(offs.size, dtype=torch.int32, device=dev)
assert L.sf_test_table_order(tz.data_ptr(), offs.size, order.data_ptr(), st) == 0
torch.cuda.synchronize()
o = order.cpu().numpy().view(np.uint32)
d = out.cpu().numpy().view(np.uint32).reshape(-1, 5)
nw = (offs.size + 63) // 64
first = o[np.arange(nw) * 64]
stat, nch = d[first, 0], d[first, 1]
prio = (stat >> 3) & 3
print("waves", nw, "prio counts", {int(p): int((prio == p).sum()) for p in np.unique(prio)})
for lo, hi in [(0, 100), (100, 200), (200, 300), (300, 344), (344, 400), (400, 514)]:
    m = (nch >= lo) & (nch < hi)
    print(f"max_nch [{lo},{hi}): waves {int(m.sum())}, prio>0: {int((prio[m] > 0).sum())}")
print("first 40 waves (order index, max_nch, prio):", [(int(w), int(nch[w]), int(prio[w])) for w in range(0, 40)])
print("status raw sample", [hex(int(x)) for x in stat[:8]])
