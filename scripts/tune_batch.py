"""A/B of the staged many-file batch (SF_TEST_STAGES) in one process: 1024 x 8 MiB files.
SF_STAGED_EXP is read per call by -DSF_TUNING builds only (SF_LIB=... a variant)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402
from syncfast_amd._lib import set_knob  # noqa: E402

GiB = 1 << 30
nf, flen, bs = 1024, 8 << 20, 4096
data = device.splitmix_tensor(nf * flen, 0x5EED0000)
files = [(i * flen, flen) for i in range(nf)]
dig = torch.empty((nf * flen // bs, 20), dtype=torch.uint8, device="cuda")
fh = torch.empty((nf, 20), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
for _ in range(30):
    device.index_device(data, bs, out=dig)
res = {}
ref = None
for r in range(5):
    for st in ["1", "16", "16e1", "16e2"]:
        set_knob("SF_TEST_STAGES", int(st[:2] if "e" in st else st))
        os.environ["SF_STAGED_EXP"] = st[3:] if "e" in st else "0"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            device.index_device_batch(data, files, bs, out=dig, hashes_out=fh)
        e1.record(s)
        torch.cuda.synchronize()
        res.setdefault(st, []).append(e0.elapsed_time(e1) / 5)
        if ref is None:
            ref = fh.clone()
        if "e" not in st:
            assert torch.equal(fh, ref)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(5):
    device.index_device(data, bs, out=dig)
e1.record(s)
torch.cuda.synchronize()
print("blocks only (no blocks_hash): %.4f ms" % (e0.elapsed_time(e1) / 5))
for st, ts in res.items():
    print(f"SF_TEST_STAGES={st}: median {statistics.median(ts):.4f} ms -> {nf * flen / GiB / (statistics.median(ts) * 1e-3):.1f} GiB/s")
