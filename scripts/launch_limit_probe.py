"""What one HIP launch does past 2^32 work-items, and that the split launch
does not: 1-B blocks over 4 GiB + 77 B (2^32 + 77 blocks, one lane each),
hashed once with the launcher's split (default) and once with it disabled
(SF_TEST_LAUNCH_MAX_BLOCKS = 2^40, one launch), each in its own process; every
digest is compared with SHA-1 of its byte (profiles/r02/split/).

usage: python scripts/launch_limit_probe.py           (parent)
       python scripts/launch_limit_probe.py child     (one measurement)"""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    import numpy as np
    import torch
    from syncfast_amd import device
    n = (1 << 32) + 77
    data = device.splitmix_tensor(n, 0x5EED0000, device="cuda:0")
    dig = device.index_device(data, 1)
    torch.cuda.synchronize()
    table = torch.from_numpy(np.stack([np.frombuffer(hashlib.sha1(bytes([b])).digest(), np.uint8)
                                       for b in range(256)])).cuda()
    bad, first_bad, step = 0, None, 1 << 28
    for a in range(0, n, step):
        b = min(n, a + step)
        ok = (dig[a:b] == table[data[a:b].long()]).all(dim=1)
        nbad = int((~ok).sum())
        if nbad and first_bad is None:
            first_bad = a + int((~ok).nonzero()[0])
        bad += nbad
    print(f"SF_TEST_LAUNCH_MAX_BLOCKS={os.environ.get('SF_TEST_LAUNCH_MAX_BLOCKS', 'default')}: {n} blocks, "
          f"{bad} wrong digests" + (f", first at block {first_bad}" if bad else ""), flush=True)


def main():
    for knob in (None, str(1 << 40)):
        env = dict(os.environ)
        if knob:
            env["SF_TEST_LAUNCH_MAX_BLOCKS"] = knob
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
        print((r.stdout.strip() or "<no output>") + ("" if r.returncode == 0 else f" rc={r.returncode} {r.stderr[-400:]}"),
              flush=True)


if __name__ == "__main__":
    child() if sys.argv[1:] == ["child"] else main()
