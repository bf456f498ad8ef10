"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read (16 B/lane loads and buffer_load ... lds alike), so it
is doubled; WRITE_SIZE is exact for streaming stores.  Averages over every
launch of the SHA-1 kernel in the pass.  The entry records the SHA-256 of the
library the passes ran, of its gfx950 code objects and of the headline
kernel's machine code (bench.py reports traffic only for the same kernel
code).  Only the full-shard launches count (the
largest grid of the pass).

usage: python scripts/pmc_traffic.py FETCH_CSV WRITE_CSV CONFIG_KEY SHARD_BYTES [OUT]
"""
import csv
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from syncfast_amd._lib import code_object_sha256, kernel_code_sha256  # noqa: E402

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "syncfast_amd", "lib", "libsyncfast_amd.so")


def avg(path, counter, match="sha1_fixed_kernel"):
    """Mean counter value over the SHA-1 kernel's launches of the full shard
    (the largest grid in the pass): the bench's clock-ramp and timed steps,
    not its smaller end-to-end stage launches."""
    rows = [r for r in csv.DictReader(open(path)) if match in r["Kernel_Name"] and r["Counter_Name"] == counter]
    grid = max(int(r["Grid_Size"]) for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == grid]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, key, shard = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    f, nf = avg(fetch_csv, "FETCH_SIZE")
    w, nw = avg(write_csv, "WRITE_SIZE")
    read_b = f * 1024 * 2
    write_b = w * 1024
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[key] = {"shard_bytes": shard, "hbm_bytes_per_launch": int(read_b + write_b),
                 "read_bytes": int(read_b), "write_bytes": int(write_b), "launches": [nf, nw],
                 "raw_kib": {"FETCH_SIZE": f, "WRITE_SIZE": w},
                 "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
                 "code_object_sha256": code_object_sha256(LIB),
                 "kernel_code_sha256": kernel_code_sha256(LIB),
                 "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
