"""Generates tests/golden/golden.json (committed).

Inputs are described by recipes (the reference KAT text, or splitmix64
streams), expected outputs come from ``hashlib.sha1`` -- independent of the C
oracle and of the HIP product, so the JSON pins both.

The reference KAT expectations are data transcribed from the reference's own
test, /root/reference/src/index.rs:765-792 and src/lib.rs:184-195; the script
asserts hashlib reproduces them before writing anything.

Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import kat_input, py_splitmix_bytes  # noqa: E402  (pure-Python parts only)

# src/index.rs:765-792 -- (offset, size, sha1) per block + blocks_hash
REF_KAT_BLOCKS = [
    (0, 11579, "fb5ef7ebadd82c8085c5ff63823622bae0e263f6"),
    (11579, 32768, "570d8b30fcfd585e4127b561f5ecd376ff4d0101"),
    (44347, 546, "b9a8c2641af2cf8fd8f36a2456a3eaa95c029127"),
]
REF_KAT_BLOCKS_HASH = "84c25d78edcdb67631639c43604cf0149564f044"
# src/lib.rs:184-195
REF_SHA1_TEST = "a94a8fe5ccb19ba61c4c0873d391e987982fbbd3"


def blocks_hash(hexes):
    h = hashlib.sha1()
    for x in hexes:
        h.update(bytes.fromhex(x))
    return h.hexdigest()


def fixed_case(seed, length, bs):
    data = py_splitmix_bytes(length, seed)
    n = (length + bs - 1) // bs
    digs = [hashlib.sha1(data[i * bs:(i + 1) * bs]).hexdigest() for i in range(n)]
    return {"seed": seed, "len": length, "block_size": bs, "digests": digs,
            "blocks_hash": blocks_hash(digs)}


def ragged_case(seed, sizes):
    length = sum(sizes)
    data = py_splitmix_bytes(length, seed)
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += s
    digs = [hashlib.sha1(data[a:a + s]).hexdigest() for a, s in zip(offs, sizes)]
    return {"seed": seed, "len": length, "offsets": offs, "sizes": sizes, "digests": digs,
            "blocks_hash": blocks_hash(digs)}


def main():
    kat = kat_input()
    assert len(kat) == 44893
    for off, size, hx in REF_KAT_BLOCKS:
        assert hashlib.sha1(kat[off:off + size]).hexdigest() == hx
    assert blocks_hash([h for _, _, h in REF_KAT_BLOCKS]) == REF_KAT_BLOCKS_HASH
    assert hashlib.sha1(b"test").hexdigest() == REF_SHA1_TEST

    # splitmix64 stream pin (first 16 bytes of seed 0x5EED0000)
    sm = py_splitmix_bytes(16, 0x5EED0000).hex()

    fixed = []
    # SHA-1 padding edges: len % 64 in {0,1,55,56,63}; tails at B-1, B, B+1
    for bs in (64, 100, 4096, 65536):
        for length in sorted({0, 1, 55, 56, 63, 64, 65, 119, 120, bs - 1, bs, bs + 1,
                              3 * bs + 55, 3 * bs + 56, 5 * bs}):
            if length < 0 or length > 400_000:
                continue
            fixed.append(fixed_case(0x5EED0000 + length, length, bs))
    # more than one wave of blocks (64 lanes) with a ragged tail
    fixed.append(fixed_case(0x5EED0001, 131 * 4096 + 1234, 4096))

    rng = random.Random(1234)
    ragged = []
    for k in range(4):
        n = [3, 64, 65, 130][k]
        sizes = [rng.choice([0, 1, 55, 56, 63, 64, 65, rng.randrange(1, 40000)]) for _ in range(n)]
        ragged.append(ragged_case(0x5EED1000 + k, sizes))

    out = {
        "_generated_by": "tests/golden/make_golden.py (hashlib)",
        "reference_kat": {
            "source": "/root/reference/src/index.rs:747-793",
            "input": "b''.join(b'Line %d\\n' % (i+1) for i in range(2000)) + b'Test content\\n'*2000",
            "len": len(kat),
            "blocks": [{"offset": o, "size": s, "sha1": h} for o, s, h in REF_KAT_BLOCKS],
            "blocks_hash": REF_KAT_BLOCKS_HASH,
        },
        "sha1_strings": {"test": REF_SHA1_TEST, "": hashlib.sha1(b"").hexdigest(),
                         "abc": hashlib.sha1(b"abc").hexdigest()},
        "splitmix_seed_5EED0000_first16": sm,
        "fixed": fixed,
        "ragged": ragged,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", len(fixed), "fixed and", len(ragged), "ragged cases")


if __name__ == "__main__":
    main()
