"""CPU: pin the oracle against the reference's own KATs and hashlib vectors.

The oracle (oracle/sf_oracle.c) is the checker for every GPU parity test, so
it is itself checked first:
  * reference KAT, /root/reference/src/index.rs:747-793 (3 blocks + blocks_hash)
  * SHA1("test"), /root/reference/src/lib.rs:184-195
  * hashlib golden vectors in tests/golden/golden.json
"""
import hashlib

import numpy as np
import pytest

import oracle


def test_reference_kat_blocks(golden):
    kat = oracle.kat_input()
    g = golden["reference_kat"]
    assert len(kat) == g["len"] == 44893
    offs = [b["offset"] for b in g["blocks"]]
    sizes = [b["size"] for b in g["blocks"]]
    # blocks tile the file; the middle one is the forced MAX_BLOCK_SIZE cut
    # (src/index.rs:786)
    assert offs[0] == 0 and offs[-1] + sizes[-1] == len(kat)
    assert offs[2] - offs[1] == 1 << 15
    dig = oracle.index_blocks(kat, offs, sizes)
    assert [bytes(d).hex() for d in dig] == [b["sha1"] for b in g["blocks"]]
    assert oracle.blocks_hash(dig).hex() == g["blocks_hash"]
    assert oracle.py_blocks_hash([bytes(d) for d in dig]).hex() == g["blocks_hash"]


def test_reference_sha1_strings(golden):
    for s, hx in golden["sha1_strings"].items():
        assert oracle.sha1(s.encode()).hex() == hx
        assert hashlib.sha1(s.encode()).hexdigest() == hx


def test_splitmix_generator(golden):
    c = oracle.splitmix_bytes(16, 0x5EED0000)
    assert c.tobytes().hex() == golden["splitmix_seed_5EED0000_first16"]
    for start, n in [(0, 1000), (3, 77), (13, 8), (1 << 20, 33)]:
        assert oracle.splitmix_bytes(n, 1234, start).tobytes() == oracle.py_splitmix_bytes(n, 1234, start)


def test_fixed_golden(golden):
    assert len(golden["fixed"]) > 40
    for case in golden["fixed"]:
        data = oracle.splitmix_bytes(case["len"], case["seed"])
        offs, sizes, dig = oracle.index_fixed(data, case["block_size"])
        assert [bytes(d).hex() for d in dig] == case["digests"], case["len"]
        assert oracle.blocks_hash(dig).hex() == case["blocks_hash"]
        n = len(case["digests"])
        assert list(offs) == [i * case["block_size"] for i in range(n)]
        assert int(sizes.sum()) == case["len"]


def test_ragged_golden(golden):
    for case in golden["ragged"]:
        data = oracle.splitmix_bytes(case["len"], case["seed"])
        dig = oracle.index_blocks(data, case["offsets"], case["sizes"])
        assert [bytes(d).hex() for d in dig] == case["digests"]
        assert oracle.blocks_hash(dig).hex() == case["blocks_hash"]


def test_empty_input_has_no_blocks():
    offs, sizes, dig = oracle.index_fixed(b"", 4096)
    assert dig.shape == (0, 20)
    assert oracle.blocks_hash(dig).hex() == "da39a3ee5e6b4b0d3255bfef95601890afd80709"


@pytest.mark.parametrize("bs", [64, 4096, 1000])
def test_mt_matches_single(bs):
    data = oracle.splitmix_bytes(bs * 37 + 11, 99)
    _, _, d1 = oracle.index_fixed(data, bs)
    d2 = oracle.index_fixed_mt(data, bs, 4)
    assert np.array_equal(d1, d2)


def test_c_matches_python_random():
    rng = np.random.default_rng(7)
    data = oracle.splitmix_bytes(300_000, 42).tobytes()
    for _ in range(20):
        bs = int(rng.integers(1, 70_000))
        _, _, d = oracle.index_fixed(data, bs)
        _, _, want = oracle.py_index_fixed(data, bs)
        assert [bytes(x) for x in d] == want


def test_adler_oracle_matches_zlib():
    # the opt-in weak sum's checker (not a reference path: SURVEY.md 8a row a8)
    import zlib
    rng = np.random.default_rng(11)
    data = oracle.splitmix_bytes(300_000, 77).tobytes()
    assert oracle.adler32(b"") == zlib.adler32(b"") == 1
    for n in [1, 63, 64, 65, 4095, 4096, 4097, 5553, 300_000]:
        assert oracle.adler32(data[:n]) == zlib.adler32(data[:n]), n
    worst = b"\xff" * (1 << 20)  # largest sums: overflow guard
    assert oracle.adler32(worst) == zlib.adler32(worst)
    for _ in range(5):
        bs = int(rng.integers(1, 70_000))
        want = [zlib.adler32(data[i:i + bs]) for i in range(0, len(data), bs)]
        assert oracle.adler_fixed(data, bs).tolist() == want
    offs, sizes = [0, 17, 1000, 299_990], [0, 5000, 64, 10]
    assert oracle.adler_blocks(data, offs, sizes).tolist() == [zlib.adler32(data[o:o + s]) for o, s in zip(offs, sizes)]


def test_zpaq_standin_is_the_surveys_restatement():
    """The configs[0] stand-in chunker (examples/zpaq_standin.h, timed by
    bench.py's config1 block) is zpaq's fragmenter in the survey's form: on
    the reference KAT input it cuts at 5,908 / 6,547 / 14,382 (SURVEY.md
    Appendix A, "Restatement that failed") -- NOT the crate's 11,579 /
    44,347 (src/index.rs:765-786), which is why it is only a cost stand-in.
    Its single pass (each block SHA-1'd as it is cut) equals hashlib per
    block, scalar and SHA-NI."""
    import hashlib
    kat = oracle.kat_input()
    sizes = oracle.zpaq_standin_sizes(kat)
    assert list(np.cumsum(sizes)[:3]) == [5908, 6547, 14382] and int(sizes.sum()) == len(kat)
    data = oracle.splitmix_bytes(3 << 20, 0x5EED0000)
    sizes = oracle.zpaq_standin_sizes(data)
    assert sizes.max() <= 32768 and sizes.min() >= 1 and int(sizes.sum()) == data.size
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    want = np.stack([np.frombuffer(hashlib.sha1(data[o:o + s].tobytes()).digest(), np.uint8)
                     for o, s in zip(offs, sizes.astype(np.int64))])
    for shani in (False, True):
        assert np.array_equal(oracle.zpaq_standin_index(data, shani), want)
