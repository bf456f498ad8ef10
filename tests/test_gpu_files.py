"""GPU: sf_index_files, the many-file pipeline behind Index.index_path
(src/index.rs:685-715 calling index_file, src/index.rs:610-659, per file).

Every file's rows and blocks_hash are compared with the oracle on the same
bytes, through each route the pipeline takes:
- mixed sizes packed into ragged stages (table kernel + per-file chains);
- files larger than a stage (one-file pipeline);
- equal-size block-aligned files (staged fused kernel);
- a block size that is not a multiple of 16 (per-lane loads).
"""
import numpy as np
import pytest

import oracle
from syncfast_amd import host

SIZES = [0, 1, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 3 * 4096, 100_000, 2_000_000, 5, 0, 65536 * 3 + 7]


def _write(tmp_path, sizes, seed0):
    paths = []
    for i, n in enumerate(sizes):
        p = tmp_path / f"f{i:04d}"
        p.write_bytes(oracle.splitmix_bytes(n, seed0 + i).tobytes())
        paths.append(p)
    return paths


def _check(paths, sizes, seed0, bs, rows, first, fh):
    assert first.tolist()[-1] == rows.shape[0]
    for i, n in enumerate(sizes):
        data = oracle.splitmix_bytes(n, seed0 + i)
        offs, szs, want = oracle.index_fixed(data, bs)
        r = rows[int(first[i]):int(first[i + 1])]
        assert r["offset"].tolist() == [int(o) for o in offs], (i, n)
        assert r["size"].tolist() == [int(s) for s in szs], (i, n)
        assert [bytes(x) for x in r["sha1"]] == [bytes(w) for w in want], (i, n, bs)
        assert bytes(fh[i]) == oracle.blocks_hash(want), (i, n, bs)


@pytest.mark.gpu
@pytest.mark.parametrize("stage", [0, 50_000, 1 << 20])
@pytest.mark.parametrize("bs", [4096, 64, 1000])
def test_index_files_mixed_sizes(gpu, tmp_path, stage, bs):
    paths = _write(tmp_path, SIZES, 900)
    rows, first, fh = host.index_files(paths, bs, stage_bytes=stage)
    _check(paths, SIZES, 900, bs, rows, first, fh)


@pytest.mark.gpu
@pytest.mark.parametrize("stage", [8 << 20, 4 << 20, 3 << 20])
def test_index_files_equal_files_staged(gpu, tmp_path, stage):
    """8 x 1 MiB files at 4 KiB: 256 blocks per file, the staged kernel's
    shape (one stage of 8 files, or 2 stages of 4, or stages of 3+3+2)."""
    sizes = [1 << 20] * 8
    paths = _write(tmp_path, sizes, 1300)
    rows, first, fh = host.index_files(paths, 4096, stage_bytes=stage)
    _check(paths, sizes, 1300, 4096, rows, first, fh)


@pytest.mark.gpu
def test_index_files_many_small(gpu, tmp_path):
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(0, 20_000, 600)]
    paths = _write(tmp_path, sizes, 5000)
    rows, first, fh = host.index_files(paths, 4096, stage_bytes=1 << 20)
    _check(paths, sizes, 5000, 4096, rows, first, fh)


@pytest.mark.gpu
def test_index_files_matches_one_file_path(gpu, tmp_path):
    paths = _write(tmp_path, [300_000, 12_345], 77)
    rows, first, fh = host.index_files(paths, 4096)
    for k, p in enumerate(paths):
        r1, bh1 = host.index_file(p, 4096)
        assert rows[int(first[k]):int(first[k + 1])].tobytes() == r1.tobytes()
        assert bytes(fh[k]) == bh1


@pytest.mark.gpu
@pytest.mark.parametrize("stage", [0, 160 << 20])
def test_index_files_large_files_pread_only(gpu, tmp_path, stage):
    """Files of 64 MiB and more in the page cache: read with pread like every
    other file (never mapped and page-locked: DESIGN.md 6), mixed in one stage
    (ragged route) and as equal files (staged route).  Stages holding 64 MiB
    files take blocks_hash on the host (long runs).  Nothing is page-locked."""
    from syncfast_amd import _lib
    locked = _lib.get_stat("pages_locked")
    sizes = [(64 << 20) + 4096, 100_000, (64 << 20) + 13, 0, 5 << 20, 77]
    paths = _write(tmp_path, sizes, 2100)
    rows, first, fh = host.index_files(paths, 4096, stage_bytes=stage)
    _check(paths, sizes, 2100, 4096, rows, first, fh)
    eq = [64 << 20] * 2
    paths = _write(tmp_path, eq, 2200)
    rows, first, fh = host.index_files(paths, 4096, stage_bytes=stage)
    _check(paths, eq, 2200, 4096, rows, first, fh)
    assert _lib.get_stat("pages_locked") == locked


@pytest.mark.gpu
def test_index_files_reports_the_failing_file(gpu, tmp_path):
    # a missing file and a directory in the list: SF_EIO naming the first
    # failing file (the error the per-file loop would raise at File::open)
    from syncfast_amd._lib import SfError
    paths = _write(tmp_path, [100, 5000, 7], 3100)
    missing = tmp_path / "gone"
    with pytest.raises(SfError) as e:
        host.index_files(paths[:2] + [missing] + paths[2:], 4096)
    assert e.value.code == -5 and str(missing) in str(e.value)
    with pytest.raises(SfError) as e:
        host.index_files([paths[0], tmp_path, paths[1]], 4096)
    assert e.value.code == -5 and str(tmp_path) in str(e.value)
    rows, first, fh = host.index_files(paths, 4096)  # and the call after an error is clean
    _check(paths, [100, 5000, 7], 3100, 4096, rows, first, fh)
