"""CPU: bench.py's launcher contract.

`python bench.py --gpus N` without torchrun must start N ranks itself (a
child torch.distributed.run, no exec) and never silently report 1 GPU; a
--gpus / WORLD_SIZE mismatch must fail.  --check-launch runs the launch and
the process-group check only (gloo, no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(extra)
    return env


def _last_json(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_self_launch_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--check-launch"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert {k: line[k] for k in ("launch_check", "n_gpus", "ranks_seen")} == \
        {"launch_check": True, "n_gpus": 2, "ranks_seen": 2}
    assert "launching 2 ranks" in r.stderr


def test_self_launch_three_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dist-backend", "gloo", "--check-launch"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert _last_json(r.stdout)["n_gpus"] == 3


def test_multi_block_three_ranks():
    """An N > 1 line carries a `multi` block (per-rank kernel time, gather
    waits as receiving rank and as sender, rank-0-reported world size).  The
    kernel needs a GPU, so on CPU the launch check builds the same block from
    stand-in per-rank numbers (rank r reports r + 1 ms) over gloo, through
    the same code (bench.multi_block) the GPU run uses."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dist-backend", "gloo", "--shard-gib", "0.01",
                        "--steps", "6", "--check-launch"], capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    m = _last_json(r.stdout)["multi"]
    assert m["world"] == 3 and m["backend"] == "gloo"
    assert m["kernel_ms"] == {"max": 3.0, "min": 1.0, "per_rank": [1.0, 2.0, 3.0]}
    assert len(m["gather_wait_ms_as_root"]) == len(m["gather_wait_ms_as_sender"]) == 3
    assert m["steps_as_root"] == [2, 2, 2]


def test_config4_multi_line_names_its_workload():
    """The driver's 8-GPU config-4 run must not mislabel itself: an N > 1
    config-4 line carries the `multi` block and config 4's workload (one 256
    GiB file at 8 GPUs, 32 GiB shard per GPU; here --shard-gib shrinks it),
    with the shard layout and the gather in `parallelism`."""
    r = subprocess.run([sys.executable, BENCH, "--config", "4", "--gpus", "3", "--dist-backend", "gloo",
                        "--shard-gib", "0.01", "--check-launch"], capture_output=True, text=True, timeout=240,
                       env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 3 and line["multi"]["world"] == 3
    c = line["config"]
    assert "one 256 GiB synthetic file" in c["workload"] and "configs[3]" in c["workload"]
    assert c["block_size"] == 4096 and c["files"] == 1
    assert c["total_bytes"] == 3 * c["bytes_per_gpu"] and c["blocks"] == c["total_bytes"] // 4096
    assert c["parallelism"] == "shard3+gloo_gather(pipelined, root rotating)"


def test_dist_timeout_is_passed():
    # a stuck collective must fail the run, not hang it: the process group
    # is created with --dist-timeout (default 300 s)
    src = open(BENCH).read()
    assert src.count("timeout=tmo") == 2 and '"--dist-timeout", type=float, default=300.0' in src


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--check-launch"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_config1_probe_reports_toolchain():
    sys.path.insert(0, ROOT)
    import shutil

    import bench
    c1 = bench.config1_probe()
    have = shutil.which("cargo") and shutil.which("rustc")
    assert c1["status"] == ("runnable (not timed here)" if have else "reference CPU path not runnable")
    assert set(c1["probe"]) == {"cargo", "rustc", "~/.cargo"}


def _plan(*args):
    r = subprocess.run([sys.executable, BENCH, "--check-plan"] + list(args), capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    return _last_json(r.stdout)


def test_library_plan_defaults_to_config4_at_n_gt_1():
    """--gpus N > 1 runs ONE process over N devices through the C-ABI
    (sf_index_device_multi_ex) on configs[3]'s 32 GiB shard per GPU; the plan
    (no GPU needed) shards one logical file of N x 32 GiB, block-aligned,
    with the rows of shard r at its place in the root's table, and rotates the
    gather's root so the last timed step's table is device 0's."""
    for n in (2, 8):
        p = _plan("--gpus", str(n))
        assert p["path"] == "library" and p["n_devices"] == n and p["config"] == 4
        assert "configs[3]" in p["workload"] and p["bytes_per_gpu"] == 32 << 30 and p["block_size"] == 4096
        assert p["total_bytes"] == n * (32 << 30) and p["blocks"] == p["total_bytes"] // 4096
        pos = 0
        for r, sh in enumerate(p["shards"]):
            assert sh["device"] == r and sh["start"] == pos and sh["first_row"] == pos // 4096
            assert sh["rows"] == (sh["bytes"] + 4095) // 4096
            pos += sh["bytes"]
        assert pos == p["total_bytes"]
        roots = p["roots_timed"]
        assert len(roots) == 20 and roots[-1] == 0
        assert max(roots.count(r) for r in range(n)) - min(roots.count(r) for r in range(n)) <= 1
        assert p["roots_warmup"] == list(range(n))


def test_library_plan_uneven_shards_and_one_device():
    # a shard size that is not a block multiple at an odd device count, and
    # the one-device library path (the GPU test runs it with the self-gather)
    p = _plan("--gpus", "3", "--shard-gib", "0.01", "--steps", "7")
    assert sum(sh["bytes"] for sh in p["shards"]) == p["total_bytes"]
    assert all(sh["start"] % 4096 == 0 for sh in p["shards"])
    assert p["roots_timed"][-1] == 0 and len(p["roots_timed"]) == 7
    one = _plan("--gpus", "1", "--multi-path", "library")
    assert one["n_devices"] == 1 and one["config"] == 2 and one["shards"][0]["bytes"] == 8 << 30


def test_multi_path_resolution():
    sys.path.insert(0, ROOT)
    import argparse

    import bench

    def ns(**kw):
        base = dict(gpus=1, config=None, multi_path="auto", check_launch=False, dist_backend="nccl")
        base.update(kw)
        return bench.resolve_args(argparse.Namespace(**base))

    assert (ns().config, ns().multi_path) == (2, "torch")  # the single-GPU line is unchanged
    assert (ns(gpus=8).config, ns(gpus=8).multi_path) == (4, "library")
    assert ns(gpus=8, check_launch=True).multi_path == "torch"
    assert ns(gpus=2, dist_backend="gloo").multi_path == "torch"
    assert ns(gpus=8, multi_path="torch").multi_path == "torch"
    assert ns(gpus=8, config=2).config == 2


def test_torchrun_library_failure_falls_back_on_every_rank():
    """The driver's torchrun with the library path: rank 0 drives every device
    in one process and the other ranks wait.  If rank 0's path fails for any
    reason -- here: no GPU, so fewer devices than --gpus, as when a launcher
    shows each rank only its own GPU -- every rank must go on to the
    per-process form (here its launch rehearsal) and the line must say why,
    never leave the other ranks waiting."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", f"--master-port={port}", BENCH, "--gpus", "2",
                        "--multi-path", "library", "--check-launch", "--dist-timeout", "60"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["launch_check"] and line["n_gpus"] == 2 and line["ranks_seen"] == 2
    assert "RuntimeError" in line["multi_fallback"] and "device(s) visible" in line["multi_fallback"]
    assert "library multi-GPU path failed" in r.stderr
