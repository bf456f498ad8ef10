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
