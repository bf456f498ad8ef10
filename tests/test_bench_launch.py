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
    assert line == {"launch_check": True, "n_gpus": 2, "ranks_seen": 2}
    assert "launching 2 ranks" in r.stderr


def test_self_launch_three_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dist-backend", "gloo", "--check-launch"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert _last_json(r.stdout)["n_gpus"] == 3


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
