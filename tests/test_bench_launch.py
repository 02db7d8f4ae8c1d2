"""bench.py launch contract: ``python bench.py --gpus N`` with no launcher
around it starts N ranks itself and reports n_gpus = N; a --gpus / WORLD_SIZE mismatch is fatal.
Runs the CPU mode (FDX_BENCH_DEVICE=cpu: same code path on CPU tensors over gloo)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["FDX_BENCH_DEVICE"] = "cpu"
    env.update(kw)
    return env


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_self_launch_two_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--rows-per-gpu", "20000"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 2 * 16000
    assert "self-launch" in r.stderr


def test_single_rank_default():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--rows-per-gpu", "20000"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"


def test_world_size_mismatch_is_fatal():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "FATAL" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
