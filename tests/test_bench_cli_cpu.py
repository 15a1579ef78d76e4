"""bench.py's rank contract, on the CPU (no GPU is touched: every case is refused before that).

VERDICT r4 item 1: `--gpus N` must be what the JSON line reports.  A launcher that started a different
number of ranks is refused, and so is `--gpus N > 1` over RCCL on a machine with fewer than N GPUs
(this container has none), instead of silently measuring one GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env_over):
    env = dict(os.environ, **env_over)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        if k not in env_over:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=120, cwd=ROOT, env=env)


def test_world_size_mismatch_is_refused():
    r = _bench(["--gpus", "4", "--no-cpu-baseline"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and not r.stdout.strip()
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr


def test_world_size_without_gpus_flag_is_refused():
    r = _bench(["--no-cpu-baseline"], WORLD_SIZE="8", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=8" in r.stderr


def test_rccl_launch_needs_a_gpu_per_rank():
    r = _bench(["--gpus", "2"])
    assert r.returncode == 2 and not r.stdout.strip()
    assert "needs 2 visible GPUs" in r.stderr


def test_gpus_must_be_positive():
    r = _bench(["--gpus", "0", "--no-cpu-baseline"])
    assert r.returncode == 2 and "--gpus must be >= 1" in r.stderr
