"""bench.py's launch contract without a device: ``--gpus N`` outside torchrun spawns N ranks
itself (each seeing WORLD_SIZE = N), and a launcher/flag mismatch is refused instead of timing
the wrong number of GPUs.  CWT_BENCH_DRYRUN stops each rank right after the process group is up
(gloo here, no GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(CWT_BENCH_DRYRUN="1", **(extra_env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=300)


def test_bench_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["ranks_seen"] == 2 for d in lines)


def test_bench_refuses_world_mismatch():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "disagrees" in (r.stderr + r.stdout)


def test_bench_gpus1_single_process():
    r = _run(["--gpus", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines == [{"rank": 0, "world": 1, "ranks_seen": 1}]
