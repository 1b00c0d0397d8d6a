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


def test_bench_train_two_ranks_cpu_standin():
    """bench.py --train past the launch check, world 2 on gloo: the CPU stand-in episode
    (CWT_BENCH_CPU_STANDIN) drives bench.py's own exchange (make_after: mean all-reduce of the
    gradient bucket, nesterov SGD) and clock (timed_region: barrier + max over ranks).  Every
    rank's replica is bitwise identical after every step although each rank ran its own
    episodes; value = world * steps / max-over-ranks time; n_gpus is the process group's."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(CWT_BENCH_CPU_STANDIN="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--train", "--steps", "3",
                        "--warmup", "1", "--size", "65"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    per_rank = {d["rank"]: d for d in lines if "rank" in d}
    assert sorted(per_rank) == [0, 1]
    d0, d1 = per_rank[0]["digests"], per_rank[1]["digests"]
    assert len(d0) == 1 + 3 and d0 == d1, (d0, d1)      # warm-up + timed steps, identical replicas
    assert len(set(d0)) == len(d0)                      # the parameters moved every step
    assert per_rank[0]["dt_max"] == per_rank[1]["dt_max"]   # one clock: the max over ranks
    (line,) = [d for d in lines if "metric" in d]
    assert line["n_gpus"] == 2 and line["steps"] == 3
    assert abs(line["value"] - 2 * 3 / per_rank[0]["dt_max"]) <= 1e-6 * line["value"]
