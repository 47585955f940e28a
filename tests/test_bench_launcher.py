"""bench.py's own multi-rank launch (CPU, gloo dry run): `bench.py --gpus N` without an external
launcher starts the N rank processes itself and reports n_gpus = N; a --gpus that disagrees
with WORLD_SIZE fails with a non-zero exit."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def test_self_launch_two_ranks_dry_run():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["backend"] == "gloo"
    # N > 1: the headline is the single row-sharded instance (strong scaling), replicas beside it
    assert d["headline"].startswith("sharded") and d["scaling"] == "strong"
    assert d["config"]["parallelism"].startswith("row-sharded x2") and d["replicas"]["scaling"] == "weak"
    assert d["ranks_aggregated"] == 2   # both ranks met the barrier and the aggregate


def test_self_launch_three_ranks_dry_run():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 3 and d["ranks_aggregated"] == 3


def test_gpus_must_match_world_size():
    env = _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_single_rank_dry_run_defaults_to_one():
    r = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 1
