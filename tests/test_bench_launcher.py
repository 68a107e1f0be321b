"""bench.py's rank launcher (CPU, no GPU touched): `--gpus N` without a launcher starts N
rank processes with the torchrun environment; under a launcher --gpus must equal
WORLD_SIZE."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_n_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--configs", "none", "--no-cpu"],
                       env=_env(BT_BENCH_SPAWN_CHECK="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(int(x["RANK"]) for x in ranks) == [0, 1, 2]
    assert all(x["WORLD_SIZE"] == "3" and x["MASTER_ADDR"] == "127.0.0.1" for x in ranks)
    assert sorted(int(x["LOCAL_RANK"]) for x in ranks) == [0, 1, 2]


def test_gpus_must_match_launcher_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--configs", "none", "--no-cpu"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", BT_BENCH_SPAWN_CHECK="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr


def test_failing_rank_ends_the_launch():
    # no GPU here: every rank fails at bt_create, and the launcher returns non-zero
    # instead of waiting on ranks stuck at a barrier
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--configs", "none", "--no-cpu", "--packets", "4096"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
