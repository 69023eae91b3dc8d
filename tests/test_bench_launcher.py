"""bench.py's rank launcher (CPU): `python bench.py --gpus N` without torch.distributed.run must
start N rank processes itself -- one per GPU, rendezvous on 127.0.0.1 -- and refuse a run whose
process count differs from --gpus (the driver's scaling runs use both forms)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_rank_plan_has_every_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--spawn-dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])["ranks"]
    assert [p["RANK"] for p in plan] == [str(i) for i in range(8)]
    assert [p["LOCAL_RANK"] for p in plan] == [str(i) for i in range(8)]
    assert {p["WORLD_SIZE"] for p in plan} == {"8"}
    assert {p["MASTER_ADDR"] for p in plan} == {"127.0.0.1"}
    assert len({p["MASTER_PORT"] for p in plan}) == 1


def test_launcher_starts_ranks_that_rendezvous():
    """Two rank processes started by bench.py itself join one gloo group (all_reduce of rank + 1)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--rank-selftest"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"world": 2, "sum": 3, "gpus": 2, "local_rank": 0}


def test_mismatched_world_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--rank-selftest"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_single_process_default():
    r = subprocess.run([sys.executable, BENCH, "--rank-selftest"], capture_output=True, text=True, env=_env(),
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["world"] == 1
