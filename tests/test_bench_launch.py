"""bench.py's multi-GPU launcher: `--gpus N` without a
torch.distributed launcher starts one as a child process with N ranks, each
seeing WORLD_SIZE = N (probed before any GPU work, so this runs on CPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240, cwd=ROOT)


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--probe-ranks"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]


def test_world_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--probe-ranks"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--probe-ranks"])
    assert r.returncode == 0
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1, "local_rank": 0}
