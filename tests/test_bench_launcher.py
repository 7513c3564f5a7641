"""bench.py --gpus N starts N rank processes itself when no launcher set WORLD_SIZE (the driver's
SCALE runs use torch.distributed.run; a plain `python bench.py --gpus 8` must measure 8 ranks too).
The dry-run mode rehearses the launcher on the CPU over gloo: no GPU call is made."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240)


def test_launcher_starts_every_rank():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                      # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == [0, 1]


def test_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "2", "--dry-run"], SKML_DRYRUN_FAIL_RANK="1")
    assert r.returncode != 0
    assert "rank(s) [1] failed" in r.stderr


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--dry-run"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=3 but --gpus 2" in r.stderr
