"""bench.py's N-rank launcher (CPU, gloo): `python bench.py --gpus N` without WORLD_SIZE starts
torch.distributed.run itself (the driver's scaling command form), and a WORLD_SIZE that
disagrees with --gpus fails loudly.  The dry run swaps the GPU decomposition for a stub, so
this covers the launch, the rank-0 JSON line and the gather over gloo -- not numbers."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=env, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus2_launches_two_ranks():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "3"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["dry_run"] is True and d["gathered_matrices"] == 6
    assert d["steps"] == 2 and d["warmup"] == 1 and d["config"]["parallelism"] == "dp2 (matrix-sharded)"


def test_gpus1_runs_in_process():
    p = _run(["--gpus", "1", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _json_lines(p.stdout)
    assert d["n_gpus"] == 1 and d["gathered_matrices"] == 4


def test_world_size_mismatch_fails_loudly():
    p = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in p.stderr
