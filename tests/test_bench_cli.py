"""bench.py's multi-GPU contract on the host (gloo rehearsal, eager solver): `--gpus N`
without a launcher starts N ranks itself, the reported n_gpus / global_batch come from the
process group, the strong-scaling companion splits the same batch, and a mismatch between
--gpus and an existing WORLD_SIZE is refused instead of reported."""
import json
import os
import subprocess
import sys

from conftest import REPO


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)


def test_bench_launches_ranks_and_accounts_batch():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--rehearse-cpu", "--workload", "tiny",
              "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                       # rank 0 only prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["traj_per_gpu"] == 64 and res["config"]["global_batch"] == 128
    assert res["scaling"] == "weak"
    assert res["strong_scaling"]["global_batch"] == 64 and res["strong_scaling"]["traj_per_gpu"] == 32
    assert res["value"] > 0 and res["strong_scaling"]["value"] > 0


def test_bench_strong_scaling_mode():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--rehearse-cpu", "--workload", "tiny",
              "--no-cpu-baseline", "--scaling", "strong"])
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["scaling"] == "strong" and res["n_gpus"] == 2
    assert res["config"]["global_batch"] == 64 and res["config"]["traj_per_gpu"] == 32


def test_bench_refuses_world_size_mismatch():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--rehearse-cpu", "--workload", "tiny",
              "--no-cpu-baseline"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
