"""bench.py host logic without a GPU: the --gpus / WORLD_SIZE contract and the CPU-baseline core
census (one process per physical core, CPU model stated)."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def test_world_size_must_match_gpus():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_self_launch_propagates_rank_failure():
    """--gpus 2 without a launcher starts 2 rank processes (RANK / WORLD_SIZE set for each); here,
    without a GPU, the ranks fail at their first device call and the parent returns nonzero
    instead of hanging or printing a line"""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_host_cores_census():
    import bench
    n, cpus, model, topo = bench.host_cores()
    assert 1 <= n <= os.cpu_count() and len(cpus) == n
    assert set(cpus) <= set(os.sched_getaffinity(0))
    assert isinstance(model, str) and model
    assert topo["physical_in_affinity"] >= n
