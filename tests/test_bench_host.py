"""bench.py host logic without a GPU: the --gpus / WORLD_SIZE contract and the CPU-baseline core
census (one process per physical core, CPU model stated)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

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


def test_roofline_inputs_from_committed_profiles():
    """the roofline fields recompute from profiles/: HBM bytes per launch from the newest PMC pass
    of the workload (scaled by frames per launch), the issue model from its SQ pass (VALU per wave,
    cycles per VALU = profiled launch time x SQ clock / VALU per wave), and the whole-chain FP64
    work per frame of SURVEY 8(d) (4 filters x (15N - 4) for stereo)"""
    import json
    import bench
    assert bench.chain_flops_per_frame(2) == 1124 and bench.chain_flops_per_frame(1) == 562
    f = bench._latest("r*_c2_pmc.json")
    pmc = json.loads(f.read_text())
    fpl = float(pmc["frames_per_launch"])
    t, src = bench.pmc_traffic("c2", "icw_iir_row", fpl)
    k = next(v for kk, v in pmc["kernels"].items() if "icw_iir_row" in kk)
    assert src == f.name and abs(t - k["hbm_bytes_corrected"]) < 1e-6 * t
    t2, _ = bench.pmc_traffic("c2", "icw_iir_row", fpl / 2)
    assert abs(t2 - t / 2) < 1e-6 * t
    m = bench.sq_model("c2", "icw_iir_row")
    valu, cpv, clk, ns, name = m
    assert 3.0 < cpv < 6.0 and 1.5 < clk < 2.5 and valu > 0
    assert abs(cpv - ns * clk / valu) < 1e-9
    assert bench.pmc_traffic("c2", "no_such_kernel", fpl) == (None, None)
    # the issue floor's cycles per VALU: the Kahan add chain of the committed latency probe
    cfl, src = bench.fp64_issue_floor()
    assert src == "r01_fp64_latency_probe.txt" and 3.5 < cfl < cpv


def test_control_backend_defaults_to_gloo(monkeypatch):
    """the bench's control plane (barriers, the elapsed-time max-reduce) is gloo whatever the
    device count, so an 8-GPU run executes the code the 2-rank tests run; RCCL only on request and
    only with one device per rank"""
    import bench
    monkeypatch.delenv("ICW_BENCH_BACKEND", raising=False)
    assert bench.control_backend(8, 8) == "gloo"
    assert bench.control_backend(1, 2) == "gloo"
    monkeypatch.setenv("ICW_BENCH_BACKEND", "nccl")
    assert bench.control_backend(8, 8) == "nccl"
    assert bench.control_backend(1, 2) == "gloo"
    monkeypatch.setenv("ICW_BENCH_BACKEND", "mpi")
    with pytest.raises(SystemExit):
        bench.control_backend(8, 8)
