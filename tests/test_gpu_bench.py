"""bench.py end to end on the GPU: the single-process line, and the multi-rank path (torchrun,
barrier, max-over-ranks timing, whole-job value) rehearsed with two ranks on the box's one GPU
over gloo -- the driver's 8-GPU run takes the same code with RCCL, one GPU per rank."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_rank_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--frames", "65536",
                        "--no-cpu-baseline", "--e2e-steps", "0"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["unit"] == "Msamples/s" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["roofline"]["avg_launch_ms"] > 0
    # value = 2 x frames x streams / time
    assert abs(d["value"] - 2.0 * 256 * 65536 / (d["ms_per_step"] / 1e3) / 1e6) < 1e-6 * d["value"]


def test_bench_two_ranks_rehearsal():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "1", "--warmup", "1", "--frames", "32768", "--streams", "64", "--e2e-steps", "0",
                        "--no-cpu-baseline", "--no-other-workloads"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["cpu_baseline"] is None and d["other_workloads"] is None
    # whole-job value: both ranks' streams over the max-over-ranks time
    assert abs(d["value"] - 2.0 * 2 * 64 * 32768 / (d["ms_per_step"] / 1e3) / 1e6) < 1e-6 * d["value"]


def test_bench_gpus_flag_self_launches():
    """python bench.py --gpus 2 with no launcher: two rank processes sharing the box's GPU (gloo),
    n_gpus 2 in the one line rank 0 prints, whole-job value; the multi-GPU line carries the C4 / C5
    legs BASELINE.json quotes at 8 GPUs (per-GPU shard sizes, whole-job values over the max-over-ranks
    time) and the roofline from rank 0's K1 events; the CPU baseline is an N = 1 field (null here)"""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--frames", "32768", "--streams", "64", "--e2e-steps", "0", "--other-frames", "16384"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    # the control plane the 8-GPU run uses too: gloo, whatever the device count (bench.control_backend)
    assert d["config"]["control_backend"] == "gloo"
    assert abs(d["value"] - 2.0 * 2 * 64 * 32768 / (d["ms_per_step"] / 1e3) / 1e6) < 1e-6 * d["value"]
    assert d["roofline"]["avg_launch_ms"] > 0 and 0 < d["roofline"]["frac"] < 1
    assert d["cpu_baseline"] is None
    ow = d["other_workloads"]
    for w, streams in (("c4", 2048), ("c5", 256), ("c4fir", 2048), ("c5fir", 256)):
        o = ow[w]
        assert o["n_gpus"] == 2 and o["streams_per_gpu"] == streams and o["streams_total"] == 2 * streams
        assert o["frames_per_stream_per_step"] == 16384
        assert abs(o["value"] - 2.0 * streams * 2 * 16384 / (o["ms_per_step"] / 1e3) / 1e6) < 1e-6 * o["value"]


def test_bench_line_fields():
    """the roofline is FP64-bound with HBM and issue-floor fields, the e2e host-buffer rate is
    reported beside `value`"""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--frames", "65536",
                        "--no-cpu-baseline", "--e2e-steps", "1"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    rf = d["roofline"]
    assert rf["bound"] == "fp64" and rf["unit"] == "TFLOP/s" and 0 < rf["frac"] < 1
    assert abs(rf["achieved"] - rf["flops_per_frame"] * rf["frames_per_launch"] / rf["avg_launch_ms"] / 1e9) \
        < 1e-9 * rf["achieved"]
    assert rf["hbm"]["unit"] == "GB/s" and 0 < rf["issue_bound"]["frac"] <= 1.0
    assert 0 < rf["chain_fp64"]["frac"] < 1
    assert d["e2e_host_buffers"]["value"] > 0


def test_bench_c1_drop_in_line():
    """C1: the C host through the drop-in boundary in 576-frame blocks; its output equals the oracle's"""
    r = subprocess.run([sys.executable, "bench.py", "--workload", "c1", "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["parity_vs_oracle"] == "bit-exact"
    assert d["value"] > 0 and d["block_latency_us"]["p50"] > 0 and d["cpu_baseline"]["cores"] == 1
