#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X: Msamples/s through Hilbert -> modulator -> render.

Workload (BASELINE.json configs[1], SURVEY 8(d) "C2"): per GPU, 256 concurrent 48 kHz 16-bit
stereo streams, quadrature Hilbert with the reference's default Type-1 (order-19) elliptic
half-band IIR in Kahan mode, one Shift node (+2/-2 Hz) + Master (S_ADD_REIM, 0.8), 16-bit
ROUND / mid-riser / flat render.  One step = one pass over 2^20 frames of every stream (the
state carries from step to step, as in a continuous decode).  Inputs are resident in HBM before
the timed region; the C-ABI is called with device pointers (ICW_F_DEVICE_PTRS).

Metric: rendered output channel-samples per second (2 x frames/s), whole job over all ranks.
Multi-GPU: one process per GPU, streams sharded (weak scaling, no collective on the data path);
barrier + synchronize around the K timed steps, max elapsed over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]

--workload picks one of the BASELINE.json configs; the default, c2, is the one the
headline metric is quoted on.  The others are measured for DESIGN.md, not for the bench line.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CLOCK_GHZ = 2.4                # MI355X max engine clock (MI355X_MICROARCH.md chip table)
# Issue floor of icw_iir_state (DESIGN.md "Roofline"): a lone wave issues one FP64 VALU instruction
# per ~5.0 cycles, dependent or not, add or mul, whatever the operand banks
# (profiles/r01_fp64_bank_probe.txt: 5.00 and 5.25 s_memtime ticks per op on two boxes). The
# recurrence compiles to 91 FP64 VALU per sample on average (71 v_add_f64 + 19 v_mul_f64 + 1
# v_cmp_f64: the order-19 Kahan loop-back sum with the zero-input steps 4 adds shorter, ISA of
# icw_iir_state<19,1,1>) plus 2 v_cndmask_b32 -> a floor of ~455 cycles per sample per chain.
# The row-broadcast kernel icw_iir_row<19> (small batches: C2) issues 75.5 FP64 VALU per sample:
# nonzero-input samples 1 + 3 + (18 v_fmac_f64_dpp + 52 v_add_f64) + 1 v_cmp + 2 product muls = 77,
# zero-input samples 2 + 3 + (17 + 49) + 1 + 2 = 74 (plus 2 v_cndmask_b32, as above).
K1_VALU_PER_SAMPLE = {0: 91, 3: 75.5}          # by ICW_K1_* (icw_last_k1_kernel)
K1_KERNEL_NAME = {0: "icw_iir_state", 1: "icw_iir_pair", 2: "icw_iir_state_mf", 3: "icw_iir_row"}
CYC_PER_FP64_VALU = 5.0
PMC_FILE = ROOT / "profiles" / "r01_c2_pmc.json"
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector (256 CU x 2.4 GHz x 128 flop/clk), vendor figure


# SURVEY 8(d) configurations, per GPU: streams, frames per stream per step, fs, input format,
# channels, DSP list, render, algorithmic bytes per frame (input + output)
WORKLOADS = {
    "c2": dict(streams=256, frames=1 << 20, fs=48000, fmt="i16", ch=2, graph="shift_master", render="round16",
               bytes=8, desc="C2: 256 x 48kHz int16 stereo streams/GPU, Type-1 (order 19) Kahan quadrature "
                             "Hilbert + Shift(+2/-2 Hz) + Master, 16-bit ROUND"),
    "c3": dict(streams=4096, frames=1 << 18, fs=96000, fmt="i16", ch=1, graph="master_only", render="round16",
               bytes=6, desc="C3: 4096 x 96kHz int16 mono streams/GPU, Hilbert + Master, 16-bit ROUND"),
    "c4": dict(streams=2048, frames=1 << 18, fs=48000, fmt="i16", ch=2, graph="pm_shift_mix", render="round16",
               bytes=8, desc="C4: 2048 x 48kHz int16 stereo streams/GPU, PM -> Shift -> Mix -> Master, 16-bit ROUND"),
    "c5": dict(streams=256, frames=1 << 18, fs=192000, fmt="f32", ch=2, graph="master_only", render="tpdf24_mew44",
               bytes=14, desc="C5: 256 x 192kHz float32 stereo streams/GPU, Hilbert + Master, 24-bit TPDF + "
                              "MEW44 noise shaping"),
}


def workload_config(w):
    from in_cwave_amd import abi, graph
    fmt = {"i16": abi.FMT_I16, "f32": abi.FMT_F32}[w["fmt"]]
    cfg = graph.default_config(w["fs"], fmt=fmt, channels=w["ch"], need24bits=w["render"].endswith("mew44"))
    if w["render"] == "tpdf24_mew44":
        cfg.render.render_type = abi.RENDER_TPDF
        cfg.render.nshape_type = abi.NSHAPE_MEW44
    nodes = {"shift_master": graph.graph_shift_master, "master_only": graph.graph_master_only,
             "pm_shift_mix": graph.graph_pm_shift_mix}[w["graph"]]()
    return cfg, nodes, fmt


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--streams", type=int, default=None, help="streams per GPU (default: the workload's)")
    ap.add_argument("--frames", type=int, default=None, help="frames per stream per step (default: the workload's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--cpu-frames", type=int, default=1 << 25)
    return ap.parse_args()


def _cpu_worker(args):
    """one CPU core: the oracle restatement (scalar C, -O2 -ffp-contract=off) over one stream"""
    s, n_frames, wname = args
    from in_cwave_amd import synth
    from oracle import oracle as O
    w = WORKLOADS[wname]
    cfg, nodes, fmt = workload_config(w)
    raw = synth.stream_pcm(s, n_frames, w["fs"], channels=w["ch"], fmt=fmt)
    st = O.Stream(cfg, nodes)
    t0 = time.perf_counter()
    st.process(raw, n_frames)
    return time.perf_counter() - t0


def cpu_baseline(workers, n_frames, wname):
    import multiprocessing as mp
    from oracle import oracle as O
    O.load()
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        per = pool.map(_cpu_worker, [(s, n_frames, wname) for s in range(workers)])
    wall = time.perf_counter() - t0
    busy = max(per)
    samples = 2.0 * n_frames * workers
    return {"value": samples / busy / 1e6, "unit": "Msamples/s", "cores": workers, "kind": "port",
            "sample": f"{workers} streams x {n_frames} frames ({wname} shape, oracle C restatement, one process "
                      f"per core), per-core {2.0 * n_frames / np.mean(per) / 1e6:.3f} Msamples/s, wall {wall:.1f}s"}


def main():
    a = parse()
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; ICW_BENCH_BACKEND=gloo + fewer GPUs than ranks is the rehearsal mode of
    # tests/test_gpu_bench.py (ranks share a device; RCCL needs one GPU per rank)
    ndev = torch.cuda.device_count()
    local_dev = local % max(1, ndev)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_dev)
        dist.init_process_group(os.environ.get("ICW_BENCH_BACKEND", "nccl"), rank=rank, world_size=world)
    dev = torch.device("cuda", local_dev)
    torch.cuda.set_device(dev)

    from in_cwave_amd import graph, synth
    from in_cwave_amd import lib as L

    W = WORKLOADS[a.workload]
    S = a.streams or W["streams"]
    T = a.frames or W["frames"]
    fs = W["fs"]
    cfg, nodes, fmt = workload_config(W)
    ctx = L.Context(cfg, nodes, S, device=local_dev)
    # synthetic input of the workload's shape for this rank's shard of streams (SURVEY 8(d)
    # generator); 16 distinct generated streams are tiled over the shard to bound setup time
    n_gen = min(S, 16)
    first = rank * S
    gen = synth.batch_pcm(n_gen, T, fs, channels=W["ch"], fmt=fmt, first=first)   # uint8 [n_gen, T*fsz]
    d_in = torch.empty((S, gen.shape[1]), dtype=torch.uint8, device=dev)
    g = torch.from_numpy(gen).to(dev)
    for s in range(S):
        d_in[s].copy_(g[s % n_gen])
    del g
    osz = 2 * ctx.render_size
    d_out = torch.empty((S, T * osz), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    hip_stream = torch.cuda.current_stream(dev).cuda_stream

    def step(timing):
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, timing=timing, hip_stream=hip_stream)

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    k1_ms = k2_ms = 0.0
    k1_n = k2_n = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
        (m1, m2), (n1, n2) = ctx.last_timing()
        k1_ms += m1
        k2_ms += m2
        k1_n += n1
        k2_n += n2
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.synchronize()     # raises if a kernel reported a failed hand-off
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames_total = float(S) * T * a.steps * world
    value = 2.0 * frames_total / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / a.steps

    # roofline of the dominant kernel (icw_iir_state), algorithmic bytes per launch / avg duration
    frames_per_launch = float(S) * T * a.steps / max(1, k1_n)
    k1_avg_s = k1_ms / 1e3 / max(1, k1_n)
    k2_avg_s = k2_ms / 1e3 / max(1, k2_n)
    alg_bytes = W["bytes"]
    achieved = alg_bytes * frames_per_launch / k1_avg_s / 1e9 if k1_avg_s > 0 else None
    flops_per_frame = 4 * 2 * (15 * 19 - 4) / 2    # the recurrence half of 1124 flops/frame
    k1_kind = ctx.last_k1_kernel()
    k1_name = K1_KERNEL_NAME.get(k1_kind, "?")
    valu = K1_VALU_PER_SAMPLE.get(k1_kind)
    traffic = None
    try:   # HBM bytes per launch of the same kernel/config from the committed PMC passes
        pmc = json.loads(PMC_FILE.read_text())
        if int(pmc["frames_per_launch"]) == int(frames_per_launch) and a.workload == "c2":
            traffic = next(v["hbm_bytes_corrected"] for k, v in pmc["kernels"].items()
                           if k.split("<")[0].split("(")[0].endswith(k1_name))
    except Exception:
        traffic = None
    samples_per_chain = frames_per_launch / S
    issue_floor_ms = (samples_per_chain * valu * CYC_PER_FP64_VALU / (CLOCK_GHZ * 1e6)) if valu else None
    roof = {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
        "issue_bound": {"valu_per_sample": valu, "cycles_per_valu": CYC_PER_FP64_VALU,
                        "clock_ghz": CLOCK_GHZ, "floor_ms_per_launch": issue_floor_ms,
                        "frac": (issue_floor_ms / (k1_avg_s * 1e3)) if (k1_avg_s and issue_floor_ms) else None},
        "kernel": k1_name, "alg_bytes_per_frame": alg_bytes,
        "frames_per_launch": frames_per_launch, "avg_launch_ms": k1_avg_s * 1e3,
        "output_kernel_avg_launch_ms": k2_avg_s * 1e3,
        "fp64_tflops_chain": (1124.0 * frames_per_launch / (k1_avg_s + k2_avg_s) / 1e12) if k1_avg_s else None,
        "fp64_peak_tflops": FP64_PEAK_TFLOPS,
        "note": f"issue-bound serial IIR recurrence ({4 * S} DF-II chains, 2 per stream with the mono dedup; "
                f"{'one 16-lane DPP row' if k1_kind == 3 else 'one lane'} per chain), {valu} FP64 VALU per "
                f"sample; frac ~1 = at the issue floor within the probe's few-% spread (DESIGN.md)",
    }
    del flops_per_frame

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.cpu_workers, a.cpu_frames, a.workload)
        except Exception as e:  # reported, never silently replaced
            cpu = {"error": repr(e)}

    if rank == 0:
        line = {
            "metric": "Msamples/s through Hilbert+mod+render",
            "value": value, "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": W["desc"],
                       "streams_per_gpu": S, "frames_per_stream_per_step": T, "fs": fs,
                       "parallelism": f"stream-shard x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
