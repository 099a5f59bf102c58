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

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5]

--gpus N without a launcher (RANK unset) starts N rank processes itself, before anything here
touches the GPU, and exits with the worst rank's status; under torch.distributed.run the world
size must equal --gpus.  The control plane (barriers, the max-reduce of the elapsed time) runs
on gloo by default (ICW_BENCH_BACKEND=nccl opts into RCCL, one GPU per rank): the data path has
no collective, so the 8-GPU run executes the same code as the 2-rank tests.  With fewer devices
than ranks (the 1-GPU box) the ranks share devices.

--workload picks one of the BASELINE.json configs; the default, c2, is the one the
headline metric is quoted on.  A default run at N=1 also measures the other configs briefly
(C3/C4/C5: 1 warmup + 2 steps each; C1: one pass) and reports them under `other_workloads` in the
same line -- beside the headline, never in `value`; --no-other-workloads or --no-cpu-baseline skip
them.
c1 is the single-stream drop-in: the C host examples/icw_transcode (no Python in its loop) decodes
a 30 s 44.1 kHz stereo track through icw_amod_process_samples in 576-frame blocks from host
memory, timing every call; its CPU baseline is the oracle on the same track on one core, and the
two outputs are compared byte for byte.

Roofline: the dominant kernel is the serial IIR recurrence K1; its bound is FP64
VALU issue, so `roofline` reports its algorithmic FP64 rate (the loop-back Kahan sum,
hblpf.c:1017-1046: 5N flops per chain-sample, 95 for N = 19) against the FP64 vector peak, with
the HBM rate and the per-wave issue floor as secondary fields.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector (256 CU x 2.4 GHz x 128 flop/clk), MI355X_MICROARCH.md
# effective engine clock under the C2 recurrence: SQ_BUSY_CYCLES / 32 shader engines / launch time
# of the K1 kernel in the newest committed SQ pass (profiles/r*_c2_sq.json; r01: 2.31 GHz)
CLOCK_GHZ = 2.31
# Issue model of the recurrence: a chain costs (VALU instructions per sample) x
# (cycles per VALU).  Both come from the newest committed SQ pass of the workload
# (profiles/r*_<workload>_sq.json: SQ_INSTS_VALU per wave / samples per chain, and the profiled
# launch time x SQ_BUSY_CYCLES clock / VALU per wave); the fallbacks are the round-2 figures
# (icw_iir_state<19> 91.1, icw_iir_row<19> 75.4 VALU per sample; 4.83 cycles per VALU).
K1_VALU_PER_SAMPLE = {0: 91.1, 3: 75.4}        # by ICW_K1_* (icw_last_k1_kernel)
K1_KERNEL_NAME = {0: "icw_iir_state", 3: "icw_iir_row", 4: "icw_iir_state_fc"}
CYC_PER_FP64_VALU = 4.83


def fp64_issue_floor():
    """cycles per dependent FP64 add on gfx950: a chain of v_add_f64, each reading the previous
    result, on one wave with 64 active lanes (tools/lat_probe.hip, profiles/r01_fp64_latency_probe.txt)"""
    import re
    f = ROOT / "profiles" / "r01_fp64_latency_probe.txt"
    try:
        m = re.search(r"active lanes 64: dep_add ([0-9.]+) cyc/op", f.read_text())
        return float(m.group(1)), f.name
    except (OSError, AttributeError, ValueError):
        return 4.62, None
# the path's algorithmic FP64 work per frame is the whole Kahan IIR of
# iir_rp_process_kahan (hblpf.c:1017-1056): 15N - 4 flops per filter-sample (N = 19: 281), over the
# 4 filters of a stereo frame (1 124) or the 2 of a mono frame under the dedup (562) -- the
# loop-back sum (K1, 5N per sample) plus the output sum (K2)
def chain_flops_per_frame(ch):
    return (2 if ch == 1 else 4) * (15 * IIR_ORDER - 4)


def _latest(pattern):
    files = sorted(glob.glob(str(ROOT / "profiles" / pattern)))
    return Path(files[-1]) if files else None


# SURVEY 8(d) configurations, per GPU: streams, frames per stream per step, fs, input format,
# channels, DSP list, render, algorithmic bytes per frame (input + output)
WORKLOADS = {
    "c1": dict(streams=1, frames=1323000, fs=44100, fmt="i16", ch=2, graph="shift_master", render="round16",
               bytes=8, desc="C1: 1 x 44.1kHz int16 stereo stream, 30 s, drop-in boundary in 576-frame blocks "
                             "(host buffers), Type-1 Kahan Hilbert + Shift(+2/-2 Hz) + Master, 16-bit ROUND"),
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
# The same configs through the FIR Hilbert converter (icw_set_fir_hilbert) with the tap counts
# BASELINE.json names (255 / 511 / 1023 taps = order 254 / 510 / 1022, Kaiser beta 8) instead of the
# reference's quadrature IIR: the converter a CWAVE header records (cwave.h:56-58), run on the fly.
# Reported under other_workloads only; the headline stays the reference's own IIR path.
FIR_BETA = 8.0
for _w, _order in (("c2", 254), ("c3", 510), ("c4", 254), ("c5", 1022)):
    _d = WORKLOADS[_w]["desc"].replace("Type-1 (order 19) Kahan quadrature Hilbert", "Hilbert")
    _d = _d.replace("streams/GPU, PM", "streams/GPU, Hilbert + PM")
    WORKLOADS[_w + "fir"] = dict(WORKLOADS[_w], fir=_order,
                                 desc=_d.replace("Hilbert", f"{_order + 1}-tap FIR Hilbert (Kaiser beta {FIR_BETA:g})", 1))
IIR_ORDER = 19                  # Type-1 filter of every workload (hblpf.c:740-820)


def workload_config(w):
    from in_cwave_amd import abi, graph
    fmt = {"i16": abi.FMT_I16, "f32": abi.FMT_F32}[w["fmt"]]
    cfg = graph.default_config(w["fs"], fmt=fmt, channels=w["ch"], need24bits=w["render"].endswith("mew44"))
    if w["render"] == "tpdf24_mew44":
        cfg.render.render_type = abi.RENDER_TPDF
        cfg.render.nshape_type = abi.NSHAPE_MEW44
    # ICW_BENCH_RENDER (diagnostics only, never the headline): a dithered render with the flat shaper,
    # "<rpdf|tpdf|stpdf|gauss>_flat", on the same shape (the frame-parallel dithered render's A/B)
    rr = os.environ.get("ICW_BENCH_RENDER")
    if rr:
        cfg.render.render_type = {"rpdf": abi.RENDER_RPDF, "tpdf": abi.RENDER_TPDF, "stpdf": abi.RENDER_STPDF,
                                  "gauss": abi.RENDER_GAUSS}[rr.split("_")[0]]
        cfg.render.nshape_type = abi.NSHAPE_FLAT
    # ICW_BENCH_GRAPH (diagnostics only, never the headline): another of the three lists on the same shape
    g = os.environ.get("ICW_BENCH_GRAPH") or w["graph"]
    nodes = {"shift_master": graph.graph_shift_master, "master_only": graph.graph_master_only,
             "pm_shift_mix": graph.graph_pm_shift_mix}[g]()
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
    ap.add_argument("--no-other-workloads", action="store_true",
                    help="c2 at N=1: skip the short C1/C3/C4/C5 runs reported under other_workloads")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: one per physical core available here")
    ap.add_argument("--cpu-frames", type=int, default=1 << 25)
    ap.add_argument("--other-frames", type=int, default=None,
                    help="frames per stream of the other_workloads legs (default: each workload's)")
    ap.add_argument("--block", type=int, default=576, help="c1: frames per boundary call (NS_PERTIME)")
    ap.add_argument("--e2e-steps", type=int, default=2,
                    help="extra steps with host buffers (H2D + D2H included), reported beside `value`")
    return ap.parse_args()


# ----------------------------------------------------------------------------- launcher -----
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus N without a launcher: N fresh rank processes of this script (one per GPU), started
    before this process touches the GPU; the first rank to fail stops the others.  Returns the
    worst exit status."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    worst = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                worst = worst or rc
                for q in live:          # a failed rank leaves the others waiting in a barrier
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return worst if worst >= 0 else 128 - worst


# ----------------------------------------------------------------------------- CPU leg ------
def host_cores():
    """physical cores this process may run on: the affinity set grouped by (package, core id),
    capped by a cgroup CPU quota; plus the CPU model string"""
    cpus = sorted(os.sched_getaffinity(0))
    phys = {}
    for c in cpus:
        base = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
        try:
            key = (base.joinpath("physical_package_id").read_text().strip(), base.joinpath("core_id").read_text().strip())
        except OSError:
            key = ("?", str(c))
        phys.setdefault(key, c)
    n = len(phys)
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    if quota:
        n = max(1, min(n, int(quota)))
    model = "?"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, sorted(phys.values())[:n], model, {"affinity_cpus": len(cpus), "physical_in_affinity": len(phys),
                                                 "cgroup_cpu_quota": quota}


def _cpu_worker(args):
    """one physical core: the oracle restatement (scalar C, -O2 -ffp-contract=off) over one stream"""
    s, n_frames, wname, cpu = args
    try:
        os.sched_setaffinity(0, {cpu})
    except OSError:
        pass
    from in_cwave_amd import synth
    from oracle import oracle as O
    w = WORKLOADS[wname]
    cfg, nodes, fmt = workload_config(w)
    raw = synth.stream_pcm(s, n_frames, w["fs"], channels=w["ch"], fmt=fmt)
    st = O.Stream(cfg, nodes)
    if w.get("fir"):
        st.set_fir(w["fir"], FIR_BETA)
    t0 = time.perf_counter()
    st.process(raw, n_frames)
    return time.perf_counter() - t0


def cpu_baseline(workers, n_frames, wname):
    """the oracle's C restatement, one process per physical core, each on one stream of the
    workload's shape; aggregate = all cores' samples over the slowest core's time"""
    import multiprocessing as mp
    from oracle import oracle as O
    O.load()
    n_avail, cpus, model, topo = host_cores()
    workers = workers or n_avail
    cpus = (cpus * ((workers + len(cpus) - 1) // len(cpus)))[:workers]
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        per = pool.map(_cpu_worker, [(s, n_frames, wname, cpus[s]) for s in range(workers)])
    wall = time.perf_counter() - t0
    samples = 2.0 * n_frames * workers
    out = {"value": samples / max(per) / 1e6, "unit": "Msamples/s", "cores": workers, "kind": "port",
           "cpu_model": model, "per_core": 2.0 * n_frames / float(np.mean(per)) / 1e6, "topology": topo,
           "sample": f"{workers} streams x {n_frames} frames ({wname} shape), oracle C restatement "
                     f"(-O2 -ffp-contract=off), one process pinned per physical core, wall {wall:.1f}s; "
                     f"the reference's own IIR/graph/render need <windows.h> and are not built here"}
    # the restatement's speed against the reference C on one CPU type (tools/cpu_calibrate.py,
    # against BASELINE.md's reference numbers measured on the same container CPU)
    cal = _latest("r*_cpu_calibration.json")
    if cal is not None:
        try:
            r = json.loads(cal.read_text().strip().splitlines()[-1])["workloads"].get(wname)
            if r:
                out["calibration"] = {"oracle_over_reference": r["oracle_over_reference"], "cpu": "container Xeon",
                                      "reference_equivalent_value": out["value"] / r["oracle_over_reference"],
                                      "source": f"profiles/{cal.name}"}
        except (ValueError, KeyError):
            pass
    return out


# ----------------------------------------------------------------------------- C1 leg -------
def _wav_i16(path, raw, rate, ch):
    import struct
    data = raw.tobytes()
    fmt = struct.pack("<HHIIHH", 1, ch, rate, rate * 2 * ch, 2 * ch, 16)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) + data
    Path(path).write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)


def bench_c1(a):
    print(json.dumps(measure_c1(a.steps, a.warmup, a.block, not a.no_cpu_baseline)), flush=True)


def measure_c1(steps, warmup, block, with_cpu):
    """single-stream drop-in: K runs of the C host over the track, W untimed"""
    import tempfile
    from in_cwave_amd import synth
    W = WORKLOADS["c1"]
    exe = ROOT / "examples" / "icw_transcode"
    if not exe.exists():
        raise SystemExit("bench.py c1: examples/icw_transcode is not built (make -C examples)")
    raw = synth.stream_pcm(0, W["frames"], W["fs"])
    tmp = Path(tempfile.mkdtemp(prefix="icw_c1_"))
    src, dst = tmp / "c1.wav", tmp / "c1_out.wav"
    _wav_i16(src, raw, W["fs"], 2)
    env = dict(os.environ, ICW_TIMING="1")
    runs = []
    for i in range(warmup + steps):
        r = subprocess.run([str(exe), str(src), str(dst), str(block), "shift", "16"], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise SystemExit(f"icw_transcode failed ({r.returncode}): {r.stderr[-500:]}")
        if i >= warmup:
            runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    out = np.frombuffer(dst.read_bytes()[44:], dtype=np.uint8)
    decode_s = sum(x["decode_s"] for x in runs)
    value = 2.0 * W["frames"] * len(runs) / decode_s / 1e6
    cpu = parity = None
    if with_cpu:
        from oracle import oracle as O
        n_avail, cpus, model, topo = host_cores()
        old_aff = os.sched_getaffinity(0)
        try:
            os.sched_setaffinity(0, {cpus[0]})
        except OSError:
            pass
        cfg, nodes, _ = workload_config(W)
        st = O.Stream(cfg, nodes)
        st.open(W["frames"])
        outs = []
        t0 = time.perf_counter()
        for f0 in range(0, W["frames"], block):
            n = min(block, W["frames"] - f0)
            outs.append(st.process(raw[f0 * 4:(f0 + n) * 4], n)[0])
        dt = time.perf_counter() - t0
        try:
            os.sched_setaffinity(0, old_aff)
        except OSError:
            pass
        ref = np.concatenate(outs)
        parity = "bit-exact" if np.array_equal(ref, out) else "MISMATCH"
        cpu = {"value": 2.0 * W["frames"] / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
               "cpu_model": model, "sample": f"the same 30 s track, oracle C restatement in {block}-frame "
                                              f"blocks on one pinned core, {dt:.2f}s"}
    last = runs[-1]
    line = {
        "metric": "Msamples/s through Hilbert+mod+render", "value": value, "unit": "Msamples/s", "n_gpus": 1,
        "steps": len(runs), "warmup": warmup, "ms_per_step": decode_s * 1e3 / len(runs),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": W["desc"], "streams_per_gpu": 1, "frames_per_stream_per_step": W["frames"],
                   "fs": W["fs"], "block_frames": block, "parallelism": "single stream"},
        "block_latency_us": last["block_us"], "realtime_x": last["realtime_x"], "parity_vs_oracle": parity,
        "cpu_baseline": cpu,
        "note": "host pointers through the drop-in boundary: each call stages its block H2D, runs K0-K2 "
                "and copies D2H before returning, as the DecodeThread needs; ms_per_step = time inside "
                "the boundary calls (file I/O excluded)",
    }
    for f in (src, dst):
        f.unlink()
    tmp.rmdir()
    return line


# ----------------------------------------------------------------------------- GPU leg ------
def pmc_traffic(wname, kernel, frames_per_launch):
    """HBM bytes per launch of `kernel` in the newest committed PMC pass of this workload
    (profiles/r*_<workload>_pmc.json, 2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950
    correction), scaled to this run's frames per launch; (bytes, file name) or (None, None)"""
    f = _latest(f"r*_{wname}_pmc.json")
    if f is None:
        return None, None
    try:
        pmc = json.loads(f.read_text())
        for k, v in pmc["kernels"].items():
            if k.split("<")[0].split("(")[0].split()[-1] == kernel:
                return v["hbm_bytes_corrected"] * frames_per_launch / float(pmc["frames_per_launch"]), f.name
    except (ValueError, KeyError, OSError):
        pass
    return None, None


def sq_model(wname, kernel):
    """(VALU per wave, cycles per VALU, clock GHz, launch ns, file) of `kernel` in the newest SQ pass"""
    f = _latest(f"r*_{wname}_sq.json")
    if f is None:
        return None
    try:
        for k, v in json.loads(f.read_text())["kernels"].items():
            if kernel in k:
                cpv = v["avg_launch_ns_trace"] * v["effective_clock_ghz"] / v["valu_per_wave"]
                return v["valu_per_wave"], cpv, v["effective_clock_ghz"], v["avg_launch_ns_trace"], f.name
    except (ValueError, KeyError, OSError, ZeroDivisionError):
        pass
    return None


def fir_roofline(wname, W, S, T, kf_ms, kf_n, k2_ms, k2_n, fused):
    """roofline of the FIR converter per launch, from its HIP events: per channel-sample nt odd
    taps x (1 subtract + 1 FMA = 3 flops); HBM traffic from the workload's committed PMC pass"""
    M = W["fir"]
    nt = (M // 2 + 1) // 2
    chans = 1 if W["ch"] == 1 else 2
    frames_per_launch = float(S) * T / max(1, kf_n)
    avg_s = kf_ms / 1e3 / max(1, kf_n)
    flops_per_frame = chans * nt * 3
    # the fused converter's ROUND renders run the signature form (icw_fir_sig) over every tile but the
    # one holding a launch block's last frame, which icw_fir_graph takes in a second launch; the HIP
    # events span both (icw_fir_graph's tile is 1/1024 of a c2fir launch's frames)
    sig = (fused and W["render"] == "round16" and not os.environ.get("ICW_BENCH_RENDER")
           and os.environ.get("ICW_FIR_SIG", "1") != "0")
    kname = ("icw_fir_sig" if sig else "icw_fir_graph") if fused else "icw_fir_hilbert"
    traffic, src = pmc_traffic(wname, kname, frames_per_launch)
    tf = flops_per_frame * frames_per_launch / avg_s / 1e12 if avg_s > 0 else None
    alg_b = W["bytes"] * frames_per_launch
    gbs = (traffic if traffic else alg_b) / avg_s / 1e9 if avg_s > 0 else None
    return {"bound": "fp64", "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": (tf / FP64_PEAK_TFLOPS) if tf else None, "traffic": traffic, "kernel": kname,
            "fir_order": M, "taps_odd": nt, "flops_per_frame": flops_per_frame, "frames_per_launch": frames_per_launch,
            "avg_launch_ms": avg_s * 1e3, "output_kernel_avg_launch_ms": k2_ms / max(1, k2_n),
            "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": (gbs / HBM_PEAK_GBS) if gbs else None,
                    "bytes_per_frame": (traffic if traffic else alg_b) / frames_per_launch,
                    "source": f"profiles/{src} (PMC)" if traffic else "algorithmic in + out bytes (no PMC pass)"},
            "note": "FIR Hilbert converter: per channel-sample nt odd taps, each a subtract + FMA; "
                    "frame-parallel (no recurrence), so it fills the chip"}


def measure_gpu(wname, streams, frames, steps, warmup, e2e_steps, dev, local_dev, dist, rank, world):
    """one workload on this rank's device: W untimed steps, then K steps between barriers +
    synchronize, max over ranks; the K1 roofline from the HIP-event timing of the timed steps"""
    import torch
    from in_cwave_amd import synth
    from in_cwave_amd import lib as L

    W = WORKLOADS[wname]
    S = streams or W["streams"]
    T = frames or W["frames"]
    fs = W["fs"]
    cfg, nodes, fmt = workload_config(W)
    ctx = L.Context(cfg, nodes, S, device=local_dev)
    if W.get("fir"):
        ctx.set_fir_hilbert(W["fir"], FIR_BETA)
    # synthetic input of the workload's shape for this rank's shard of streams (SURVEY 8(d)
    # generator): every stream its own seed (global stream index), generated by host threads
    first = rank * S
    gen = synth.batch_pcm(S, T, fs, channels=W["ch"], fmt=fmt, first=first,
                          workers=synth.cpu_workers())                      # uint8 [S, T*fsz]
    d_in = torch.from_numpy(gen).to(dev)
    osz = 2 * ctx.render_size
    d_out = torch.empty((S, T * osz), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    hip_stream = torch.cuda.current_stream(dev).cuda_stream

    def step(timing):
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, timing=timing, hip_stream=hip_stream)

    for _ in range(warmup):
        step(False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # per-launch kernel times from HIP events on the kernels' own streams, recorded in the LAST
    # timed step (the events cost ~12 us per launch block; the other steps run without them)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i == steps - 1)
    (k1_ms, k2_ms), (k1_n, k2_n) = ctx.last_timing()
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

    frames_total = float(S) * T * steps * world
    value = 2.0 * frames_total / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / steps

    # ---- end to end from host memory (H2D + D2H in the loop), one rank's view, not `value`
    e2e = None
    if e2e_steps > 0 and rank == 0:
        # pinned host buffers (icw_host_alloc): the call copies each launch block's slices in and
        # out on a copy stream beside the other blocks' kernels
        h_in = L.host_array((S, gen.shape[1]))
        h_in[:] = gen
        h_out = L.host_array((S, T * osz))
        ctx.process(h_in, T, out=h_out)                       # warm the staging buffers
        te = time.perf_counter()
        for _ in range(e2e_steps):
            ctx.process(h_in, T, out=h_out)
        te = time.perf_counter() - te
        del h_out, h_in
        e2e = {"value": 2.0 * S * T * e2e_steps / te / 1e6, "unit": "Msamples/s",
               "ms_per_step": te * 1e3 / e2e_steps, "steps": e2e_steps,
               "note": "host input and output in pinned memory (icw_host_alloc): H2D of each launch "
                       "block's input, the kernels and D2H of its output, the copies on a copy stream "
                       "beside the other blocks' kernels; one GPU"}

    if W.get("fir"):
        roof = fir_roofline(wname, W, S, T, k1_ms, k1_n, k2_ms, k2_n, os.environ.get("ICW_FIR_FUSED", "1") != "0")
        ctx.close()
        return {"value": value, "ms_per_step": ms_per_step, "roofline": roof, "e2e": e2e, "W": W, "S": S, "T": T,
                "fs": fs}

    # ---- roofline of the dominant kernel K1 (the serial recurrence), per launch, from HIP events
    # recorded on the stream K1 runs on (icw_last_timing)
    k1_kind = ctx.last_k1_kernel()
    k1_name = K1_KERNEL_NAME.get(k1_kind, "?")
    frames_per_launch = float(S) * T / max(1, k1_n)
    k1_avg_s = k1_ms / 1e3 / max(1, k1_n)
    k2_avg_s = k2_ms / 1e3 / max(1, k2_n)
    chains_per_stream = 2 if (W["ch"] == 1) else 4        # the mono dedup runs the left chains only
    flops_per_frame = chains_per_stream * 5 * IIR_ORDER   # loop-back Kahan sum: N x (1 mul + 4 add)
    achieved_tf = flops_per_frame * frames_per_launch / k1_avg_s / 1e12 if k1_avg_s > 0 else None
    hbm_gbs = W["bytes"] * frames_per_launch / k1_avg_s / 1e9 if k1_avg_s > 0 else None
    traffic, pmc_src = pmc_traffic(wname, k1_name, frames_per_launch)
    samples_per_chain = frames_per_launch / S
    sq = sq_model(wname, k1_name)
    if sq is not None:
        valu_wave, cpv, clock_ghz, sq_ns, sq_src = sq
        # the SQ pass's launches cover its own samples per chain: VALU per sample from its frames
        pmc_f = _latest(f"r*_{wname}_pmc.json")
        sq_frames = None
        try:
            sq_frames = float(json.loads(pmc_f.read_text())["frames_per_launch"]) if pmc_f else None
        except (ValueError, KeyError, OSError):
            pass
        valu = valu_wave / (sq_frames / S) if sq_frames else K1_VALU_PER_SAMPLE.get(k1_kind)
    else:
        valu, cpv, clock_ghz, sq_src = K1_VALU_PER_SAMPLE.get(k1_kind), CYC_PER_FP64_VALU, 2.32, None
    # the issue floor: the kernel's VALU per sample, each at the dependent FP64 add rate (the
    # recurrence is one dependent chain: ~74 of its ~75 VALU per sample are on it), at
    # the clock of the SQ pass; the SQ pass's own cycles per VALU is the kernel as profiled (frac ~1)
    cfl, cfl_src = fp64_issue_floor()
    floor_ms = (samples_per_chain * valu * cfl / (clock_ghz * 1e6)) if valu else None
    model_ms = (samples_per_chain * valu * cpv / (clock_ghz * 1e6)) if valu else None
    # the whole path's FP64 work over the step: every filter's Kahan IIR, per GPU
    chain_fpf = chain_flops_per_frame(W["ch"])
    chain_tf = chain_fpf * float(S) * T / (ms_per_step / 1e3) / 1e12
    roof = {
        "bound": "fp64", "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": (achieved_tf / FP64_PEAK_TFLOPS) if achieved_tf else None, "traffic": traffic,
        "kernel": k1_name, "flops_per_frame": flops_per_frame, "frames_per_launch": frames_per_launch,
        "avg_launch_ms": k1_avg_s * 1e3, "output_kernel_avg_launch_ms": k2_avg_s * 1e3,
        "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (hbm_gbs / HBM_PEAK_GBS) if hbm_gbs else None,
                "alg_bytes_per_frame": W["bytes"], "traffic_source": f"profiles/{pmc_src}" if traffic else None},
        "chain_fp64": {"flops_per_frame": chain_fpf, "achieved": chain_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": chain_tf / FP64_PEAK_TFLOPS,
                       "note": "SURVEY 8(d): the Kahan IIR of every filter (15N - 4 flops per filter-sample, "
                               "hblpf.c:1017-1056), per GPU, over ms_per_step"},
        "issue_bound": {"valu_per_sample": valu, "cycles_per_valu_floor": cfl, "clock_ghz": clock_ghz,
                        "floor_ms_per_launch": floor_ms,
                        "frac": (floor_ms / (k1_avg_s * 1e3)) if (k1_avg_s and floor_ms) else None,
                        "floor_source": f"profiles/{cfl_src}" if cfl_src else "constant",
                        "sq_source": f"profiles/{sq_src}" if sq_src else "round-2 constants",
                        "sq_cycles_per_valu": cpv, "sq_model_ms_per_launch": model_ms,
                        "note": "floor = VALU per sample (SQ pass) x cycles per dependent FP64 add (a v_add_f64 "
                                "chain on one wave, latency probe) / the SQ pass's clock; frac = floor / this "
                                "run's launch time.  sq_model = the same VALU at the SQ pass's own cycles per "
                                "VALU (the kernel as profiled: ~1 x the launch time)"},
        "note": f"serial IIR recurrence: {chains_per_stream * S} DF-II chains per GPU, each a dependent "
                f"chain of ~{4 * IIR_ORDER} FP64 ops per sample ({'one 16-lane DPP row' if k1_kind == 3 else 'one lane'}"
                f" per chain); `frac` is the algorithmic FP64 rate (5N = {5 * IIR_ORDER} flops per chain-sample) "
                f"against the FP64 vector peak, small because {chains_per_stream * S} chains cannot fill "
                f"1024 SIMDs (DESIGN.md 5)",
    }

    ctx.close()
    return {"value": value, "ms_per_step": ms_per_step, "roofline": roof, "e2e": e2e, "W": W, "S": S, "T": T,
            "fs": fs}


def control_backend(ndev, world):
    """torch.distributed backend of the bench's control plane: the barriers and the one-scalar
    max-reduce of the elapsed time.  The data path has no collective (north_star: streams are
    sharded, nothing is exchanged), so the timing needs no RCCL; gloo on the host is the default
    whatever the device count -- the code the 8-GPU run executes is the code the 2-rank tests run.
    ICW_BENCH_BACKEND=nccl opts into RCCL, which needs one device per rank."""
    b = os.environ.get("ICW_BENCH_BACKEND", "gloo")
    if b not in ("gloo", "nccl"):
        raise SystemExit(f"bench.py: ICW_BENCH_BACKEND={b!r} (gloo | nccl)")
    if b == "nccl" and ndev < world:
        b = "gloo"          # ranks sharing a device (the 1-GPU rehearsal) cannot use RCCL
    return b


def main():
    a = parse()
    if a.workload == "c1":
        if a.gpus != 1:
            raise SystemExit("bench.py c1 is the single-stream drop-in: --gpus 1")
        return bench_c1(a)
    if "RANK" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    ndev = torch.cuda.device_count()          # counts without initialising the GPU
    dist = None
    local_dev = local % max(1, ndev)
    backend = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = control_backend(ndev, world)
        torch.cuda.set_device(local_dev)
        dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", local_dev)
    torch.cuda.set_device(dev)

    r = measure_gpu(a.workload, a.streams, a.frames, a.steps, a.warmup, a.e2e_steps, dev, local_dev, dist, rank,
                    world)
    W, S, T, fs = r["W"], r["S"], r["T"], r["fs"]
    value, ms_per_step, roof, e2e = r["value"], r["ms_per_step"], r["roofline"], r["e2e"]

    # ---- the other BASELINE configs, measured in the same run: short runs of the same harness,
    # reported beside the headline, never in `value`.  N = 1: C3 / C4 / C5 and their FIR forms, and
    # the C1 drop-in.  N > 1: the configs BASELINE.json quotes "sharded across 8xMI355X" -- C4 and
    # C5 (and their 255 / 1023-tap FIR forms) at their per-GPU shard sizes (2 048 / 256 streams per
    # rank: 16 384 / 2 048 at N = 8), timed like the headline (barriers, max over ranks), whole-job
    others = None
    want_others = a.workload == "c2" and not a.no_other_workloads and (
        world > 1 or (not a.no_cpu_baseline and a.streams is None and a.frames is None))
    if want_others:
        others = {}
        import gc
        default = "c4,c5,c4fir,c5fir" if world > 1 else "c3,c4,c5,c2fir,c3fir,c4fir,c5fir"
        for w in os.environ.get("ICW_BENCH_OTHERS_MULTI" if world > 1 else "ICW_BENCH_OTHERS", default).split(","):
            gc.collect()
            torch.cuda.empty_cache()
            # 3 timed steps after 2 warm-up steps: a leg follows a different workload (round 5's mid-round
            # default run read c2fir 136 k where --workload c2fir runs read 142-146 k)
            o = measure_gpu(w, None, a.other_frames, 3, 2, 0, dev, local_dev, dist, rank, world)
            ro = o["roofline"]
            others[w] = {"value": o["value"], "unit": "Msamples/s", "ms_per_step": o["ms_per_step"], "steps": 3,
                         "warmup": 2, "n_gpus": world, "workload": o["W"]["desc"], "streams_per_gpu": o["S"],
                         "streams_total": o["S"] * world, "frames_per_stream_per_step": o["T"],
                         "k1_kernel": ro["kernel"], "k1_avg_launch_ms": ro["avg_launch_ms"],
                         "k2_avg_launch_ms": ro["output_kernel_avg_launch_ms"], "fp64_frac": ro["frac"]}
            if "chain_fp64" in ro:
                others[w]["chain_fp64_frac"] = ro["chain_fp64"]["frac"]
            if o["W"].get("fir"):
                others[w].update({"fir_kernel_avg_launch_ms": ro["avg_launch_ms"], "fir_tflops": ro["achieved"],
                                  "fir_hbm_gbs": ro["hbm"]["achieved"], "fir_hbm_source": ro["hbm"]["source"]})
                for k in ("k1_kernel", "k1_avg_launch_ms"):
                    others[w].pop(k)
        if world == 1:
            try:
                c1 = measure_c1(1, 1, 576, True)
                others["c1"] = {k: c1[k] for k in ("value", "unit", "ms_per_step", "block_latency_us", "realtime_x",
                                                   "parity_vs_oracle", "cpu_baseline")}
                others["c1"]["workload"] = c1["config"]["workload"]
            except (SystemExit, Exception) as e:      # reported, never silently replaced
                others["c1"] = {"error": repr(e)}

    # ---- the CPU baseline: at N = 1 only (the task's contract), after the GPU legs (never beside GPU
    # timing); a multi-GPU line carries null
    if dist:
        torch.cuda.synchronize()
        dist.barrier()
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.cpu_workers, a.cpu_frames, a.workload)
        except Exception as e:  # reported, never silently replaced
            cpu = {"error": repr(e)}
    if dist:
        dist.barrier()

    if rank == 0:
        line = {
            "metric": "Msamples/s through Hilbert+mod+render",
            "value": value, "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "input_mframes_per_s": value / 2.0,             # input frames/s beside the metric
            "dtype": "f64", "data": "synthetic, every stream its own generated input (SURVEY 8(d) generator)",
            "config": {"workload": W["desc"],
                       "streams_per_gpu": S, "frames_per_stream_per_step": T, "fs": fs,
                       "parallelism": f"stream-shard x{world}",
                       "control_backend": backend},
            "roofline": roof,
            "e2e_host_buffers": e2e,
            "cpu_baseline": cpu,
            "other_workloads": others,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
