#!/usr/bin/env python3
"""K2 cost of the DSP program: the C4 shape (2048 x 48 kHz int16 stereo streams, 16 384-frame
launches) with the graph swapped -- Master only, Shift -> Master, PM -> Shift -> Mix -> Master --
timed with the per-launch HIP events (icw_last_timing).  ICW_SERIALIZE=1 gives standalone kernel
times.  Prints one line per graph."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from in_cwave_amd import graph, synth  # noqa: E402
from in_cwave_amd import lib as L  # noqa: E402


def main():
    W = dict(bench.WORKLOADS["c4"])
    S, T, fs = W["streams"], 1 << 16, W["fs"]
    dev = torch.device("cuda", 0)
    gen = synth.batch_pcm(16, T, fs)
    d_in = torch.empty((S, gen.shape[1]), dtype=torch.uint8, device=dev)
    g = torch.from_numpy(gen).to(dev)
    for s in range(S):
        d_in[s].copy_(g[s % 16])
    d_out = torch.empty((S, T * 4), dtype=torch.uint8, device=dev)
    hs = torch.cuda.current_stream(dev).cuda_stream
    for name in ("master_only", "shift_master", "pm_shift_mix"):
        W["graph"] = name
        cfg, nodes, fmt = bench.workload_config(W)
        ctx = L.Context(cfg, nodes, S, device=0)
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, hip_stream=hs)
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, timing=True, hip_stream=hs)
        (k1, k2), (n1, n2) = ctx.last_timing()
        print(f"{name:14s} K1 {k1 / n1:.3f} ms  K2 {k2 / n2:.3f} ms per launch ({n1} launches)", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
