#!/usr/bin/env python3
"""Two C3-shaped contexts (R: re-create A on its buffers, F: free B) alive at once, stepped alternately: does a context's K1 speed depend on
creation order / allocation history?   python tools/ctx_probe.py [order e.g. ABAB] [free_first]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
from in_cwave_amd import lib as L, synth  # noqa: E402

order = sys.argv[1] if len(sys.argv) > 1 else "ABAB"
W = bench.WORKLOADS["c3"]
S, T = W["streams"], W["frames"]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cfg, nodes, fmt = bench.workload_config(W)
gen = synth.batch_pcm(16, T, W["fs"], channels=W["ch"], fmt=fmt)
g = torch.from_numpy(gen).to(dev)
bufs = {}
for name in "AB":
    ctx = L.Context(cfg, nodes, S, device=0)
    d_in = torch.empty((S, gen.shape[1]), dtype=torch.uint8, device=dev)
    for s in range(S):
        d_in[s].copy_(g[s % 16])
    d_out = torch.empty((S, T * 4), dtype=torch.uint8, device=dev)
    bufs[name] = (ctx, d_in, d_out)
torch.cuda.synchronize()
hs = torch.cuda.current_stream(dev).cuda_stream
for name in order:
    if name == "R":          # close context A and create a fresh one on the same torch buffers
        _, d_in, d_out = bufs["A"]
        bufs["A"][0].close()
        bufs["A"] = (L.Context(cfg, nodes, S, device=0), d_in, d_out)
        name = "A"
    if name == "N":          # a new context C on B's buffers (allocated now)
        if "C" not in bufs:
            bufs["C"] = (L.Context(cfg, nodes, S, device=0), bufs["A"][1], bufs["A"][2])
        name = "C"
    if name == "F":          # free B's torch buffers and context entirely
        bufs["B"][0].close()
        bufs.pop("B")
        torch.cuda.empty_cache()
        continue
    ctx, d_in, d_out = bufs[name]
    ms = []
    for _ in range(2):
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, timing=True, hip_stream=hs)
        (m1, m2), (n1, n2) = ctx.last_timing()
        ms.append(round(m1 / n1, 3))
    print(json.dumps({"ctx": name, "k1_ms_per_launch": ms}), flush=True)
