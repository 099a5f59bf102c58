#!/usr/bin/env python3
"""Cost split of the fused FIR kernel KF2 by variation: one launch block (T frames) of S streams
through the FIR converter for several orders (order 2 = one odd tap: the staging, graph and render
with almost no sums) and graphs.  Prints one JSON line per case: ms per call (HIP events around
the device-pointer call, median of K calls).

    python tools/fir_probe.py [--streams 256] [--frames 65536] [--calls 7]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from in_cwave_amd import abi, graph
from in_cwave_amd import lib as L

GRAPHS = {"master": graph.graph_master_only, "shift_master": graph.graph_shift_master,
          "pm_shift_mix": graph.graph_pm_shift_mix}


def run(S, T, ch, order, gname, calls):
    cfg = graph.default_config(48000, fmt=abi.FMT_I16, channels=ch)
    ctx = L.Context(cfg, GRAPHS[gname](), S)
    ctx.set_fir_hilbert(order, 8.0)
    g = torch.Generator(device="cpu").manual_seed(7)
    raw = torch.randint(0, 256, (S, T * 2 * ch), dtype=torch.uint8, generator=g)
    d_in = raw.cuda()
    d_out = torch.zeros((S, T * 4), dtype=torch.uint8, device="cuda")
    ms = []
    for k in range(calls + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T)
        e1.record()
        torch.cuda.synchronize()
        if k >= 2:
            ms.append(e0.elapsed_time(e1))
    ctx.close()
    med = statistics.median(ms)
    return {"streams": S, "frames": T, "ch": ch, "order": order, "graph": gname, "ms": round(med, 4),
            "msamples_per_s": round(S * T * ch / med / 1e3, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--calls", type=int, default=7)
    ap.add_argument("--cases", default="2:master,2:shift_master,254:master,254:shift_master,254:pm_shift_mix,30:shift_master")
    a = ap.parse_args()
    for ch in (2, 1):
        for case in a.cases.split(","):
            o, gname = case.split(":")
            print(json.dumps(run(a.streams, a.frames, ch, int(o), gname, a.calls)), flush=True)


if __name__ == "__main__":
    main()
