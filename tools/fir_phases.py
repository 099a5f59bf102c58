#!/usr/bin/env python3
"""KF2 (icw_fir_graph) phase times from the diagnostic stamps of a build with -DICW_FIR_STAMPS=1
(ICW_LIB=<that build>.so python tools/fir_phases.py [workload ...]).  One launch block (65 536
frames) of the workload's streams; per workgroup wave 0 stamps the shader clock after the prologue,
the staging, the barrier, the sums, the graph + stores and the meters, and the 100 MHz clock at its
start and end.  Prints one JSON line per workload: mean / p50 cycles per phase, the workgroup
lifetime, the launch span and the mean number of workgroups resident (sum of lifetimes / span)."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

PHASES = ["stage", "barrier", "sums", "graph_store", "meters"]


def run(name, frames=1 << 16):
    import torch
    import bench
    from in_cwave_amd import lib as L, synth
    W = bench.WORKLOADS[name]
    cfg, nodes, fmt = bench.workload_config(W)
    S = W["streams"]
    ctx = L.Context(cfg, nodes, S, device=0)
    ctx.set_fir_hilbert(W["fir"], bench.FIR_BETA)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(synth.batch_pcm(S, frames, W["fs"], channels=W["ch"], fmt=fmt,
                                            workers=synth.cpu_workers())).to(dev)
    d_out = torch.empty((S, frames * 2 * ctx.render_size), dtype=torch.uint8, device=dev)
    for _ in range(3):
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), frames)
    torch.cuda.synchronize()
    lib = L.load()
    tf = 1024 if W["ch"] == 2 else 2048
    n_wg = min(S * ((frames + tf - 1) // tf), 1 << 16)     # the stamp array holds the first 65 536 workgroups
    buf = np.zeros(n_wg * 8, dtype=np.uint64)
    lib.icw_fir_stamps_read.argtypes = [C.c_void_p, C.c_size_t]
    if lib.icw_fir_stamps_read(buf.ctypes.data, buf.size) != 0:
        raise SystemExit("icw_fir_stamps_read failed (not a -DICW_FIR_STAMPS=1 build?)")
    st = buf.reshape(n_wg, 8).astype(np.int64)
    ctx.close()
    d = np.diff(st[:, 1:7], axis=1)                      # shader cycles per phase
    rt0, rt1 = st[:, 0], st[:, 7]
    life = (rt1 - rt0) * 10.0                            # ns (100 MHz)
    span = (rt1.max() - rt0.min()) * 10.0
    out = {"workload": name, "workgroups": n_wg, "span_us": span / 1e3,
           "wg_life_us": {"mean": float(life.mean() / 1e3), "p50": float(np.median(life) / 1e3)},
           "resident_mean": float(life.sum() / span),
           "cycles": {p: {"mean": float(d[:, i].mean()), "p50": float(np.median(d[:, i]))} for i, p in enumerate(PHASES)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for w in sys.argv[1:] or ["c2fir", "c4fir", "c3fir"]:
        run(w)
