#!/usr/bin/env python3
"""A/B: ms per step of one workload with and without the per-launch timing events (icw flag 4),
same harness as bench.py's measure_gpu, alternating 3 rounds of K steps each."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from in_cwave_amd import lib as L  # noqa: E402
from in_cwave_amd import synth  # noqa: E402


def main(wname, steps=3):
    W = bench.WORKLOADS[wname]
    S, T, fs = W["streams"], W["frames"], W["fs"]
    cfg, nodes, fmt = bench.workload_config(W)
    dev = torch.device("cuda", 0)
    ctx = L.Context(cfg, nodes, S, device=0)
    gen = synth.batch_pcm(min(S, 16), T, fs, channels=W["ch"], fmt=fmt)
    d_in = torch.empty((S, gen.shape[1]), dtype=torch.uint8, device=dev)
    g = torch.from_numpy(gen).to(dev)
    for s in range(S):
        d_in[s].copy_(g[s % g.shape[0]])
    d_out = torch.empty((S, T * 2 * ctx.render_size), dtype=torch.uint8, device=dev)
    hs = torch.cuda.current_stream(dev).cuda_stream

    def run(timing):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T, timing=timing, hip_stream=hs)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    run(False)
    for r in range(3):
        a, b = run(True), run(False)
        print(f"{wname} round {r}: timing {a:.3f} ms/step, no timing {b:.3f} ms/step", flush=True)
    ctx.close()


if __name__ == "__main__":
    for w in sys.argv[1:]:
        main(w)
