#!/usr/bin/env python3
"""Time the oracle restatement (oracle/icw_oracle.c, gcc -O2 -ffp-contract=off) on one core of this
machine on the survey's probe workloads, to relate bench.py's cpu_baseline (the same restatement on
the GPU box's cores) to the reference's own speed, which SURVEY.md / BASELINE.md measured on this
container's CPU type with the reference C (1 core: C1 2.89, C2 2.82, C3 3.44, C4 2.21, C5 2.96
Msamples/s).  Prints one JSON line.

    python tools/cpu_calibrate.py [--frames 1048576]
"""
import argparse
import json
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from in_cwave_amd import abi, graph, synth      # noqa: E402
from oracle import oracle as O                   # noqa: E402

REF = {"c1": 2.89, "c2": 2.82, "c3": 3.44, "c4": 2.21, "c5": 2.96}   # BASELINE.md, reference C, 1 core


def shape(w):
    if w == "c1":
        return graph.default_config(44100), graph.graph_shift_master(), 2
    if w == "c2":
        return graph.default_config(48000), graph.graph_shift_master(), 2
    if w == "c3":
        return graph.default_config(96000, channels=1), graph.graph_master_only(), 1
    if w == "c4":
        return graph.default_config(48000), graph.graph_pm_shift_mix(), 2
    cfg = graph.default_config(192000, fmt=abi.FMT_F32, need24bits=True)
    cfg.render.render_type, cfg.render.nshape_type = abi.RENDER_TPDF, abi.NSHAPE_MEW44
    return cfg, graph.graph_master_only(), 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    args = ap.parse_args()
    O.build()
    cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")),
               platform.processor())
    res = {}
    for w in ("c1", "c2", "c3", "c4", "c5"):
        cfg, nodes, ch = shape(w)
        raw = synth.batch_pcm(1, args.frames, cfg.sample_rate, channels=ch, fmt=cfg.in_format, first=9)[0]
        st = O.Stream(cfg, nodes)
        t = time.perf_counter()
        st.process(raw, args.frames)
        dt = time.perf_counter() - t
        ms = 2 * args.frames / dt / 1e6          # rendered channel-samples (output is always stereo)
        res[w] = {"oracle_msamples_s": round(ms, 3), "reference_msamples_s": REF[w],
                  "oracle_over_reference": round(ms / REF[w], 3)}
    print(json.dumps({"cpu": cpu, "frames": args.frames, "cores": 1, "workloads": res}))


if __name__ == "__main__":
    main()
