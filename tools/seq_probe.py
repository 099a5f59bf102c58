#!/usr/bin/env python3
"""Run bench.py workloads back to back in one process (A/B of in-process interference):
    python tools/seq_probe.py c3,c2,c3 [steps]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402

seq = sys.argv[1].split(",")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for w in seq:
    o = bench.measure_gpu(w, None, None, steps, 1, 0, dev, 0, None, 0, 1)
    r = o["roofline"]
    print(json.dumps({"workload": w, "value": round(o["value"], 1), "ms_per_step": round(o["ms_per_step"], 2),
                      "k1": r["kernel"], "k1_ms": round(r["avg_launch_ms"], 3),
                      "k2_ms": round(r["output_kernel_avg_launch_ms"], 3)}), flush=True)
