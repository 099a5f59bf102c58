#!/usr/bin/env python3
"""Throughput of the GPU CRC-32 (icw_crc32_cells) over data resident in HBM: one range of
--gib GiB, or --ranges equal ranges covering it (a batch of CWAVE data parts).  Prints wall-clock
GB/s per call; the kernel's own duration comes from rocprofv3 --kernel-trace --stats
(profiles/r01_crc_kernel_stats.csv)."""
import argparse
import json
import sys
import time
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--ranges", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch
    from in_cwave_amd import lib as L
    n = int(a.gib * (1 << 30))
    dev = torch.empty(n // 8, dtype=torch.int64, device="cuda").random_().view(torch.uint8)
    per = n // a.ranges
    offs = [i * per for i in range(a.ranges)]
    lens = [per] * a.ranges
    L.crc32_batch(dev, offs, lens, device_ptrs=True)         # warm-up (tables, code objects)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        got = L.crc32_batch(dev, offs, lens, device_ptrs=True)
        ts.append(time.perf_counter() - t0)
    chk = dev[:1 << 24].cpu().numpy().tobytes()
    ok = L.crc32_batch(dev, [0], [1 << 24], device_ptrs=True)[0] == zlib.crc32(chk)
    best = min(ts)
    print(json.dumps({"bytes": n, "ranges": a.ranges, "best_wall_s": best, "wall_GBps": n / best / 1e9,
                      "zlib_check_16MiB": ok, "crc0": got[0]}))


if __name__ == "__main__":
    main()
