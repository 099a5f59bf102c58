#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (tools/trace_wl.sh): per bench step, the K1 launches' busy
time, the gaps between consecutive K1s, the fill (first kernel -> first K1) and the drain (last K1
end -> last kernel end)."""
import csv
import glob
import sys


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # steps: split where the K1 sequence has a gap of > 5 ms (host work between steps)
    k1 = [r for r in rows if "icw_iir_" in r[2]]
    groups, cur = [], [k1[0]]
    for r in k1[1:]:
        if r[0] - cur[-1][1] > 5_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    for g in groups:
        t0, t1 = g[0][0], g[-1][1]
        ks = [r for r in rows if t0 - 20_000_000 < r[0] and r[1] < t1 + 20_000_000]
        # the step's kernels: between the previous K1 group and the next one
        busy = sum(r[1] - r[0] for r in g)
        gaps = [g[i + 1][0] - g[i][1] for i in range(len(g) - 1)]
        pre = [r for r in ks if r[1] <= t0 and r[0] > t0 - 5_000_000]
        post = [r for r in ks if r[0] >= t1 - 1 and r[0] < t1 + 5_000_000]
        fill = (t0 - min(r[0] for r in pre)) / 1e6 if pre else 0.0
        drain = (max(r[1] for r in post) - t1) / 1e6 if post else 0.0
        print(f"K1 x{len(g)}: span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f}, gaps sum {sum(gaps) / 1e6:.3f} "
              f"max {max(gaps or [0]) / 1e6:.3f}; fill {fill:.3f} ms; drain {drain:.3f} ms")
        if "-v" in sys.argv:
            for i, r in enumerate(g):
                print(f"   K1[{i}] {(r[0] - t0) / 1e6:8.3f} .. {(r[1] - t0) / 1e6:8.3f}  ({(r[1] - r[0]) / 1e6:.3f})")
            for r in ks:
                if "icw_iir_" not in r[2]:
                    print(f"   {r[2][:40]:40s} {(r[0] - t0) / 1e6:8.3f} .. {(r[1] - t0) / 1e6:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
