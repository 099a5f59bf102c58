#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace of one bench workload (tools/trace_wl.sh): the call of each
bench step is one K1 (icw_iir_*) sequence, steps are split at K1 gaps > 0.5 ms.  Per step: the K1
launches' busy time (sum K1), the gaps between consecutive K1s, the fill (the step's first kernel ->
its first K1), the drain (its last K1 end -> its last kernel end) and the span (first kernel -> last
kernel); ratio = span / sum K1.  -v lists every K1."""
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
    k1 = [r for r in rows if "icw_iir_" in r[2]]
    steps, cur = [], [k1[0]]
    for r in k1[1:]:
        if r[0] - cur[-1][1] > 500_000:
            steps.append(cur)
            cur = []
        cur.append(r)
    steps.append(cur)
    bounds = [s[0][0] for s in steps] + [rows[-1][1] + 1]
    prev_end = rows[0][0] - 1
    for i, g in enumerate(steps):
        t0, t1 = g[0][0], g[-1][1]
        # the step's kernels: after the previous step's last K1, before the next step's first K1
        lo = steps[i - 1][-1][1] if i else rows[0][0] - 1
        ks = [r for r in rows if r[0] > lo and r[0] < bounds[i + 1]]
        ks_before = [r for r in ks if r[0] < t0 and r[0] > prev_end]
        first = min([r[0] for r in ks if r[0] >= (ks_before[0][0] if ks_before else t0)] + [t0])
        # drain: kernels that start after the last K1 began and before the next step's first kernel
        nxt = bounds[i + 1]
        after = [r for r in rows if r[0] >= g[-1][0] and r[0] < nxt and "icw_unpack" not in r[2] or
                 (r[0] >= t1 and r[0] < nxt and "icw_advance" in r[2])]
        last = max([r[1] for r in after if r[0] < nxt] + [t1])
        busy = sum(r[1] - r[0] for r in g)
        gaps = [g[j + 1][0] - g[j][1] for j in range(len(g) - 1)]
        fill = (t0 - first) / 1e6
        drain = (last - t1) / 1e6
        span = (last - first) / 1e6
        prev_end = last
        print(f"step {i}: K1 x{len(g)} sum {busy / 1e6:.3f} ms, gaps {sum(gaps) / 1e6:.3f} ms "
              f"(mean {sum(gaps) / max(1, len(gaps)) / 1e3:.1f} us), fill {fill:.3f} ms, drain {drain:.3f} ms, "
              f"span {span:.3f} ms, span / sum K1 = {span / (busy / 1e6):.4f}")
        if "-v" in sys.argv:
            for j, r in enumerate(g):
                print(f"   K1[{j}] {(r[0] - t0) / 1e6:8.3f} .. {(r[1] - t0) / 1e6:8.3f}  ({(r[1] - r[0]) / 1e6:.3f})")


if __name__ == "__main__":
    main(sys.argv[1])
