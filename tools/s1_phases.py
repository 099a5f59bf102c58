#!/usr/bin/env python3
"""K5 (icw_stream1) phase times from the diagnostic stamps (ICW_S1_STAMPS=1, one stderr line per
call: frames, then per phase the shader-clock cycles and the 100 MHz ticks of K0, K1r, K2): median
microseconds per phase and the shader clock the recurrence ran at."""
import statistics
import sys


def main(path):
    rows = []
    for line in open(path):
        p = line.split()
        if p and p[0] == "icw_s1":
            rows.append([int(x) for x in p[1:]])
    rows = rows[len(rows) // 10:]              # skip the warm-up calls
    for n in sorted({r[0] for r in rows}):
        rr = [r for r in rows if r[0] == n]
        out = {"frames": n, "calls": len(rr)}
        for k, name in enumerate(("k0", "k1r", "k2")):
            cyc = statistics.median(r[1 + 2 * k] for r in rr)
            us = statistics.median(r[2 + 2 * k] for r in rr) / 100.0
            out[name + "_us"] = round(us, 2)
            out[name + "_ghz"] = round(cyc / (us * 1e3), 3) if us > 0 else None
        out["k1r_ns_per_sample"] = round(out["k1r_us"] * 1e3 / n, 1)
        print(out)


if __name__ == "__main__":
    main(sys.argv[1])
