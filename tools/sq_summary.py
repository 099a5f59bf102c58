#!/usr/bin/env python3
"""Summarise one rocprofv3 --pmc pass of SQ counters into profiles/<name>.json: per kernel, the
per-dispatch average of every counter, and -- given the kernel-trace stats of the same workload --
the effective engine clock SQ_BUSY_CYCLES / 32 shader engines / average launch time, VALU
instructions per wave and cycles per VALU.

    python tools/sq_summary.py gpurun_out/pmc_c4_SQ_WAVES gpurun_out/prof_c4 profiles/r02_c4_sq.json --note "..."
"""
import argparse
import collections
import csv
import json
from pathlib import Path

KERNELS = ("icw_fir_hilbert", "icw_fir_graph", "icw_fir_sig", "icw_unpack_frames", "icw_iir_state", "icw_iir_row", "icw_output", "icw_trig_table", "icw_dither_coop", "icw_dith_twist", "icw_dith_samples", "icw_dith_fix",
           "icw_render_serial", "icw_render_row", "icw_graph_serial")
N_SE = 32          # shader engines whose busy cycles SQ_BUSY_CYCLES sums (MI355X: 8 XCDs x 4)


def counters(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(x in k for x in KERNELS):
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in tot.items()}


def stats(d):
    out = {}
    for f in Path(d).rglob("*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            out[r["Name"]] = float(r["AverageNs"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("stats_dir")
    ap.add_argument("out")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    cs, st = counters(a.pmc_dir), stats(a.stats_dir)
    res = {}
    for k, c in sorted(cs.items()):
        e = dict(c)
        ns = st.get(k)
        if ns:
            e["avg_launch_ns_trace"] = ns
            if "SQ_BUSY_CYCLES" in c:
                e["effective_clock_ghz"] = c["SQ_BUSY_CYCLES"] / N_SE / ns
        if c.get("SQ_WAVES"):
            e["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_WAVES"]
        res[k] = e
    Path(a.out).write_text(json.dumps({"note": a.note, "kernels": res}, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
