#!/usr/bin/env python3
"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/<name>.json.

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_c2_pmc.json \
        --frames-per-launch 4194304 --note "..."

Per kernel: KB per dispatch averaged over dispatches, and the HBM bytes per launch with the gfx950
correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of 16-B/lane
streaming reads, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact.
"""
import argparse
import collections
import csv
import json
from pathlib import Path

KERNELS = ("icw_fir_hilbert", "icw_fir_graph", "icw_fir_sig", "icw_unpack_frames", "icw_iir_state", "icw_iir_row", "icw_output", "icw_trig_table", "icw_dither_coop", "icw_dith_twist", "icw_dith_samples", "icw_dith_fix",
           "icw_render_serial", "icw_render_row")


def per_dispatch(d, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            if not any(x in k for x in KERNELS):
                continue
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--frames-per-launch", type=int, required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    fe = per_dispatch(a.fetch_dir, "FETCH_SIZE")
    wr = per_dispatch(a.write_dir, "WRITE_SIZE")
    ks = {}
    for k in sorted(set(fe) | set(wr)):
        f, w = fe.get(k, 0.0), wr.get(k, 0.0)
        ks[k] = {"FETCH_SIZE_KB": f, "WRITE_SIZE_KB": w, "hbm_bytes_corrected": 2.0 * f * 1024 + w * 1024}
    Path(a.out).write_text(json.dumps({"note": a.note, "frames_per_launch": a.frames_per_launch, "kernels": ks},
                                      indent=1) + "\n")
    print(json.dumps(ks, indent=1))


if __name__ == "__main__":
    main()
