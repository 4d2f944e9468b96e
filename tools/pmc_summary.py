#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc_engine.sh per kernel.

usage: python tools/pmc_summary.py OUTDIR [--json OUT.json --dims MX,MY,MZ [--fp16]]
(OUTDIR holds p1/ .. p4/; the JSON feeds bench.py's roofline.traffic)

Per kernel (averaged over its dispatches): duration, HBM traffic per launch
(FETCH_SIZE x 2 + WRITE_SIZE, in KB units per rocprofv3; FETCH_SIZE counts
half the bytes of wide coalesced reads on gfx950 -- MI355X_MICROARCH.md), the
derived GB/s, and the SQ counters of passes 1-2.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+<[^>]*>)", name)
    return m.group(1) if m else name[:60]


def main(out, json_out=None, dims=None, fp16=False):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, "p*", "*_counter_collection.csv"))):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    avg = lambda xs: sum(xs) / len(xs) if xs else float("nan")
    cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"]
    cols += [c for c in ("SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU")
             if any(c in v for v in vals.values())]
    print("| kernel | us (avg) | HBM MB/launch (2*FETCH+WRITE) | GB/s | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * (3 + len(cols)))
    table = {}
    for k in sorted(vals):
        v = vals[k]
        fetch = avg(v.get("FETCH_SIZE", []))
        write = avg(v.get("WRITE_SIZE", []))
        t = avg(dur[k])
        traffic = (2 * fetch + write) * 1024
        row = [k, f"{t * 1e6:.1f}", f"{traffic / 1e6:.1f}", f"{traffic / t / 1e9:.0f}"]
        row += [f"{avg(v.get(c, [])):.3g}" for c in cols]
        print("| " + " | ".join(row) + " |")
        med = lambda xs: sorted(xs)[len(xs) // 2] if xs else float("nan")
        # median launch: a kernel name can also cover short launches (the y pass of the
        # compact kernel spectra, 2kc+1 planes) that pull the mean below a data pass
        tmed = (2 * med(v.get("FETCH_SIZE", [])) + med(v.get("WRITE_SIZE", []))) * 1024
        table[k] = {"avg_us": round(t * 1e6, 2), "hbm_bytes_per_launch": int(traffic),
                    "hbm_bytes_per_launch_median": int(tmed),
                    "fetch_kb_x2": 2 * fetch, "write_kb": write}
    if json_out:
        import json
        with open(json_out, "w") as f:
            json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                 "tools/pmc_engine.sh; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                                 "(gfx950 FETCH_SIZE counts half of wide reads)",
                       "file": os.path.relpath(json_out, os.path.dirname(os.path.dirname(
                           os.path.abspath(__file__)))),
                       "fft_dims": dims, "fp16": fp16, "kernels": table}, f, indent=1)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--json")
    ap.add_argument("--dims", default="540,540,540")
    ap.add_argument("--fp16", action="store_true")
    a = ap.parse_args()
    main(a.outdir, a.json, [int(x) for x in a.dims.split(",")], a.fp16)
