#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs (all passes under a dir) per kernel: mean per dispatch."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = ("spmm_window" if "spmm_win_kernel" in k else "spmm_bcast" if "spmm_vec_kernel" in k else "spmm_tiled" if "spmm3_tiled" in k
                 else "dense" if "dense_kernel" in k else None)
        if short is None:
            continue
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(f"{d}/*/*kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = ("spmm_window" if "spmm_win_kernel" in k else "spmm_bcast" if "spmm_vec_kernel" in k else "spmm_tiled" if "spmm3_tiled" in k
                 else "dense" if "dense_kernel" in k else None)
        if short:
            dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in vals.items():
    print(f"== {k}  (profiled dispatch avg {sum(dur[k]) / max(1, len(dur[k])):.1f} us)")
    for c, v in sorted(cs.items()):
        print(f"   {c:34s} {sum(v) / len(v):16.1f}")
