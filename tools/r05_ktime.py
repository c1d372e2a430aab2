#!/usr/bin/env python3
"""Median duration (us) per kernel-name substring from a rocprofv3 kernel_trace.csv, split into the small and
large launches of each name (the F = 128 and F = 256 cases of tools/r05_dgrad_time.py):
  tools/r05_ktime.py <dir> <substring> [...]"""
import collections
import csv
import glob
import statistics as st
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for key in sys.argv[2:]:
        if key in r["Kernel_Name"]:
            d[key].append(t)
for k, v in d.items():
    lo = [x for x in v if x < min(v) * 2]
    hi = [x for x in v if x >= min(v) * 2]
    print(k, "small", round(st.median(lo), 1), len(lo), "large", round(st.median(hi), 1) if hi else None, len(hi))
