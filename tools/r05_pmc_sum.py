#!/usr/bin/env python3
"""Average per-dispatch PMC counter values of the kernels whose names contain a substring, from rocprofv3
counter_collection.csv files: tools/r05_pmc_sum.py <dir> <substring> [<substring> ...]"""
import csv
import glob
import sys
from collections import defaultdict

files = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
for sub in sys.argv[2:]:
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(sub, {k: round(sum(v) / len(v)) for k, v in sorted(vals.items())}, "dispatch-counter rows", sum(map(len, vals.values())))
