#!/usr/bin/env python3
"""Per-kernel summary (the columns of rocprofv3 --stats' kernel_stats.csv) from a rocprofv3 --kernel-trace database
(rocpd SQLite, ROCm 7's default output format): Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs.
usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_bench_kernel_stats.csv"""
import csv
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                  "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
dur = defaultdict(list)
for name, t0, t1 in rows:
    dur[name].append(t1 - t0)
total = sum(sum(v) for v in dur.values())
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / total, 2), min(v), max(v)])
