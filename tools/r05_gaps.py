#!/usr/bin/env python3
"""Per-step kernel timeline of a bench run from a rocprofv3 kernel trace (csv): steps are the intervals between
consecutive ends of a marker kernel (default the head kernel; `adam` for a training step); prints, for the median
step, each kernel's duration and the idle gap before it.
  tools/r05_gaps.py <kernel_trace.csv> [steps=20] [marker=head]"""
import csv
import statistics
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
MARK = sys.argv[3] if len(sys.argv) > 3 else "head"
ends = [i for i, (s, e, k) in enumerate(rows) if MARK in k]
steps = []
for a, b in zip(ends[-K - 1:-1], ends[-K:]):
    seg = rows[a:b + 1]
    wall = seg[-1][1] - seg[0][1]
    busy = sum(e - s for s, e, k in seg[1:])
    steps.append((wall, busy, seg))
steps.sort(key=lambda t: t[0])
wall, busy, seg = steps[len(steps) // 2]
print(f"median step: wall {wall / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, idle {(wall - busy) / 1e3:.1f} us "
      f"({len(seg) - 1} launches); walls {statistics.mean(t[0] for t in steps) / 1e3:.1f} mean")
prev_end = seg[0][1]
for s, e, k in seg[1:]:
    print(f"  gap {(s - prev_end) / 1e3:6.2f} us  run {(e - s) / 1e3:7.2f} us  {k[:80]}")
    prev_end = e
