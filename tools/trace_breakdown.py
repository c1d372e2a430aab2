#!/usr/bin/env python3
"""Per-step GPU time by kernel from a rocprofv3 kernel trace (csv) of tools/middle_train_probe.py --ranks R --reps K:
the last K steps (the HIP-graph replays) are the intervals between the last K*A + 1 ends of the Adam kernel (A launches
per step: one per parameter group).
usage: tools/trace_breakdown.py <kernel_trace.csv> [K=10] [top=25] [A=2]"""
import collections
import csv
import sys

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
A = int(sys.argv[4]) if len(sys.argv) > 4 else 2
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
rows.sort()
ends = [e for s, e, k in rows if "adam_kernel" in k]
t0, t1 = ends[-K * A - 1], ends[-1]
seg = [(s, e, k) for s, e, k in rows if s > t0 and e <= t1]
tot = collections.defaultdict(float)
cnt = collections.Counter()
for s, e, k in seg:
    tot[k] += e - s
    cnt[k] += 1
busy = sum(tot.values()) / K / 1e3
print(f"last {K} steps: {len(seg) / K:.0f} launches per step, GPU busy {busy:.1f} us per step, "
      f"wall {(t1 - t0) / K / 1e3:.1f} us per step")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{v / K / 1e3:9.1f} us/step {cnt[k] / K:5.1f} calls/step  {k[:110]}")
