#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs (all passes under a dir) per kernel: mean per dispatch."""
import collections
import csv
import glob
import re
import sys



def classify(k):
    if "ngram_mid_kernel" in k:
        return "ngram_mid"
    if "ngram_spmm3t_kernel" in k:
        return "ngram_spmm3t"
    if "ngram_spmm3_lds_kernel" in k:
        return "ngram_spmm3_lds_gated" if ", true>" in k else "ngram_spmm3_lds"
    if "ngram_spmm3_cs_kernel" in k:
        return "ngram_spmm3_cs_gated" if ", true>" in k else "ngram_spmm3_cs"
    if "ngram_spmm3_kernel" in k:
        return "ngram_spmm3_gated" if ", true>" in k else "ngram_spmm3"
    if re.search(r"spmm_win_kernel<\d+, \d+, \d+, 0, 256, true>", k):
        return "spmm3_gated_window"
    m = re.search(r"spmm_win_kernel<\d+, \d+, \d+, (\d)(, \d+, false)?>", k)
    if m:
        return {"0": "spmm3_window", "1": "spmm3_fusednorm_window", "2": "spmm3t_window"}.get(m.group(1), "spmm_window")
    if "dense_x3p_kernel" in k:  # pipelined split-bf16 dense kernel: <pregated, stamp>
        return "dense_x3p_pregated" if "<true" in k else "dense_x3p"
    if "head_f128_kernel" in k:
        return "head_f128"
    if "head_x3_kernel" in k:
        return "head_x3"
    if "dense_x3_kernel" in k:  # split-bf16 W-stationary dense kernel: <F_IN, KSEG, pregated>
        return "dense_x3_pregated" if k.rstrip(")").find("true>") >= 0 else "dense_x3"
    for key, short in (("spmm_vec_kernel", "spmm_bcast"),
                       ("dgrad_kernel", "dense_dgrad"), ("wgrad_kernel", "dense_wgrad"),
                       ("reduce_splits", "wgrad_reduce"), ("dense_kernel", "dense"), ("head_kernel", "head")):
        if key in k:
            return short
    return None


d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = classify(k)
        if short is None:
            continue
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = classify(k)
        if short:
            dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in vals.items():
    print(f"== {k}  (profiled dispatch avg {sum(dur[k]) / max(1, len(dur[k])):.1f} us)")
    for c, v in sorted(cs.items()):
        print(f"   {c:34s} {sum(v) / len(v):16.1f}")
