#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic.

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced
(16 B/lane) reads on gfx950 -> read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for
16 B/lane stores -> write bytes = WRITE_SIZE * 1024. Averages over all dispatches of each kernel.
The "dominant" kernel is the propagation kernel with the largest total duration in the FETCH_SIZE pass's trace.
Used by bench.py (live, every N=1 run) and from the command line:
usage: tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> <workload-tag>
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def durations(d):
    """Total and per-dispatch duration (ns) per kernel from the pass's kernel trace."""
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            tot[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            cnt[k] += 1
    return {k: (tot[k], tot[k] / cnt[k]) for k in tot}


def reduce(fetch_dir, write_dir, prefer=("ngram", "spmm")):
    """Per-kernel traffic; "kernel" = the propagation kernel (a name containing one of `prefer`) with the largest
    total duration, else the kernel with the largest total duration (a pass over the trainer's COO entry also traces
    the one-time COO -> CSR sorts, which must not be mistaken for the dominant kernel)."""
    fetch, nf = per_kernel(fetch_dir, "FETCH_SIZE")
    write, nw = per_kernel(write_dir, "WRITE_SIZE")
    dur = durations(fetch_dir)
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        kernels[k] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
                      "FETCH_SIZE_KiB": fetch.get(k), "WRITE_SIZE_KiB": write.get(k),
                      "dispatches": [nf.get(k, 0), nw.get(k, 0)],
                      "avg_ns_under_pmc": dur.get(k, (0, 0))[1]}
    res = {"correction": "read = 2*FETCH_SIZE KiB (gfx950 half-count on 16B/lane reads); write = WRITE_SIZE KiB",
           "kernels": kernels}
    ranked = sorted((k for k in kernels if k in dur), key=lambda k: -dur[k][0])
    pref = [k for k in ranked if any(t in k for t in prefer)]
    if pref or ranked:
        res["kernel"] = (pref or ranked)[0]
        res["kernel_bytes_per_launch"] = kernels[res["kernel"]]["bytes_per_launch"]
    # per class of hot-path kernel (bench.py's roofline entries): the kernel of that class with the largest total
    # duration in the pass
    res["by_class"] = {}
    for cls, tags in CLASSES.items():
        hits = [k for k in ranked if any(t in k for t in tags)]
        if hits:
            res["by_class"][cls] = {"kernel": hits[0], "bytes_per_launch": kernels[hits[0]]["bytes_per_launch"],
                                    "avg_ns_under_pmc": kernels[hits[0]]["avg_ns_under_pmc"]}
    return res


# kernel-name tags of the hot-path kernel classes (the HIP kernels' symbol names)
CLASSES = {"propagation": ("ngram_mid_kernel", "ngram_spmm3_kernel", "spmm_win_kernel", "spmm_vec_kernel",
                           "spmm_scalar_kernel", "spmm_bf16_kernel"),
           "dense": ("dense_",),
           "head": ("head_",)}


def main():
    fetch_dir, write_dir, out, tag = sys.argv[1:5]
    res = reduce(fetch_dir, write_dir)
    res["workload"] = tag
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: round(v["bytes_per_launch"] / 1e6, 1) for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
