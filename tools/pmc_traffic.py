#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic (profiles/traffic_rNN.json).

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced
(16 B/lane) reads on gfx950 -> read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for
16 B/lane stores -> write bytes = WRITE_SIZE * 1024. Averages over all dispatches of each kernel.
usage: tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> <workload-tag>
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fetch_dir, write_dir, out, tag = sys.argv[1:5]
    fetch, nf = per_kernel(fetch_dir, "FETCH_SIZE")
    write, nw = per_kernel(write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        kernels[k] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
                      "FETCH_SIZE_KiB": fetch.get(k), "WRITE_SIZE_KiB": write.get(k),
                      "dispatches": [nf.get(k, 0), nw.get(k, 0)]}
    # the bench's propagation kernel: variant C (window), MODE 0 (three precomputed weights), gated store
    # (pg_spmm3_gated_f32, the inference path); the ungated training instance stays under "kernels"
    spmm = [k for k in kernels if re.search(r"spmm_win_kernel<\d+, \d+, \d+, 0, 256, true>", k)]
    spmm = spmm or [k for k in kernels if re.search(r"spmm_win_kernel<\d+, \d+, \d+, 0>", k)]
    res = {"workload": tag, "correction": "read = 2*FETCH_SIZE KiB (gfx950 half-count on 16B/lane reads); "
                                          "write = WRITE_SIZE KiB",
           "kernels": kernels}
    if spmm:
        res["kernel"] = spmm[0]
        res["kernel_bytes_per_launch"] = kernels[spmm[0]]["bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: round(v["bytes_per_launch"] / 1e6, 1) for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
