#!/usr/bin/env python3
"""Probe of ROCm torch's index gather at results of >= 1 GiB (the failure graph.take guards against).

For several result sizes and row widths, gathers t[idx] on the GPU in one call (and index_select), and compares the
result with the host gather of the same inputs; then the same through graph.take. Prints one line per case:
  rows row_bytes result_GiB  raw_ok raw_bad_rows  index_select_ok  take_ok
Usage: python tools/gather_probe.py [--out profiles/r03_gather_probe.txt]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ap = argparse.ArgumentParser()
ap.add_argument("--out", default=None)
args = ap.parse_args()
dev = torch.device("cuda:0")
lines = [f"# torch {torch.__version__}, device {torch.cuda.get_device_name(0)}",
         "# rows row_bytes result_GiB raw_ok raw_bad_rows first_bad index_select_ok take_ok"]
print(lines[0], flush=True)
for cols, dtype, nrows in ((4, torch.int32, 114_800_000), (128, torch.float32, 2_400_000), (4, torch.int32, 40_000_000),
                           (128, torch.float32, 1_600_000)):
    gen = torch.Generator().manual_seed(1)
    t = torch.randint(0, 1 << 30, (nrows, cols), generator=gen, dtype=torch.int64).to(dtype) if dtype == torch.int32 \
        else torch.randn(nrows, cols, generator=gen)
    idx = torch.randint(0, nrows, (nrows,), generator=gen)
    ref = t[idx]
    td, idd = t.to(dev), idx.to(dev)
    raw = td[idd].cpu()
    bad = (raw != ref).any(1) if raw.dim() > 1 else raw != ref
    nb = int(bad.sum())
    first = int(bad.nonzero()[0]) if nb else -1
    isel = bool(torch.equal(torch.index_select(td, 0, idd).cpu(), ref))
    tk = bool(torch.equal(pkg.graph.take(td, idd).cpu(), ref))
    gib = nrows * cols * t.element_size() / 2 ** 30
    line = f"{nrows} {cols * t.element_size()} {gib:.3f} {nb == 0} {nb} {first} {isel} {tk}"
    print(line, flush=True)
    lines.append(line)
    del td, idd, raw, ref, t, idx
    torch.cuda.empty_cache()
if args.out:
    with open(args.out, "w") as f:
        f.write("\n".join(lines) + "\n")
