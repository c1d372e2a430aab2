"""Helpers to read the committed golden fixtures (tests/golden/*.npz, made by tools/golden/make_golden.py)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["f1_fasta2", "f1_debruijn2", "f2_edge", "f2_empty", "f3_bench", "f4_cluster", "f5_fasta3",
         "f5_debruijn3", "f6_pe1"]


def load(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def params(fx, prefix):
    """'L_p:lin_main_in.weight' -> {'lin_main_in.weight': tensor}"""
    tag = f"{prefix}:"
    return {k[len(tag):]: torch.from_numpy(v.copy()) for k, v in fx.items() if k.startswith(tag)}


def graph(fx):
    """(edge_index, edge_weight) per adjacency as the trainer wires them (None when absent)."""
    ei, ew = {}, {}
    for k in ("in", "out", "und"):
        ei[k] = torch.from_numpy(fx[f"{k}_idx"].astype(np.int64)).reshape(2, -1)
        ew[k] = torch.from_numpy(fx[f"{k}_val"].copy()) if f"{k}_val" in fx else None
    return ei, ew


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a).copy())
