"""Seeded synthetic n-gram graphs, regenerable on the GPU box without fixtures.

Two generators:

* :func:`de_bruijn_edges` -- the complete n-gram transition graph B(20, n) in the reference's
  node order. The reference numbers n-grams by the rank of the sorted n-gram strings
  (``src/pipeline/data_builder.py:164,172-173``); with every n-gram present that rank is the
  base-20 value of the string over the sorted alphabet ``ACDEFGHIKLMNPQRSTVWY``. Edge
  ``s -> (20*s + c) mod 20**n`` (c = 0..19) is the window shift of ``data_builder.py:45-54``.
  Raw transition count ``1 + splitmix64(0x5eed ^ (20*s + c)) mod 64``.
* :func:`fasta_edges` -- random protein sequences cut into overlapping windows exactly as
  ``data_builder.py:38-54`` does (no space padding), then grouped into unique
  ``(source, target) -> count`` rows as ``data_builder.py:267-273`` does.

:func:`protein_sequences` makes seeded protein-like inputs for ``ngram.ngram_transitions`` (the builder's padded
graphs, off the complete grid).

Both edge generators return ``(num_nodes, src int64[E], dst int64[E], count float32[E])`` with unique
``(src, dst)`` pairs sorted row-major, i.e. the content of the reference's edge parquet.
"""
from __future__ import annotations

import numpy as np

ALPHABET = "ACDEFGHIKLMNPQRSTVWY"
SIGMA = 20
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser on uint64 (wrap-around arithmetic)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def de_bruijn_sizes(n: int) -> dict:
    """|V|, E and shared-pattern nnz of the complete B(20, n) graph."""
    N = SIGMA ** n
    E = SIGMA ** (n + 1)
    # 2*(non-loop transitions) - mutual pairs (the 380 two-periodic strings) + diagonal
    nnz = 2 * (E - SIGMA) - SIGMA * (SIGMA - 1) + N
    return {"N": N, "E": E, "nnz": nnz}


def de_bruijn_edges(n: int, seed: int = 0x5EED):
    N = SIGMA ** n
    s = np.repeat(np.arange(N, dtype=np.int64), SIGMA)
    c = np.tile(np.arange(SIGMA, dtype=np.int64), N)
    eid = s * SIGMA + c
    dst = eid % N
    cnt = (splitmix64(np.uint64(seed) ^ eid.astype(np.uint64)) % np.uint64(64)).astype(np.float32) + 1.0
    return N, s, dst, cnt


def random_sequences(num_seqs: int, length: int, seed: int = 0) -> list[str]:
    rng = np.random.default_rng(seed)
    letters = np.array(list(ALPHABET))
    return ["".join(letters[rng.integers(0, SIGMA, size=length)]) for _ in range(num_seqs)]


# UniProtKB/Swiss-Prot amino-acid composition (percent, ALPHABET order), for protein-like synthetic sequences
_AA_PERCENT = (8.25, 1.38, 5.46, 6.72, 3.86, 7.07, 2.27, 5.91, 5.80, 9.64, 2.41, 4.06, 4.74, 3.93, 5.53, 6.65, 5.36,
               6.86, 1.10, 2.92)


def protein_sequences(num_seqs: int, mean_len: int = 350, seed: int = 0, rare: float = 0.001,
                      composition: str = "swissprot") -> list[str]:
    """Seeded protein-like sequences for builder-produced graphs (the input run_graph_builder.py reads): lengths
    uniform in [mean_len / 2, 3 mean_len / 2], letters drawn with the Swiss-Prot composition ('uniform': equal), and
    a `rare` share of positions replaced by the non-standard letters X / U / B / Z (which put n-grams off the
    20-letter grid, as the padding ' ' of data_builder.py:29-35 does)."""
    rng = np.random.default_rng(seed)
    letters = np.array(list(ALPHABET))
    if composition == "uniform":
        prob = np.full(SIGMA, 1.0 / SIGMA)
    else:
        prob = np.asarray(_AA_PERCENT, dtype=np.float64)
        prob = prob / prob.sum()
    lo, hi = max(1, mean_len // 2), max(1, mean_len // 2) + mean_len
    odd = np.array(list("XUBZ"))
    out = []
    for _ in range(num_seqs):
        L = int(rng.integers(lo, hi + 1))
        seq = letters[rng.choice(SIGMA, size=L, p=prob)]
        if rare > 0:
            hit = rng.random(L) < rare
            if hit.any():
                seq[hit] = odd[rng.integers(0, odd.size, size=int(hit.sum()))]
        out.append("".join(seq))
    return out


def fasta_edges(n: int, sequences: list[str]):
    """n-gram map (sorted unique strings -> rank) and unique transition counts."""
    grams = set()
    for seq in sequences:
        for i in range(len(seq) - n + 1):
            grams.add(seq[i:i + n])
    ordered = sorted(grams)
    ids = {g: i for i, g in enumerate(ordered)}
    pairs: dict[tuple[int, int], int] = {}
    for seq in sequences:
        for i in range(len(seq) - n):
            key = (ids[seq[i:i + n]], ids[seq[i + 1:i + 1 + n]])
            pairs[key] = pairs.get(key, 0) + 1
    keys = sorted(pairs)
    src = np.array([k[0] for k in keys], dtype=np.int64)
    dst = np.array([k[1] for k in keys], dtype=np.int64)
    cnt = np.array([pairs[k] for k in keys], dtype=np.float32)
    return len(ordered), src, dst, cnt, ordered


def trainer_coo(g):
    """The three propagation matrices of a shared-pattern CSRGraph in the form the reference trainer hands them to
    the model: ``edge_index_* = mathcal_A_*.indices()`` and ``edge_weight_* = mathcal_A_*.values()`` of a coalesced
    torch sparse COO (``protgram_directgcn_trainer.py:362-367``; coalesced by ``graph_utils.py:154, 193-195, 269``),
    i.e. entries sorted by (row, col) with PyG's flow ``out[ei[1]] += w * x[ei[0]]``: ei[0] = source, ei[1] =
    destination. Returns (ei_in, w_in, ei_out, w_out, ei_und, w_und) on g's device; the three index tensors are
    distinct tensors with equal values, as the trainer's are. Test and bench input construction only."""
    import torch
    from .graph import take
    if not g.shared:
        raise ValueError("trainer_coo needs a shared-pattern graph")
    dev = g.rowptr.device
    dst = torch.repeat_interleave(torch.arange(g.n_rows, device=dev), g.rowptr[1:] - g.rowptr[:-1])
    src = g.edges3[:, 0].to(torch.int64)
    order = torch.sort(src * g.n_rows + dst).indices  # coalesced: by (row = source, col = destination)
    ei = torch.stack([take(src, order), take(dst, order)])
    w = [take(g.edges3[:, 1 + k].contiguous(), order).view(torch.float32) for k in range(3)]
    return ei, w[0], ei.clone(), w[1], ei.clone(), w[2]


def trainer_data(g, x):
    """A Data object wired like the reference trainer's (``protgram_directgcn_trainer.py:343-344, 362-367``): x plus
    the COO tensors of trainer_coo(g) under the attribute names the model reads (``protgram_directgcn.py:196-203``)."""
    from .data import Data
    ei_in, w_in, ei_out, w_out, ei_und, w_und = trainer_coo(g)
    return Data(x=x, edge_index_in=ei_in, edge_weight_in=w_in, edge_index_out=ei_out, edge_weight_out=w_out,
                edge_index_undirected_norm=ei_und, edge_weight_undirected_norm=w_und)
