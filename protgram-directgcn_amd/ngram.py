"""Upstream n-gram graph producer on the GPU.

The reference builds each level's transition graph with Dask string processing
(``src/pipeline/data_builder.py``):

* sequences come from ``DataLoader.parse_sequences`` (``src/utils/data_utils.py:182-212``: '>' headers,
  id = header.split('|')[1] or the first word, sequence lines stripped and upper-cased);
* only the FIRST sequence gets a leading space and EVERY sequence a trailing space
  (``_preprocess_sequence_tuple_for_bag``, :29-35);
* nodes are the distinct length-n windows, ids = ranks in sorted string order (:38-42, :171-175);
* transitions are consecutive windows inside one sequence (:45-54), aggregated to counts (:277-281).

Here the windows become base-K integer keys with an order-preserving character code, computed by the HIP
kernel ``pg_ngram_keys`` (one block per sequence); node ids and transition counts come from two GPU sorts
(``torch.unique``). The result is the raw transition table that ``graph.build_propagation_csr`` (or the
reference's ``DirectedNgramGraph``) consumes.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, load_library


def read_fasta(path: str) -> Iterator[Tuple[str, str]]:
    """(protein_id, sequence) pairs with the parsing rules of DataLoader.parse_sequences
    (data_utils.py:182-212)."""
    pid: Optional[str] = None
    parts: List[str] = []
    with open(os.path.normpath(path), "r", encoding="utf-8", errors="ignore") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith(">"):
                if pid and parts:
                    yield pid, "".join(parts)
                header = line[1:]
                fields = header.split("|")
                pid = fields[1] if len(fields) > 1 and fields[1] else header.split()[0]
                parts = []
            elif pid is not None:
                parts.append(line.upper())
    if pid and parts:
        yield pid, "".join(parts)


def preprocess(sequences: Sequence[str], pad: bool = True) -> List[str]:
    """data_builder.py:29-35 + :98-103: a leading space on the first sequence only, a trailing space on every
    sequence (pad=False: the sequences as given)."""
    if not pad:
        return list(sequences)
    return [(" " if i == 0 else "") + s + " " for i, s in enumerate(sequences)]


@dataclass
class NgramTransitions:
    n: int
    num_nodes: int
    src: torch.Tensor      # int64 [E] (sorted by (src, dst))
    dst: torch.Tensor      # int64 [E]
    cnt: torch.Tensor      # float32 [E] transition counts (the reference's edge weights)
    node_keys: torch.Tensor  # int64 [N] sorted window keys (node id = position)
    alphabet: str          # characters in code order (code = index)

    def node_strings(self) -> List[str]:
        """Decode the node keys to the n-gram strings (the reference's idx_to_node map, data_builder.py:264)."""
        return decode_keys(self.node_keys.cpu().numpy(), self.alphabet, self.n)


def decode_keys(keys: np.ndarray, alphabet: str, n: int) -> List[str]:
    K = len(alphabet)
    k = keys.astype(np.int64).copy()
    digits = np.empty((k.size, n), dtype=np.int64)
    for j in range(n - 1, -1, -1):
        digits[:, j] = k % K
        k //= K
    table = np.array(list(alphabet))
    return ["".join(row) for row in table[digits]] if k.size else []


def encode(sequences: Sequence[str]):
    """Concatenated bytes, int64 offsets, the order-preserving code table and the alphabet."""
    try:
        raw = [s.encode("latin-1") for s in sequences]
    except UnicodeEncodeError as e:
        raise ValueError("sequences must be single-byte (latin-1) text: windows are taken over characters") from e
    lens = np.fromiter((len(b) for b in raw), dtype=np.int64, count=len(raw))
    offsets = np.zeros(len(raw) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(raw), dtype=np.uint8)
    present = np.flatnonzero(np.bincount(buf, minlength=256)) if buf.size else np.zeros(0, dtype=np.int64)
    lut = np.full(256, 0, dtype=np.int32)
    lut[present] = np.arange(present.size, dtype=np.int32)  # byte order == code point order for latin-1
    alphabet = "".join(chr(b) for b in present)
    return buf, offsets, lut, alphabet


def ngram_transitions(sequences: Sequence[str], n: int, device="cuda", pad: bool = True) -> NgramTransitions:
    """Nodes and weighted transitions of the level-n graph (data_builder.py run(), phases 1-2)."""
    if n < 1:
        raise ValueError("n must be >= 1")
    seqs = preprocess(sequences, pad)
    buf, offsets, lut, alphabet = encode(seqs)
    K = max(len(alphabet), 1)
    if n * math.log2(K) >= 62.5:
        raise ValueError(f"{K}^{n} windows do not fit a 64-bit key")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("the n-gram producer runs on the MI355X only (no CPU path)")
    T = int(buf.size)
    e = torch.zeros(0, dtype=torch.int64, device=dev)
    if T == 0:
        return NgramTransitions(n, 0, e, e, e.float(), e, alphabet)
    b = torch.from_numpy(buf.copy()).to(dev)
    off = torch.from_numpy(offsets).to(dev)
    lt = torch.from_numpy(lut).to(dev)
    keys = torch.empty(T, dtype=torch.int64, device=dev)
    nxt = torch.empty(T, dtype=torch.int64, device=dev)
    lib = load_library()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    check(lib.pg_ngram_keys(len(seqs), ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                            ctypes.c_void_p(lt.data_ptr()), n, K, ctypes.c_void_p(keys.data_ptr()),
                            ctypes.c_void_p(nxt.data_ptr()), stream), "pg_ngram_keys")
    node_keys = torch.unique(keys[keys >= 0])  # sorted: node id = rank of the window in string order
    N = int(node_keys.numel())
    m = nxt >= 0
    si = torch.searchsorted(node_keys, keys[m])
    di = torch.searchsorted(node_keys, nxt[m])
    pairs, cnt = torch.unique(si * max(N, 1) + di, return_counts=True)
    return NgramTransitions(n, N, pairs // max(N, 1), pairs % max(N, 1), cnt.to(torch.float32), node_keys, alphabet)
