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


# ------------------------------------------------------------------------------------------------------------
# The builder's on-disk level files, next-node labels and (n-1)-gram feature pooling
# ------------------------------------------------------------------------------------------------------------

def _keys_of(strings: Sequence[str], alphabet: str, n: int) -> np.ndarray:
    """Base-K keys of equal-length strings under `alphabet`'s code (index = code)."""
    if len(strings) == 0:
        return np.zeros(0, dtype=np.int64)
    lut = np.full(256, -1, dtype=np.int64)
    for i, ch in enumerate(alphabet):
        lut[ord(ch)] = i
    try:
        raw = np.frombuffer("".join(strings).encode("latin-1"), dtype=np.uint8)
    except UnicodeEncodeError as e:
        raise ValueError("n-gram strings must be single-byte (latin-1) text") from e
    if raw.size != n * len(strings):
        raise ValueError(f"every n-gram must have length {n}")
    codes = lut[raw].reshape(len(strings), n)
    if (codes < 0).any():
        raise ValueError("n-gram strings use characters outside the alphabet")
    K = len(alphabet)
    keys = np.zeros(len(strings), dtype=np.int64)
    for j in range(n):
        keys = keys * K + codes[:, j]
    return keys


def transitions_from_table(n: int, src, dst, cnt, node_strings: Sequence[str], alphabet: Optional[str] = None,
                           device=None) -> NgramTransitions:
    """An NgramTransitions from a plain table: node ids must be the ranks of `node_strings` in sorted string order
    (the reference's ids, data_builder.py:171-175); `alphabet` defaults to the characters present, in code-point
    order (pass the other level's alphabet to pool across levels)."""
    node_strings = list(node_strings)
    if alphabet is None:
        alphabet = "".join(sorted(set("".join(node_strings))))
    if len(alphabet) and n * math.log2(max(len(alphabet), 2)) >= 62.5:
        raise ValueError(f"{len(alphabet)}^{n} windows do not fit a 64-bit key")
    keys = _keys_of(node_strings, alphabet, n)
    if keys.size > 1 and not (np.diff(keys) > 0).all():
        raise ValueError("node ids are not the ranks of the n-grams in sorted string order")
    dev = torch.device(device) if device is not None else torch.device("cpu")
    as64 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64)).to(dev)  # noqa: E731
    return NgramTransitions(n, len(node_strings), as64(src), as64(dst),
                            torch.as_tensor(np.asarray(cnt, dtype=np.float32)).to(dev), as64(keys), alphabet)


def level_paths(directory: str, n: int) -> Tuple[str, str]:
    """(ngram_map_n{n}.parquet, aggregated_edges_n{n}.parquet) -- the builder's files for level n
    (data_builder.py:145, :281)."""
    return (os.path.join(directory, f"ngram_map_n{n}.parquet"), os.path.join(directory, f"aggregated_edges_n{n}.parquet"))


def write_level(t: NgramTransitions, directory: str) -> Tuple[str, str]:
    """Write a level in the builder's schema: the n-gram map {id: int64, ngram: string} sorted by id
    (data_builder.py:170-177) and the aggregated edges {source, target, weight: int64}
    (groupby(['source', 'target']).size(), :268-286)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    os.makedirs(directory, exist_ok=True)
    mpath, epath = level_paths(directory, t.n)
    pq.write_table(pa.table({"id": pa.array(np.arange(t.num_nodes, dtype=np.int64)),
                             "ngram": pa.array(t.node_strings(), type=pa.string())}), mpath)
    pq.write_table(pa.table({"source": pa.array(t.src.cpu().numpy().astype(np.int64)),
                             "target": pa.array(t.dst.cpu().numpy().astype(np.int64)),
                             "weight": pa.array(t.cnt.cpu().numpy().astype(np.int64))}), epath)
    return mpath, epath


def read_level(directory: str, n: int, device=None, alphabet: Optional[str] = None) -> NgramTransitions:
    """Read a level written by the reference's builder (or write_level): nodes from the n-gram map, weighted
    edges from the aggregated-edge file read as DirectedNgramGraph does (graph_utils.py:106-117: source/target
    int64, weight float32); edges are returned sorted by (source, target)."""
    import pyarrow.parquet as pq
    mpath, epath = level_paths(directory, n)
    nodes = pq.read_table(mpath, columns=["id", "ngram"]).to_pandas()
    nodes = nodes.sort_values("id")
    ids = nodes["id"].to_numpy(dtype=np.int64)
    if not np.array_equal(ids, np.arange(ids.size)):
        raise ValueError(f"{mpath}: ids are not 0..N-1")
    strings = nodes["ngram"].astype(str).tolist()
    if os.path.exists(epath):
        e = pq.read_table(epath, columns=["source", "target", "weight"]).to_pandas()
        src = e["source"].to_numpy(dtype=np.int64)
        dst = e["target"].to_numpy(dtype=np.int64)
        w = e["weight"].to_numpy(dtype=np.float32)
        order = np.lexsort((dst, src))
        src, dst, w = src[order], dst[order], w[order]
    else:  # the builder removes the file when a level has no edges (data_builder.py:291-294)
        src = dst = np.zeros(0, dtype=np.int64)
        w = np.zeros(0, dtype=np.float32)
    N = len(strings)
    if src.size and (src.min() < 0 or dst.min() < 0 or src.max() >= N or dst.max() >= N):
        raise ValueError(f"{epath}: edge endpoints outside 0..{N - 1}")
    return transitions_from_table(n, src, dst, w, strings, alphabet, device)


def read_edge_parts(paths: Sequence[str]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The builder's raw transition parts ('source target' per line, data_builder.py:263-266) aggregated like
    groupby(['source', 'target']).size(): (source, target, count), sorted by (source, target). Malformed lines
    are skipped (on_bad_lines='skip')."""
    pairs = []
    for path in paths:
        with open(path, "r", encoding="utf-8", errors="ignore") as f:
            for line in f:
                parts = line.split()
                if len(parts) != 2:
                    continue
                try:
                    pairs.append((int(parts[0]), int(parts[1])))
                except ValueError:
                    continue
    if not pairs:
        z = np.zeros(0, dtype=np.int64)
        return z, z, z
    a = np.asarray(pairs, dtype=np.int64)
    uniq, counts = np.unique(a, axis=0, return_counts=True)  # lexicographic = sorted by (source, target)
    return uniq[:, 0], uniq[:, 1], counts.astype(np.int64)


def next_node_labels(t: NgramTransitions, tie_break: str = "first",
                     generator: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, int]:
    """The trainer's next_node task labels (protgram_directgcn_trainer.py:222-236) for all nodes at once: the
    successor with the largest transition count, the node itself when it has none; num_classes = N. The
    reference breaks ties with random.choice; tie_break='first' takes the smallest successor id, 'random' a
    uniformly random one (torch `generator` on the transitions' device)."""
    N = t.num_nodes
    dev = t.src.device
    labels = torch.arange(N, dtype=torch.int64, device=dev)
    if N == 0 or t.src.numel() == 0:
        return labels, max(N, 1) if N == 0 else N
    w = t.cnt.to(torch.float32)
    rowmax = torch.full((N,), float("-inf"), device=dev).scatter_reduce(0, t.src, w, "amax")
    cand = w == rowmax[t.src]
    cs, cd = t.src[cand], t.dst[cand]
    if tie_break == "first":
        pick = torch.full((N,), N, dtype=torch.int64, device=dev).scatter_reduce(0, cs, cd, "amin")
    elif tie_break == "random":
        r = torch.rand(cs.numel(), generator=generator, device=dev)
        best = torch.full((N,), -1.0, device=dev).scatter_reduce(0, cs, r, "amax")
        win = r == best[cs]
        pick = torch.full((N,), N, dtype=torch.int64, device=dev).scatter_reduce(0, cs[win], cd[win], "amin")
    else:
        raise ValueError("tie_break must be 'first' or 'random'")
    has = pick < N
    labels[has] = pick[has]
    return labels, N


def pool_features(cur: NgramTransitions, prev: NgramTransitions, emb_prev: torch.Tensor) -> torch.Tensor:
    """Initial level-n features from the level-(n-1) embeddings (protgram_directgcn_trainer.py:317-330): the mean
    of the prefix (ngram[:-1]) and suffix (ngram[1:]) rows that exist at level n-1 -- both: (a + b) / 2 in fp32 as
    np.mean does, one: that row, none: zeros. Both levels must share one alphabet code."""
    if cur.n != prev.n + 1:
        raise ValueError("prev must be level n-1")
    if cur.alphabet != prev.alphabet:
        raise ValueError("the two levels use different alphabet codes (build them from the same sequences, or pass "
                         "one alphabet to transitions_from_table / read_level)")
    if emb_prev.size(0) != prev.num_nodes:
        raise ValueError("emb_prev must have one row per level-(n-1) node")
    dev = emb_prev.device
    K = max(len(cur.alphabet), 1)
    keys = cur.node_keys.to(dev)
    pk = prev.node_keys.to(dev)
    prefix = keys // K
    suffix = keys % (K ** (cur.n - 1))
    F = emb_prev.size(1)
    x = torch.zeros(cur.num_nodes, F, dtype=emb_prev.dtype, device=dev)
    if cur.num_nodes == 0 or pk.numel() == 0:
        return x

    def lookup(q):
        i = torch.searchsorted(pk, q).clamp_(max=pk.numel() - 1)
        return i, pk[i] == q

    pi, pok = lookup(prefix)
    si, sok = lookup(suffix)
    both = pok & sok
    x[both] = (emb_prev[pi[both]] + emb_prev[si[both]]) / 2
    only_p = pok & ~sok
    x[only_p] = emb_prev[pi[only_p]]
    only_s = sok & ~pok
    x[only_s] = emb_prev[si[only_s]]
    return x
