#!/usr/bin/env python3
"""Golden vectors for the n-gram producer, from the REFERENCE's own builder functions (build container only).

Imports, unchanged, ``src/utils/data_utils.py`` (``DataLoader.parse_sequences``, the FASTA reader) and
``src/pipeline/data_builder.py`` (``_preprocess_sequence_tuple_for_bag``, ``_extract_ngrams_from_sequence_tuple``,
``_extract_edges_from_sequence_tuple``, :29-54). Their module-level imports that are absent here and unused by those
functions are stubbed in ``sys.modules``: ``dask.bag`` / ``dask.dataframe`` (the builder's scheduling), ``config``,
``Bio`` and ``h5py``; PyG through ``pyg_boundary.install()``. ``GraphBuilder.run``'s glue around the helpers
(data_builder.py:97-103 first-sequence flag, :151-173 distinct + sort + rank ids, :203-206 edge strings, :267-271
groupby(['source','target']).size()) is restated here in a few lines of plain Python -- Dask only distributes it.

Writes ``tests/golden/p1_fasta.npz``: the FASTA text (input) and, per level n = 1..4, the sorted n-gram strings and
the aggregated (source, target, weight) table the builder hands to DirectedNgramGraph. No reference source or
bytecode is written (``sys.dont_write_bytecode``).

Usage:  python tools/golden/make_producer_golden.py
"""
import collections
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
if not os.path.isdir(os.path.join(REF, "src")):
    sys.exit("make_producer_golden.py: /root/reference is absent; fixtures can only be generated in the build container")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, HERE)
import pyg_boundary  # noqa: E402

pyg_boundary.install()


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Config:  # the builder's configuration object; the helper functions never read it
    pass


dask = _stub("dask")
dask.bag = _stub("dask.bag")
dask.dataframe = _stub("dask.dataframe")
_stub("config", Config=_Config)
bio = _stub("Bio")
bio.SeqIO = _stub("Bio.SeqIO")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from src.pipeline import data_builder as ref_builder  # noqa: E402
from src.utils.data_utils import DataLoader  # noqa: E402

ALPHABET = "ACDEFGHIKLMNPQRSTVWYXU"


def fasta_text(seed=7):
    """Ragged records with the header forms parse_sequences distinguishes, blank lines, lower case and wrapped
    sequence lines."""
    rng = np.random.default_rng(seed)
    lens = [0, 1, 2, 3, 5, 40, 400, 7, 1, 250, 60, 33]
    lines = []
    for i, L in enumerate(lens):
        seq = "".join(rng.choice(list(ALPHABET), size=L))
        if i % 3 == 0:
            lines.append(f">sp|P{i:05d}|PROT{i}_HUMAN protein {i}")
        elif i % 3 == 1:
            lines.append(f">seq{i} some description")
        else:
            lines.append(f">tr||X{i} empty accession field")
        if i == 4:
            seq = seq.lower()
        for k in range(0, L, 61):  # wrapped
            lines.append(seq[k:k + 61])
        if i == 6:
            lines.append("")
    return "\n".join(lines) + "\n"


def level(pre, n):
    """GraphBuilder.run, phase 1 (data_builder.py:151-228) and the phase-2 aggregation (:267-273)."""
    grams = set()
    for t in pre:
        grams.update(ref_builder._extract_ngrams_from_sequence_tuple(t, n_val=n))
    ordered = sorted(grams)
    ids = {g: i for i, g in enumerate(ordered)}
    counts = collections.Counter()
    for t in pre:
        for line in ref_builder._extract_edges_from_sequence_tuple(t, n_val=n, ngram_to_id_map=ids):
            s, d = line.split()
            counts[(int(s), int(d))] += 1
    keys = sorted(counts)
    src = np.array([k[0] for k in keys], np.int64)
    dst = np.array([k[1] for k in keys], np.int64)
    w = np.array([counts[k] for k in keys], np.int64)
    return ordered, src, dst, w


def main():
    text = fasta_text()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "in.fasta")
        with open(path, "w") as f:
            f.write(text)
        records = list(DataLoader.parse_sequences(path))
    # data_builder.py:97-103 + :119: the first sequence is preprocessed with add_initial_space=True
    pre = [ref_builder._preprocess_sequence_tuple_for_bag(t, i == 0) for i, t in enumerate(records)]
    fx = {"fasta": np.frombuffer(text.encode(), np.uint8),
          "ids": np.array([r[0] for r in records]), "seqs": np.array([r[1] for r in records]),
          "pre": np.array([p[1] for p in pre])}
    for n in (1, 2, 3, 4):
        ordered, src, dst, w = level(pre, n)
        fx[f"n{n}_ngrams"] = np.array(ordered)
        fx[f"n{n}_src"], fx[f"n{n}_dst"], fx[f"n{n}_w"] = src, dst, w
        print(f"  n={n}: {len(ordered)} n-grams, {src.size} transitions, {int(w.sum())} counted")
    out = os.path.join(OUT, "p1_fasta.npz")
    np.savez_compressed(out, **fx)
    print(f"  wrote {os.path.relpath(out, REPO)} ({os.path.getsize(out) / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
