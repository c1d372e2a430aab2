"""n-gram producer (ngram.py): host-side semantics of the reference's builder on CPU; the GPU key kernel and
sorts against the Python restatement (synth.fasta_edges, which made the golden fixtures) and the fixtures'
own raw transition tables. p1_fasta (tools/golden/make_producer_golden.py) pins both to the reference's own
FASTA reader and builder functions (data_utils.py:182-212, data_builder.py:29-54) run on a committed FASTA text."""
import numpy as np
import pytest
import torch

from golden_util import load


# ----------------------------------------------------------------------------------------------------------
# p1_fasta: outputs of the reference's DataLoader.parse_sequences and data_builder helpers (n = 1..4)
# ----------------------------------------------------------------------------------------------------------
def _p1():
    return load("p1_fasta")


def _p1_path(tmp_path):
    f = tmp_path / "p1.fasta"
    f.write_bytes(_p1()["fasta"].tobytes())
    return str(f)


def test_p1_read_fasta_and_preprocess_match_reference(pkg, tmp_path):
    from protgram_directgcn_amd import ngram
    fx = _p1()
    got = list(ngram.read_fasta(_p1_path(tmp_path)))
    assert [g[0] for g in got] == fx["ids"].tolist()
    assert [g[1] for g in got] == fx["seqs"].tolist()
    assert ngram.preprocess([g[1] for g in got]) == fx["pre"].tolist()


@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_p1_restatement_matches_reference_builder(pkg, n):
    """synth.fasta_edges (which made the f1/f5 FASTA fixtures and is the CPU check of the GPU producer) against the
    reference builder's own n-gram map and aggregated transition table."""
    fx = _p1()
    N, s, d, c, ordered = pkg.synth.fasta_edges(n, fx["pre"].tolist())
    assert ordered == fx[f"n{n}_ngrams"].tolist() and N == len(ordered)
    assert np.array_equal(s, fx[f"n{n}_src"]) and np.array_equal(d, fx[f"n{n}_dst"])
    assert np.array_equal(c, fx[f"n{n}_w"].astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_p1_gpu_producer_matches_reference_builder(pkg, cuda, tmp_path, n):
    from protgram_directgcn_amd import ngram
    fx = _p1()
    seqs = [g[1] for g in ngram.read_fasta(_p1_path(tmp_path))]
    got = ngram.ngram_transitions(seqs, n, device=cuda, pad=True)
    assert got.node_strings() == fx[f"n{n}_ngrams"].tolist()
    assert np.array_equal(got.src.cpu().numpy(), fx[f"n{n}_src"])
    assert np.array_equal(got.dst.cpu().numpy(), fx[f"n{n}_dst"])
    assert np.array_equal(got.cnt.cpu().numpy(), fx[f"n{n}_w"].astype(np.float32))


def test_read_fasta_follows_parse_sequences(pkg, tmp_path):
    from protgram_directgcn_amd import ngram
    f = tmp_path / "x.fasta"
    f.write_text(">sp|P12345|NAME_HUMAN desc\nmkv\n\nLLA\n>plainid other words\nacd\n>empty\n>sp||Q\nwy\n")
    got = list(ngram.read_fasta(str(f)))
    # '|' field 1 when present and non-empty, else the first word; lines upper-cased and joined; empty
    # records skipped (data_utils.py:182-212)
    assert got == [("P12345", "MKVLLA"), ("plainid", "ACD"), ("sp||Q", "WY")]


def test_preprocess_padding_quirk(pkg):
    from protgram_directgcn_amd import ngram
    assert ngram.preprocess(["AB", "CD", "E"]) == [" AB ", "CD ", "E "]  # data_builder.py:29-35, :98-103
    assert ngram.preprocess(["AB"], pad=False) == ["AB"]


def test_codes_preserve_string_order(pkg):
    from protgram_directgcn_amd import ngram
    buf, off, lut, alphabet = ngram.encode([" MKV ", "XA"])
    assert alphabet == " AKMVX" and off.tolist() == [0, 5, 7]
    keys = np.array([3, 17, 40, 200])
    strings = ngram.decode_keys(keys, alphabet, 3)
    assert strings == sorted(strings)
    K = len(alphabet)
    back = [sum(alphabet.index(ch) * K ** (2 - j) for j, ch in enumerate(s)) for s in strings]
    assert back == keys.tolist()


def test_key_overflow_and_no_cpu_path(pkg):
    from protgram_directgcn_amd import ngram
    with pytest.raises(ValueError):
        ngram.ngram_transitions(["ACDEFGHIKLMNPQRSTVWY"], 15, device="cuda")  # 21^15 > 2^63
    with pytest.raises(RuntimeError):
        ngram.ngram_transitions(["ACD"], 2, device="cpu")


def _ragged_sequences():
    rng = np.random.default_rng(7)
    letters = np.array(list("ACDEFGHIKLMNPQRSTVWYXU"))
    lens = [0, 1, 2, 3, 5, 40, 400, 7, 1, 250]
    return ["".join(letters[rng.integers(0, 22, size=L)]) for L in lens]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("pad", [False, True])
def test_gpu_transitions_match_restatement(pkg, cuda, n, pad):
    from protgram_directgcn_amd import ngram
    seqs = _ragged_sequences()
    got = ngram.ngram_transitions(seqs, n, device=cuda, pad=pad)
    N, s, d, c, ordered = pkg.synth.fasta_edges(n, ngram.preprocess(seqs, pad))
    assert got.num_nodes == N
    assert got.node_strings() == ordered
    assert np.array_equal(got.src.cpu().numpy(), s) and np.array_equal(got.dst.cpu().numpy(), d)
    assert np.array_equal(got.cnt.cpu().numpy(), c)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,nseq,length,seed", [("f1_fasta2", 2, 64, 400, 0), ("f5_fasta3", 3, 40, 300, 1)])
def test_gpu_transitions_match_fixture(pkg, cuda, name, n, nseq, length, seed):
    """The raw transition tables the golden fixtures fed to the reference's DirectedNgramGraph."""
    from protgram_directgcn_amd import ngram
    fx = load(name)
    seqs = pkg.synth.random_sequences(nseq, length, seed=seed)
    got = ngram.ngram_transitions(seqs, n, device=cuda, pad=False)
    assert got.num_nodes == int(fx["N"].item())
    assert np.array_equal(got.src.cpu().numpy(), fx["src"]) and np.array_equal(got.dst.cpu().numpy(), fx["dst"])
    assert np.array_equal(got.cnt.cpu().numpy(), fx["cnt"])


# ----------------------------------------------------------------------------------------------------------
# level files, next-node labels, feature pooling (CPU: tables from synth.fasta_edges, the builder restatement)
# ----------------------------------------------------------------------------------------------------------

def _level(pkg, n, seqs, alphabet=None):
    from protgram_directgcn_amd import ngram
    N, s, d, c, ordered = pkg.synth.fasta_edges(n, ngram.preprocess(seqs))
    return ngram.transitions_from_table(n, s, d, c, ordered, alphabet), ordered


def test_transitions_from_table_checks_order(pkg):
    from protgram_directgcn_amd import ngram
    with pytest.raises(ValueError):
        ngram.transitions_from_table(2, [0], [1], [1.0], ["BA", "AB"])  # ids not in sorted string order
    with pytest.raises(ValueError):
        ngram.transitions_from_table(2, [0], [1], [1.0], ["AB", "ABC"])  # ragged n-grams


def test_level_files_round_trip(pkg, tmp_path):
    import pyarrow.parquet as pq
    from protgram_directgcn_amd import ngram
    t, ordered = _level(pkg, 3, _ragged_sequences())
    mpath, epath = ngram.write_level(t, str(tmp_path))
    m = pq.read_table(mpath).to_pandas()  # the builder's schema (data_builder.py:170-177, :268-286)
    assert list(m.columns) == ["id", "ngram"] and m["ngram"].tolist() == ordered
    assert m["id"].tolist() == list(range(len(ordered)))
    e = pq.read_table(epath).to_pandas()
    assert list(e.columns) == ["source", "target", "weight"] and str(e["weight"].dtype) == "int64"
    back = ngram.read_level(str(tmp_path), 3)
    assert back.num_nodes == t.num_nodes and back.node_strings() == ordered
    assert torch.equal(back.src, t.src) and torch.equal(back.dst, t.dst) and torch.equal(back.cnt, t.cnt)
    assert torch.equal(back.node_keys, t.node_keys)


def test_read_level_written_like_the_builder(pkg, tmp_path):
    """Files made the way data_builder.py makes them (pandas -> parquet, edges unsorted, int64 counts), a level
    with no edge file (removed by the builder when empty), and endpoint validation."""
    import pandas as pd
    from protgram_directgcn_amd import ngram
    mpath, epath = ngram.level_paths(str(tmp_path), 2)
    pd.DataFrame({"id": [0, 1, 2], "ngram": [" A", "AB", "B "]}).to_parquet(mpath, index=False)
    pd.DataFrame({"source": [1, 0, 1], "target": [2, 1, 0], "weight": [3, 1, 2]}).to_parquet(epath, index=False)
    t = ngram.read_level(str(tmp_path), 2)
    assert t.num_nodes == 3 and t.alphabet == " AB"
    assert t.src.tolist() == [0, 1, 1] and t.dst.tolist() == [1, 0, 2] and t.cnt.tolist() == [1.0, 2.0, 3.0]
    import os
    os.remove(epath)
    assert ngram.read_level(str(tmp_path), 2).src.numel() == 0
    pd.DataFrame({"source": [0], "target": [7], "weight": [1]}).to_parquet(epath, index=False)
    with pytest.raises(ValueError):
        ngram.read_level(str(tmp_path), 2)


def test_read_edge_parts_matches_groupby(pkg, tmp_path):
    from oracle.ngram_cpu import aggregate_parts_ref
    from protgram_directgcn_amd import ngram
    rng = np.random.default_rng(3)
    paths = []
    for k in range(3):
        p = tmp_path / f"part-{k}.txt"
        lines = [f"{a} {b}" for a, b in rng.integers(0, 9, size=(200, 2))]
        lines.insert(5, "garbage line here")
        p.write_text("\n".join(lines) + "\n")
        paths.append(str(p))
    s, d, c = ngram.read_edge_parts(paths)
    ref = aggregate_parts_ref(paths)
    assert s.tolist() == ref["source"].tolist() and d.tolist() == ref["target"].tolist()
    assert c.tolist() == ref["weight"].tolist()


@pytest.mark.parametrize("n", [1, 2, 3])
def test_next_node_labels_vs_reference_loop(pkg, n):
    from oracle.ngram_cpu import next_node_labels_ref
    from protgram_directgcn_amd import ngram
    t, _ = _level(pkg, n, _ragged_sequences())
    ties = next_node_labels_ref(t.num_nodes, t.src.numpy(), t.dst.numpy(), t.cnt.numpy())
    first, C = ngram.next_node_labels(t)
    assert C == t.num_nodes
    assert [int(v) for v in first] == [min(s) for s in ties]
    rnd, _ = ngram.next_node_labels(t, "random", torch.Generator().manual_seed(0))
    assert all(int(v) in s for v, s in zip(rnd, ties))
    assert any(len(s) > 1 for s in ties)  # the case exercises ties


@pytest.mark.parametrize("n", [2, 3, 4])
def test_pool_features_vs_reference_loop(pkg, n):
    from oracle.ngram_cpu import pool_features_ref
    from protgram_directgcn_amd import ngram
    seqs = _ragged_sequences()
    prev, prev_strings = _level(pkg, n - 1, seqs)
    cur, cur_strings = _level(pkg, n, seqs, alphabet=prev.alphabet)
    emb = torch.randn(prev.num_nodes, 24, generator=torch.Generator().manual_seed(n))
    got = ngram.pool_features(cur, prev, emb)
    ref = pool_features_ref(cur_strings, prev_strings, emb.numpy())
    assert torch.equal(got, torch.from_numpy(ref))
    # the padded builder input makes some prefixes / suffixes absent at level n-1 (one-sided pooling)
    with pytest.raises(ValueError):
        ngram.pool_features(prev, cur, emb)


@pytest.mark.gpu
def test_labels_and_pooling_on_gpu(pkg, cuda):
    from oracle.ngram_cpu import next_node_labels_ref, pool_features_ref
    from protgram_directgcn_amd import ngram
    seqs = _ragged_sequences()
    prev = ngram.ngram_transitions(seqs, 2, device=cuda)
    cur = ngram.ngram_transitions(seqs, 3, device=cuda)
    assert cur.alphabet == prev.alphabet
    lab, _ = ngram.next_node_labels(cur)
    ties = next_node_labels_ref(cur.num_nodes, cur.src.cpu().numpy(), cur.dst.cpu().numpy(), cur.cnt.cpu().numpy())
    assert [int(v) for v in lab.cpu()] == [min(s) for s in ties]
    emb = torch.randn(prev.num_nodes, 32, generator=torch.Generator().manual_seed(1))
    got = ngram.pool_features(cur, prev, emb.to(cuda))
    ref = pool_features_ref(cur.node_strings(), prev.node_strings(), emb.numpy())
    assert torch.equal(got.cpu(), torch.from_numpy(ref))
