"""n-gram producer (ngram.py): host-side semantics of the reference's builder on CPU; the GPU key kernel and
sorts against the Python restatement (synth.fasta_edges, which made the golden fixtures) and the fixtures'
own raw transition tables."""
import numpy as np
import pytest
import torch

from golden_util import load


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
