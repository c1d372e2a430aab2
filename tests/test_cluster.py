"""Cluster-GCN subgraph extraction (cluster.py) against the reference's per-cluster construction
(protgram_directgcn_trainer.py:172-197): PyG subgraph(cluster_nodes, ei, ew, relabel_nodes=True) restated
per cluster as a mask + relabel, on CPU. Host logic only (no kernels)."""
import collections

import pytest
import torch

from golden_util import graph, load


def _pyg_subgraph(nodes, ei, ew, n):
    """PyG utils.subgraph(subset=nodes, relabel_nodes=True): keep entries with both ends in the subset, in
    order; relabel to positions in `nodes`."""
    mask = torch.zeros(n, dtype=torch.bool)
    mask[nodes] = True
    keep = mask[ei[0]] & mask[ei[1]]
    idx = torch.full((n,), -1, dtype=torch.long)
    idx[nodes] = torch.arange(nodes.numel())
    return idx[ei[:, keep]], (ew[keep] if ew is not None else None)


def _reference_clusters(parts):
    clusters = collections.defaultdict(list)
    for node, cid in enumerate(parts.tolist()):
        clusters[cid].append(node)
    return [torch.tensor(c, dtype=torch.long) for c in clusters.values()]


@pytest.mark.parametrize("kind", ["random", "range", "range_sched"])
def test_build_subgraphs_matches_pyg_subgraph(pkg, kind):
    from protgram_directgcn_amd import cluster
    fx = load("f1_fasta2")
    ei, ew = graph(fx)
    n = int(fx["N"].item())
    g = torch.Generator().manual_seed(3)
    if kind == "random":
        parts = torch.randint(0, 7, (n,), generator=g) * 13 + 5  # arbitrary ids
    elif kind == "range":
        parts = cluster.range_clusters(n, cluster.cluster_count(n, target_nodes=60))
    else:
        N, s, d, c = pkg.synth.de_bruijn_edges(2)
        order = pkg.graph.locality_schedule(n, torch.from_numpy(s), torch.from_numpy(d)).long()
        parts = cluster.range_clusters(n, 6, order=order)
    x = torch.randn(n, 8, generator=g)
    y = torch.randint(0, 5, (n,), generator=g)
    subs = cluster.build_subgraphs(n, parts, ei["in"], ew["in"], ei["out"], ew["out"], ei["und"], ew["und"], x, y)
    ref = _reference_clusters(parts)
    assert len(subs) == len(ref)
    for d, nodes in zip(subs, ref):
        assert torch.equal(d.original_indices, nodes)
        assert torch.equal(d.x, x[nodes]) and torch.equal(d.y, y[nodes])
        for k, ik, wk in (("in", "edge_index_in", "edge_weight_in"), ("out", "edge_index_out", "edge_weight_out"),
                          ("und", "edge_index_undirected_norm", "edge_weight_undirected_norm")):
            rei, rew = _pyg_subgraph(nodes, ei[k], ew[k], n)
            assert torch.equal(getattr(d, ik), rei), (kind, k)
            assert torch.equal(getattr(d, wk), rew), (kind, k)
        # the attached CSR is the one csr_from_coo builds from the subgraph's COO
        want = pkg.graph.csr_from_coo(nodes.numel(), d.edge_index_in, d.edge_weight_in, d.edge_index_out,
                                      d.edge_weight_out, d.edge_index_undirected_norm, d.edge_weight_undirected_norm,
                                      cache=False) if d.edge_index_in.numel() else None
        if want is not None:
            for f in ("rowptr", "edges3", "rowptr_t", "edges3_t"):
                assert torch.equal(getattr(d.graph, f), getattr(want, f)), f
            assert d.graph.symmetric == want.symmetric
        else:
            assert d.graph.nnz == 0


def test_union_graph_is_block_diagonal(pkg):
    from protgram_directgcn_amd import cluster
    fx = load("f1_fasta2")
    ei, ew = graph(fx)
    n = int(fx["N"].item())
    parts = cluster.range_clusters(n, 5)
    x = torch.randn(n, 4)
    subs = cluster.build_subgraphs(n, parts, ei["in"], ew["in"], ei["out"], ew["out"], ei["und"], ew["und"], x)
    u = cluster.union_graph(subs)
    assert u.n_rows == n and u.nnz == sum(d.graph.nnz for d in subs)
    off = 0
    for d in subs:  # every row's columns stay inside its own cluster's block
        rp = u.rowptr[off:off + d.graph.n_rows + 1]
        cols = u.edges3[int(rp[0]):int(rp[-1]), 0]
        assert bool(((cols >= off) & (cols < off + d.graph.n_rows)).all())
        off += d.graph.n_rows


def test_cluster_count_rule():
    from protgram_directgcn_amd import cluster
    assert cluster.cluster_count(160000) == 320   # 4-gram: ceil(N/500)
    assert cluster.cluster_count(400) == 2        # GCN_MIN_CLUSTERS
    assert cluster.cluster_count(3200000) == 500  # GCN_MAX_CLUSTERS


def test_layout_is_first_appearance_order():
    from protgram_directgcn_amd import cluster
    parts = torch.tensor([9, 4, 9, 7, 4, 7, 1])
    lay = cluster.layout_of(parts)
    assert lay.nodes.tolist() == [0, 2, 1, 4, 3, 5, 6]
    assert lay.ptr.tolist() == [0, 2, 4, 6, 7]
