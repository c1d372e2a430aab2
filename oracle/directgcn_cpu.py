"""ORACLE (test infrastructure only): fp32 CPU restatement of the reference DirectGCN path.

Every function restates, op for op and in the same order, the reference code it cites, so that its
results equal the reference's on the same inputs (bit-exact on the golden fixtures; see
``tests/test_oracle_golden.py``). It runs on ATen CPU kernels, i.e. it IS the reference's CPU
algorithm (index_select -> mul -> scatter_add_ per propagate), which is why ``bench.py`` times it as
the ``cpu_baseline`` ("port").

Parameters are passed as a dict keyed like the reference ``state_dict`` (e.g. ``lin_main_in.weight``,
``C_in_vec``, ``constant``; model keys ``convs.{i}.*``, ``res_projs.{i}.*``, ``decoder_fc.{0,3}.*``,
``pe_layer.weight``). Tensors may require grad: autograd through these functions gives the
reference's gradients.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------------------------
# PyG boundary (third-party, not vendored): MessagePassing(aggr='add').propagate, flow
# source_to_target, PyG >= 2.3 sum path; message() = protgram_directgcn.py:137-140.
# --------------------------------------------------------------------------------------------
def propagate(edge_index: torch.Tensor, x: torch.Tensor, edge_weight: Optional[torch.Tensor]) -> torch.Tensor:
    x_j = x.index_select(0, edge_index[0])
    msg = x_j if edge_weight is None else edge_weight.view(-1, 1) * x_j
    index = edge_index[1].view(-1, 1).expand_as(msg)
    return msg.new_zeros((x.size(0), msg.size(1))).scatter_add_(0, index, msg)


class _RowChunkedPropagate(torch.autograd.Function):
    """``propagate`` evaluated over consecutive chunks of entries (each chunk index_select -> mul ->
    scatter_add_ into the same output, in entry order), with the autograd rule of those three ops written out:
    grad of scatter_add_ = gather of the output gradient at ei[1], times w (mul), index_add_ at ei[0]
    (index_select). Chunk boundaries fall between destination rows when ei[1] is sorted, so every output
    element receives its terms in the same order as the one-shot ``propagate``: the forward is identical to it
    (tested on the golden graphs) while only one chunk's [chunk, F] message tensor exists at a time and
    autograd saves no [nnz, F] tensors -- what makes 4-/5-gram autograd runs fit in host memory."""

    @staticmethod
    def forward(ctx, x, edge_index, edge_weight, bounds):
        out = x.new_zeros((x.size(0), x.size(1)))
        for a, b in zip(bounds[:-1], bounds[1:]):
            src, dst = edge_index[0, a:b], edge_index[1, a:b]
            x_j = x.index_select(0, src)
            msg = x_j if edge_weight is None else edge_weight[a:b].view(-1, 1) * x_j
            out.scatter_add_(0, dst.view(-1, 1).expand_as(msg), msg)
        ctx.save_for_backward(edge_index, edge_weight if edge_weight is not None else x.new_empty(0))
        ctx.has_w, ctx.bounds, ctx.n = edge_weight is not None, bounds, x.size(0)
        return out

    @staticmethod
    def backward(ctx, gout):
        edge_index, w = ctx.saved_tensors
        gx = gout.new_zeros((ctx.n, gout.size(1)))
        for a, b in zip(ctx.bounds[:-1], ctx.bounds[1:]):
            g = gout.index_select(0, edge_index[1, a:b])
            if ctx.has_w:
                g = w[a:b].view(-1, 1) * g
            gx.index_add_(0, edge_index[0, a:b], g)
        return gx, None, None, None


def row_chunk_bounds(edge_index: torch.Tensor, chunk: int) -> list:
    """Entry offsets [0, ..., nnz] at most ~chunk apart, each moved forward to the next change of ei[1] (a
    destination-row boundary when ei[1] is sorted; one chunk otherwise)."""
    nnz = edge_index.size(1)
    dst = edge_index[1]
    if nnz <= chunk or bool((dst[1:] < dst[:-1]).any()):
        return [0, nnz]
    cuts = torch.arange(chunk, nnz, chunk)
    cuts = torch.searchsorted(dst, dst[cuts], right=True)  # first entry of the next destination row
    return sorted({0, nnz, *[int(c) for c in cuts if 0 < int(c) < nnz]})


def propagate_chunked(edge_index: torch.Tensor, x: torch.Tensor, edge_weight: Optional[torch.Tensor],
                      chunk: int = 1 << 21) -> torch.Tensor:
    """``propagate`` with bounded memory (see _RowChunkedPropagate); same values and gradients."""
    return _RowChunkedPropagate.apply(x, edge_index, edge_weight, row_chunk_bounds(edge_index, chunk))


def linear(x, w, b=None):
    return F.linear(x, w, b)


# --------------------------------------------------------------------------------------------
# DirectGCNLayer.forward -- src/models/protgram_directgcn.py:93-135
# --------------------------------------------------------------------------------------------
def layer_forward(p: dict, x, ei_in, ew_in, ei_out, ew_out, ei_u, ew_u, original_indices=None,
                  use_vector_coeffs: bool = True, prefix: str = "", prop=propagate):
    """``prop``: ``propagate`` (the reference's PyG path) or ``propagate_chunked`` (same values and gradients,
    bounded memory, for the 4-/5-gram sizes)."""
    g = lambda k: p[prefix + k]  # noqa: E731
    propagate = prop
    # the reference layer drops to scalar coefficients when num_nodes == 0 (:48-60)
    use_vector_coeffs = use_vector_coeffs and (prefix + "C_in_vec") in p
    # :101-103
    h_main_in = propagate(ei_in, linear(x, g("lin_main_in.weight")), ew_in)
    h_shared_in = propagate(ei_in, linear(x, g("lin_shared.weight")), ew_in)
    ic = (h_main_in + g("bias_main_in")) + (h_shared_in + g("bias_directed_shared_in"))
    # :106-108
    h_main_out = propagate(ei_out, linear(x, g("lin_main_out.weight")), ew_out)
    h_shared_out = propagate(ei_out, linear(x, g("lin_shared.weight")), ew_out)
    oc = (h_main_out + g("bias_main_out")) + (h_shared_out + g("bias_directed_shared_out"))
    # :111-113
    h_main_u = propagate(ei_u, linear(x, g("lin_undirected.weight")), ew_u)
    h_shared_u = propagate(ei_u, linear(x, g("lin_shared.weight")), ew_u)
    uc = (h_main_u + g("bias_undirected")) + (h_shared_u + g("bias_undirected_shared"))
    # :116-128
    const = p.get(prefix + "constant")
    if use_vector_coeffs and original_indices is not None:
        oi = original_indices
        c_in, c_out = g("C_in_vec")[oi], g("C_out_vec")[oi]
        c_dir, c_u, c_all = g("C_directed_vec")[oi], g("C_undirected_vec")[oi], g("C_all_vec")[oi]
        const_t = const[oi] if const is not None else 0
    elif use_vector_coeffs:
        c_in, c_out = g("C_in_vec"), g("C_out_vec")
        c_dir, c_u, c_all = g("C_directed_vec"), g("C_undirected_vec"), g("C_all_vec")
        const_t = const if const is not None else 0
    else:
        c_in, c_out, c_dir, c_u, c_all = g("C_in"), g("C_out"), g("C_directed"), g("C_undirected"), g("C_all")
        const_t = 0
    # :131-133
    directed = c_dir * ((c_in * ic) + (c_out * oc))
    undirected = c_u * uc
    return (c_all * (undirected + directed)) + const_t


def l2_normalize(x, eps=1e-12):
    """EmbeddingProcessor.l2_normalize_torch, src/utils/models_utils.py:139-147 (eps added to the norm)."""
    if x.ndim == 1:
        return x / (torch.norm(x, p=2, keepdim=True) + eps)
    return x / (torch.norm(x, p=2, dim=1, keepdim=True) + eps)


def apply_pe(p: dict, x, n_gram_len: int, one_gram_dim: int):
    """ProtGramDirectGCN._apply_pe, protgram_directgcn.py:182-193, written out-of-place (the reference's
    in-place add raises under autograd when x does not require grad; values are identical)."""
    w = p.get("pe_layer.weight")
    if w is None:
        return x
    if n_gram_len > 0 and one_gram_dim > 0 and x.shape[1] == n_gram_len * one_gram_dim:
        pos = min(n_gram_len, w.shape[0])
        xr = x.view(-1, n_gram_len, one_gram_dim)
        if pos > 0:
            add = torch.zeros(n_gram_len, one_gram_dim, dtype=x.dtype)
            add = torch.cat([w[:pos], add[pos:]], 0)
            xr = xr + add.unsqueeze(0)
        return xr.reshape(-1, n_gram_len * one_gram_dim)
    return x


def model_forward(p: dict, layer_dims, x, ei_in, ew_in, ei_out, ew_out, ei_u, ew_u, original_indices=None,
                  n_gram_len: int = 0, one_gram_dim: int = 0, use_vector_coeffs: bool = True,
                  training: bool = False, dropout: float = 0.5, l2_eps: float = 1e-12, prop=propagate,
                  act_masks=None, pre_acts=None):
    """ProtGramDirectGCN.forward, protgram_directgcn.py:195-222 (eval: dropout inactive).

    ``act_masks`` (tests only): per layer, a boolean [N, F] mask choosing leaky_relu's branch instead of the sign of
    this computation's own pre-activation -- F.leaky_relu's formula (v if v > 0 else 0.01 v) on a given branch.
    Comparing two fp32 computations of the same model, a pre-activation within rounding of 0 can fall on either
    side of the kink and change that element's gradient by 100x; passing the other computation's branches
    compares the two on the same piecewise-linear function. An extra last mask does the same for the decoder's
    ReLU (where a hidden unit within rounding of 0 switches a whole term of that row's gradient on or off).
    ``pre_acts`` (tests only): a list that receives this computation's own pre-activations (each layer's, then the
    decoder's), so a test can check that the masks it passed disagree with their signs only within rounding of 0."""
    h = apply_pe(p, x, n_gram_len, one_gram_dim)
    for i in range(len(layer_dims) - 1):
        h_res = h
        out = layer_forward(p, h_res, ei_in, ew_in, ei_out, ew_out, ei_u, ew_u, original_indices,
                            use_vector_coeffs, prefix=f"convs.{i}.", prop=prop)
        if f"res_projs.{i}.weight" in p:
            res = linear(h_res, p[f"res_projs.{i}.weight"], p[f"res_projs.{i}.bias"])
        else:
            res = h_res
        z = out + res
        if pre_acts is not None:
            pre_acts.append(z.detach())
        h = F.leaky_relu(z) if act_masks is None else torch.where(act_masks[i], z, z * 0.01)
        h = F.dropout(h, p=dropout, training=training)
    z = linear(h, p["decoder_fc.0.weight"], p["decoder_fc.0.bias"])
    if pre_acts is not None:
        pre_acts.append(z.detach())
    nl = len(layer_dims) - 1
    z = F.relu(z) if act_masks is None or len(act_masks) <= nl else torch.where(act_masks[nl], z, z * 0)
    z = F.dropout(z, p=0.5, training=training)
    logits = linear(z, p["decoder_fc.3.weight"], p["decoder_fc.3.bias"])
    return F.log_softmax(logits, dim=-1), l2_normalize(h, eps=l2_eps)
