"""Drop-in ``DirectGCNLayer`` / ``ProtGramDirectGCN`` (reference: ``src/models/protgram_directgcn.py``).

Same constructor and ``forward()`` signatures, parameter names (so ``state_dict`` round-trips with the
reference), parameter creation order (so ``torch.manual_seed`` gives the reference's init), and error
behaviour. The arithmetic runs in the gfx950 kernels of ``libpgdgcn.so``:

  layer forward = the 3 adjacencies in one pass (replaces the 6 propagate calls): pg_spmm3_ngram_mid_f32 on
                  complete n-gram graphs (the mapped variant + a residual CSR pass on builder-produced levels),
                  pg_spmm3_f32 (bit-exact CSR kernel) on any other graph
                + pg_directgcn_dense_f32 (the 6 Linear calls, biases, gates, constant on MFMA)

``ProtGramDirectGCN`` additionally fuses the residual, ``leaky_relu`` and (training) the dropout of each block into
the dense kernel's epilogue. In inference the decoder, log_softmax and the L2 normalisation run in one kernel
(pg_directgcn_head_f32); in training ``train.train_step`` runs the head's forward and backward in one kernel
(pg_head_train_f32 at F = 128, pg_head_train_bf16 in bf16 mode at F = 256), and autograd runs the framework ops
(ops.row_linear, log_softmax) for every other shape.
"""
from __future__ import annotations

import weakref
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .graph import csr_from_coo, _single, _key

_ROWS_OK: dict = {}


def _check_rows(rows: torch.Tensor, limit: int):
    """Range check of original_indices (the dense kernel gathers gates/constant rows by them), cached per
    tensor: the entry holds a weak reference to the tensor, so a new tensor at a reused address never hits it and
    the cache keeps no index tensor alive."""
    k = _key(rows, n=limit)
    hit = _ROWS_OK.get(k)
    if hit is not None and hit() is rows:
        return
    if rows.numel():
        lo, hi = int(rows.min()), int(rows.max())
        if lo < 0 or hi >= limit:
            raise IndexError(f"original_indices in [{lo}, {hi}] outside [0, {limit})")
    if len(_ROWS_OK) > 64:
        _ROWS_OK.clear()
    _ROWS_OK[k] = weakref.ref(rows)


class DirectGCNLayer(nn.Module):
    """Hierarchical-gated directed/undirected GCN layer (protgram_directgcn.py:20-140).

    The reference subclasses PyG ``MessagePassing(aggr='add')``; this class provides the same
    ``propagate``/``message`` semantics natively (``propagate`` runs ``pg_spmm1_f32``)."""

    def __init__(self, in_channels: int, out_channels: int, num_nodes: int, use_vector_coeffs: bool = True):
        super().__init__()
        self.aggr = "add"
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_nodes = num_nodes
        self.use_vector_coeffs = use_vector_coeffs
        # creation order = reference order (:34-66): nn.Linear draws from the global RNG on construction
        self.lin_main_in = nn.Linear(in_channels, out_channels, bias=False)
        self.lin_main_out = nn.Linear(in_channels, out_channels, bias=False)
        self.lin_undirected = nn.Linear(in_channels, out_channels, bias=False)
        self.bias_main_in = nn.Parameter(torch.empty(out_channels))
        self.bias_main_out = nn.Parameter(torch.empty(out_channels))
        self.bias_undirected = nn.Parameter(torch.empty(out_channels))
        self.lin_shared = nn.Linear(in_channels, out_channels, bias=False)
        self.bias_directed_shared_in = nn.Parameter(torch.empty(out_channels))
        self.bias_directed_shared_out = nn.Parameter(torch.empty(out_channels))
        self.bias_undirected_shared = nn.Parameter(torch.empty(out_channels))
        if self.use_vector_coeffs and self.num_nodes > 0:
            self.C_in_vec = nn.Parameter(torch.empty(num_nodes, 1))
            self.C_out_vec = nn.Parameter(torch.empty(num_nodes, 1))
            self.C_directed_vec = nn.Parameter(torch.empty(num_nodes, 1))
            self.C_undirected_vec = nn.Parameter(torch.empty(num_nodes, 1))
            self.C_all_vec = nn.Parameter(torch.empty(num_nodes, 1))
        else:
            self.use_vector_coeffs = False
            self.C_in = nn.Parameter(torch.empty(1))
            self.C_out = nn.Parameter(torch.empty(1))
            self.C_directed = nn.Parameter(torch.empty(1))
            self.C_undirected = nn.Parameter(torch.empty(1))
            self.C_all = nn.Parameter(torch.empty(1))
        if self.num_nodes > 0:
            self.constant = nn.Parameter(torch.empty(num_nodes, out_channels))
        else:
            self.constant = None
        self.reset_parameters()

    def reset_parameters(self):
        # :70-91
        for lin in [self.lin_main_in, self.lin_main_out, self.lin_shared, self.lin_undirected]:
            nn.init.xavier_uniform_(lin.weight)
        for bias in [self.bias_main_in, self.bias_main_out, self.bias_directed_shared_in,
                     self.bias_directed_shared_out, self.bias_undirected, self.bias_undirected_shared]:
            nn.init.zeros_(bias)
        if self.use_vector_coeffs:
            for c in (self.C_in_vec, self.C_out_vec, self.C_directed_vec, self.C_undirected_vec, self.C_all_vec):
                nn.init.ones_(c)
        else:
            for c in (self.C_in, self.C_out, self.C_directed, self.C_undirected, self.C_all):
                nn.init.ones_(c)
        if self.constant is not None:
            nn.init.xavier_uniform_(self.constant)

    # --- PyG MessagePassing surface -------------------------------------------------------------
    def message(self, x_j: torch.Tensor, edge_weight: Optional[torch.Tensor]) -> torch.Tensor:
        if edge_weight is None:
            return x_j
        return edge_weight.view(-1, 1) * x_j

    def propagate(self, edge_index: torch.Tensor, x: torch.Tensor, edge_weight: Optional[torch.Tensor] = None):
        """out[ei[1]] += w * x[ei[0]] with out rows = x.size(0) (PyG aggr='add')."""
        ops._require_gpu(x, edge_index)
        k = ("p1",) + _key(edge_index, edge_weight, n=x.size(0))
        hit = _P1_CACHE.get(k)
        if hit is None:
            a = _single(edge_index, edge_weight, x.size(0))
            if len(_P1_CACHE) > 16:
                _P1_CACHE.clear()
            _P1_CACHE[k] = ((edge_index, edge_weight), a)  # holds its keys (no stale address reuse)
        else:
            a = hit[1]
        return ops.Propagate1.apply(x, a)

    # --- forward ----------------------------------------------------------------------------------
    def _dense_params(self):
        if self.use_vector_coeffs:
            C = (self.C_in_vec, self.C_out_vec, self.C_directed_vec, self.C_undirected_vec, self.C_all_vec)
        else:
            C = (self.C_in, self.C_out, self.C_directed, self.C_undirected, self.C_all)
        return (self.lin_main_in.weight, self.lin_main_out.weight, self.lin_undirected.weight, self.lin_shared.weight,
                self.bias_main_in, self.bias_directed_shared_in, self.bias_main_out, self.bias_directed_shared_out,
                self.bias_undirected, self.bias_undirected_shared, *C)

    def fused_forward(self, x, graph, original_indices=None, res_x=None, W_res=None, b_res=None, act=False,
                      fused_norm: bool = False, drop=None):
        """Layer output (+ optional residual and leaky_relu) from a prepared CSRGraph. drop = (p, seed): the dropout
        the model applies to the layer's output (protgram_directgcn.py:216), fused into the dense epilogue (act only;
        seed a device int64 [1])."""
        if drop is not None and not act:
            raise ValueError("fused dropout needs the activation")
        M = x.size(0)
        rows = None
        if self.use_vector_coeffs:
            if original_indices is not None:
                rows = original_indices.to(device=x.device, dtype=torch.int64)
                if rows.numel() != M:
                    raise ValueError("original_indices must have one entry per row of x")
                _check_rows(rows, self.num_nodes)
            elif self.num_nodes != M:
                raise RuntimeError(f"vector coefficients hold {self.num_nodes} nodes but x has {M} rows "
                                   "(pass original_indices for subgraphs)")
        if graph.n_rows != M:
            raise ValueError("graph rows != x rows")
        constant = self.constant if self.use_vector_coeffs else None
        gate_mode = 0 if self.use_vector_coeffs else 1
        params = self._dense_params()
        if (ops.PREGATED_INFERENCE and rows is None and not fused_norm
                and not (torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)))):
            # inference: the gates are applied by the propagation's store (pg_spmm3_gated_f32) and the dense kernel
            # takes the pre-gated operand (W-stationary kernel where the shape allows)
            prm = dict(zip(ops._DENSE_KEYS, params))
            Z = ops.spmm3_gated(graph, x, prm, gate_mode)
            if Z is not None:
                return ops.layer_dense(Z, prm, gate_mode, constant=constant, res_x=res_x, W_res=W_res, b_res=b_res,
                                       act=act, pregated=True, drop=drop)
        if (ops.SPAN_BACKWARD and torch.is_grad_enabled() and x.requires_grad
                and ops.PropagateDense.supports(graph, x, self.out_channels, res_x, W_res, rows, fused_norm)):
            # training through a layer whose input needs its gradient: the input's whole gradient (diagonal term and
            # identity residual from the dense backward, off-diagonal part accumulated into it) in two launches
            return ops.PropagateDense.apply(x, graph, res_x is not None, constant, gate_mode, act, ops.LEAKY_SLOPE,
                                            drop, *params)
        Z = ops.Propagate3.apply(x, graph, fused_norm)
        return ops.LayerDense.apply(Z, res_x, constant, W_res, b_res, rows, gate_mode, act, ops.LEAKY_SLOPE, drop,
                                    *params)

    def forward(self, x: torch.Tensor,
                edge_index_in: torch.Tensor, edge_weight_in: Optional[torch.Tensor],
                edge_index_out: torch.Tensor, edge_weight_out: Optional[torch.Tensor],
                edge_index_undirected: torch.Tensor, edge_weight_undirected: Optional[torch.Tensor],
                original_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        ops._require_gpu(x, edge_index_in, edge_index_out, edge_index_undirected)
        g = csr_from_coo(x.size(0), edge_index_in, edge_weight_in, edge_index_out, edge_weight_out,
                         edge_index_undirected, edge_weight_undirected)
        return self.fused_forward(x, g, original_indices)


_P1_CACHE: dict = {}


class ProtGramDirectGCN(nn.Module):
    """The model wrapper (protgram_directgcn.py:143-222)."""

    def __init__(self, layer_dims: List[int], num_graph_nodes: Optional[int],
                 task_num_output_classes: int, n_gram_len: int,
                 one_gram_dim: int, max_pe_len: int, dropout: float,
                 use_vector_coeffs: bool, l2_eps: float = 1e-12):
        super().__init__()
        self.n_gram_len = n_gram_len
        self.one_gram_dim = one_gram_dim
        self.dropout = dropout
        self.l2_eps = l2_eps
        self.pe_layer = None
        if one_gram_dim > 0 and max_pe_len > 0:
            self.pe_layer = nn.Embedding(max_pe_len, one_gram_dim)
        self.convs = nn.ModuleList()
        self.res_projs = nn.ModuleList()
        if not layer_dims or len(layer_dims) < 2:
            raise ValueError("layer_dims must contain at least input and output dimensions (length >= 2).")
        for i in range(len(layer_dims) - 1):
            in_dim, out_dim = layer_dims[i], layer_dims[i + 1]
            current_num_nodes = num_graph_nodes if num_graph_nodes is not None else 0
            effective = use_vector_coeffs and current_num_nodes > 0
            self.convs.append(DirectGCNLayer(in_dim, out_dim, current_num_nodes, effective))
            self.res_projs.append(nn.Linear(in_dim, out_dim) if in_dim != out_dim else nn.Identity())
        final_dim = layer_dims[-1]
        hidden = final_dim // 2 if final_dim > 1 else 1
        self.decoder_fc = nn.Sequential(nn.Linear(final_dim, hidden), nn.ReLU(), nn.Dropout(p=0.5),
                                        nn.Linear(hidden, task_num_output_classes))
        self.fused_norm = False  # use pg_spmm3_fusednorm_f32 when the graph carries raw counts
        # torch.float32 (default, the reference's CPU precision) or torch.bfloat16 (bf16 storage of features,
        # aggregates and activations with fp32 accumulation; BASELINE config 5). Not part of the state_dict.
        self.compute_dtype = torch.float32

    def _apply_pe(self, x: torch.Tensor) -> torch.Tensor:
        """:182-193, out of place (the reference's in-place add fails under autograd when x has no grad)."""
        if self.pe_layer is None:
            return x
        if self.n_gram_len > 0 and self.one_gram_dim > 0 and x.shape[1] == self.n_gram_len * self.one_gram_dim:
            pos = min(self.n_gram_len, self.pe_layer.num_embeddings)
            xr = x.view(-1, self.n_gram_len, self.one_gram_dim)
            if pos > 0:
                pe = self.pe_layer(torch.arange(0, pos, device=x.device, dtype=torch.long))
                pad = pe.new_zeros(self.n_gram_len - pos, self.one_gram_dim)
                xr = xr + torch.cat([pe, pad], 0).unsqueeze(0)
            return xr.reshape(-1, self.n_gram_len * self.one_gram_dim)
        return x

    def graph_of(self, data):
        """CSRGraph for a Data object: a prebuilt ``data.graph`` (build_propagation_csr) or the COO inputs."""
        g = getattr(data, "graph", None)
        if g is not None:
            x = getattr(data, "x", None)
            if x is not None and g.device != x.device:
                g = g.to(x.device)  # e.g. a PyG Data moved with .to(), which leaves non-tensor attributes
                data.graph = g
            return g
        x = data.x
        return csr_from_coo(x.size(0), data.edge_index_in, getattr(data, "edge_weight_in", None),
                            data.edge_index_out, getattr(data, "edge_weight_out", None),
                            data.edge_index_undirected_norm, getattr(data, "edge_weight_undirected_norm", None))

    def forward(self, data) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.head(self.body(data))

    def body(self, data) -> torch.Tensor:
        """The layers (protgram_directgcn.py:195-216): h before the prediction head."""
        x = getattr(data, "x", None)
        ei_in = getattr(data, "edge_index_in", None)
        ei_out = getattr(data, "edge_index_out", None)
        ei_undir = getattr(data, "edge_index_undirected_norm", None)
        original_indices = getattr(data, "original_indices", None)
        has_graph = getattr(data, "graph", None) is not None
        if x is None or (not has_graph and (ei_in is None or ei_out is None or ei_undir is None)):
            raise ValueError("ProtGramDirectGCN requires 'x', 'edge_index_in', 'edge_index_out', and "
                             "'edge_index_undirected_norm' in the Data object.")
        ops._require_gpu(x)
        g = self.graph_of(data)
        h = self._apply_pe(x)
        if self.compute_dtype == torch.bfloat16:
            h = self.bf16_input(h) if (h is x and h.dtype != torch.bfloat16 and not h.requires_grad) else h.to(
                torch.bfloat16)
        elif self.compute_dtype != torch.float32:
            raise ValueError("compute_dtype must be torch.float32 or torch.bfloat16")
        # the dropout after each layer: fused into the dense epilogue (ops.FUSED_DROPOUT; one device draw of the
        # layers' seeds per forward), else F.dropout
        p = float(self.dropout) if self.training else 0.0
        seeds = None
        if ops.FUSED_DROPOUT and 0.0 < p < 1.0:
            seeds = torch.randint(0, 1 << 62, (len(self.convs),), device=x.device, dtype=torch.int64)
        for i, (conv, res) in enumerate(zip(self.convs, self.res_projs)):
            drop = (p, seeds[i:i + 1]) if seeds is not None else None
            if isinstance(res, nn.Linear):
                h = conv.fused_forward(h, g, original_indices, res_x=h, W_res=res.weight, b_res=res.bias, act=True,
                                       fused_norm=self.fused_norm, drop=drop)
            else:
                h = conv.fused_forward(h, g, original_indices, res_x=h, act=True, fused_norm=self.fused_norm,
                                       drop=drop)
            if drop is None:
                h = F.dropout(h, p=self.dropout, training=self.training)
        return h

    _xb = None

    def bf16_input(self, x: torch.Tensor) -> torch.Tensor:
        """bf16 copy of a step-invariant input (no PE, no gradient) in bf16 mode: converted once and again only when x
        changes (another tensor, or a new version counter: copy_ and in-place writes bump it), in place, so a captured
        step reads the refreshed values at the same address (train.GraphedTrainStep calls this before each replay).
        The per-step conversion was a 35 us pass of config 5's training step."""
        c = self._xb
        if c is not None and c[0]() is x and c[1] == x._version:
            return c[2]
        if c is not None and c[2].shape == x.shape and c[2].device == x.device:
            xb = c[2]
            xb.copy_(x)
        else:
            xb = x.to(torch.bfloat16)
        import weakref
        self._xb = (weakref.ref(x), x._version, xb)
        return xb

    def head_train_args(self):
        """(W1, b1, W2, b2, dropout p) of the decoder when ops.head_train takes it (Linear, ReLU, Dropout, Linear),
        else None."""
        dec = self.decoder_fc
        if not (len(dec) == 4 and isinstance(dec[0], nn.Linear) and isinstance(dec[1], nn.ReLU) and
                isinstance(dec[2], nn.Dropout) and isinstance(dec[3], nn.Linear)):
            return None
        return dec[0].weight, dec[0].bias, dec[3].weight, dec[3].bias, dec[2].p if self.training else 0.0

    def head(self, h, need_emb: bool = True):
        """decoder_fc -> log_softmax, and l2_normalize (protgram_directgcn.py:218-222). Inference (eval, no
        autograd) runs the fused pg_directgcn_head_f32 kernel; training runs the decoder Linears through
        ops.row_linear (weight gradients in pg_gemm_at_b_f32). need_emb=False (a trainer whose loss reads only the
        log-probs) returns (log_probs, None) on the training path: the embeddings take no part in the loss."""
        dec = self.decoder_fc
        if not self.training and not torch.is_grad_enabled() and h.is_cuda:
            return ops.head(h, dec[0].weight, dec[0].bias, dec[3].weight, dec[3].bias, self.l2_eps)
        h = h.float()  # bf16 mode: the decoder and the embeddings are computed in fp32
        if h.is_cuda and len(dec) == 4 and isinstance(dec[0], nn.Linear) and isinstance(dec[3], nn.Linear):
            a = dec[2](dec[1](ops.row_linear(h, dec[0].weight, dec[0].bias)))  # Linear, ReLU, Dropout
            logits = ops.row_linear(a, dec[3].weight, dec[3].bias)
        else:
            logits = dec(h)
        if not need_emb:
            return F.log_softmax(logits, dim=-1), None
        emb = h / (torch.norm(h, p=2, dim=1, keepdim=True) + self.l2_eps)  # models_utils.py:139-147
        return F.log_softmax(logits, dim=-1), emb
