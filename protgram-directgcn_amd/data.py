"""Minimal stand-in for ``torch_geometric.data.Data`` as used on the DirectGCN path.

The reference model reads ``x, edge_index_in, edge_weight_in, edge_index_out, edge_weight_out,
edge_index_undirected_norm, edge_weight_undirected_norm, original_indices`` with ``getattr(.., None)``
(``src/models/protgram_directgcn.py:196-203``) and the trainer moves it with ``.to(device)``
(``src/pipeline/protgram_directgcn_trainer.py:80``). Any object with those attributes (including a
real PyG ``Data``) is accepted by :class:`ProtGramDirectGCN`; this class exists so that PyG is not a
dependency.
"""
import torch


class Data:
    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def to(self, device, non_blocking: bool = False):
        for k, v in list(vars(self).items()):
            if torch.is_tensor(v):
                setattr(self, k, v.to(device, non_blocking=non_blocking))
            elif hasattr(v, "to") and hasattr(v, "tensors"):  # a prebuilt CSRGraph (data.graph)
                setattr(self, k, v.to(device))
        return self

    @property
    def num_nodes(self):
        n = vars(self).get("_num_nodes")
        if n is not None:
            return n
        x = getattr(self, "x", None)
        return None if x is None else x.size(0)

    @num_nodes.setter
    def num_nodes(self, n):
        self._num_nodes = n

    def __repr__(self):
        parts = [f"{k}={list(v.shape) if torch.is_tensor(v) else v}" for k, v in vars(self).items()]
        return f"Data({', '.join(parts)})"
