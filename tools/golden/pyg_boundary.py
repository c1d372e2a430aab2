"""Container-only restatement of the PyTorch-Geometric boundary the reference imports.

PyG (``torch_geometric``, unpinned pip dependency of the reference:
``unified_environment.yml:38``, ``tensorflow-pytorch-environment.txt:17``) is not
installed here and cannot be fetched. The reference's hot-path modules use exactly
four PyG symbols; this file restates their documented semantics (PyG >= 2.3) so
that ``src/models/protgram_directgcn.py`` and ``src/utils/graph_utils.py`` can be
imported unchanged to produce golden vectors:

* ``torch_geometric.data.Data``        -- attribute bag with ``.to(device)``
* ``torch_geometric.nn.MessagePassing`` -- ``aggr='add'``, flow source_to_target:
  ``x_j = x.index_select(0, ei[0])``; ``msg = self.message(x_j, **kw)``;
  ``out = msg.new_zeros(x.size(0), F).scatter_add_(0, ei[1], msg)``
* ``torch_geometric.utils.add_self_loops`` -- APPENDS ``arange(N)`` loops (even where
  a loop already exists), returns ``(edge_index, None)`` when no edge attr is given
* ``torch_geometric.utils.degree``      -- scatter-add of ones

Used only by ``tools/golden/make_golden.py`` in the build container. Never shipped,
never imported by the product or by tests.
"""
import sys
import types

import torch
import torch.nn as nn


class Data:
    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def to(self, device):
        for k, v in list(vars(self).items()):
            if torch.is_tensor(v):
                setattr(self, k, v.to(device))
        return self


class MessagePassing(nn.Module):
    def __init__(self, aggr='add'):
        super().__init__()
        assert aggr == 'add'
        self.aggr = aggr

    def propagate(self, edge_index, x, **kwargs):
        x_j = x.index_select(0, edge_index[0])
        msg = self.message(x_j, **kwargs)
        index = edge_index[1].view(-1, 1).expand_as(msg)
        return msg.new_zeros((x.size(0), msg.size(1))).scatter_add_(0, index, msg)

    def message(self, x_j, **kwargs):
        return x_j


def add_self_loops(edge_index, edge_attr=None, fill_value=None, num_nodes=None):
    n = int(num_nodes) if num_nodes is not None else int(edge_index.max()) + 1
    loop = torch.arange(n, dtype=edge_index.dtype, device=edge_index.device).view(1, -1).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1), None


def degree(index, num_nodes=None, dtype=None):
    n = int(num_nodes) if num_nodes is not None else int(index.max()) + 1
    out = torch.zeros((n,), dtype=dtype, device=index.device)
    one = torch.ones((index.numel(),), dtype=out.dtype, device=out.device)
    return out.scatter_add_(0, index, one)


def install():
    """Register the restated modules (and an empty h5py) in sys.modules."""
    tg = types.ModuleType('torch_geometric')
    tg_data = types.ModuleType('torch_geometric.data')
    tg_nn = types.ModuleType('torch_geometric.nn')
    tg_utils = types.ModuleType('torch_geometric.utils')
    tg_data.Data = Data
    tg_nn.MessagePassing = MessagePassing
    tg_utils.add_self_loops = add_self_loops
    tg_utils.degree = degree
    tg.data, tg.nn, tg.utils = tg_data, tg_nn, tg_utils
    sys.modules.update({'torch_geometric': tg, 'torch_geometric.data': tg_data,
                        'torch_geometric.nn': tg_nn, 'torch_geometric.utils': tg_utils})
    if 'h5py' not in sys.modules:
        try:
            import h5py  # noqa: F401
        except ImportError:
            sys.modules['h5py'] = types.ModuleType('h5py')
