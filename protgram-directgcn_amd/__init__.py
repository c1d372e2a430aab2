"""protgram_directgcn_amd -- MI355X-native DirectGCN message passing.

Drop-in for the reference's hot path (``src/models/protgram_directgcn.py``): same class names,
constructor and ``forward()`` signatures, ``state_dict`` keys and init. Propagation and the dense
contraction run in hand-written gfx950 HIP kernels behind a C-ABI library (``csrc/``, loaded with
ctypes); there is no CPU fallback -- without the library the layer raises.
"""
from . import cluster, ngram, synth, train  # noqa: F401
from ._lib import load_library, library_path, NativeLibraryError  # noqa: F401
from .data import Data  # noqa: F401
from .graph import (CSRGraph, ShapedAdjacency, attach_ngram_map, build_ngram_map, build_propagation_csr,  # noqa: F401
                    csr_from_coo)
from .layer import DirectGCNLayer, ProtGramDirectGCN  # noqa: F401
