"""pfsgnn -- MI355X-native bipartite message-passing engine.

Drop-in for the hot path of joshua-lintropic/pfs-neural-net: the
``src/gnn.py`` operator surface (BipartiteData, MLP, EdgeModel, SModel,
TModel, GlobalModel, Block, GNN) and the ``src/train.py`` objective
(``softfloor``, ``loss_function``), computed by hand-written HIP kernels for
gfx950 in ``libpfsgnn.so`` (C ABI: ``include/pfsgnn.h``).
"""
from .native import NativeUnavailable, HipBackend, set_edge_path, get_edge_path  # noqa: F401
from .gnn import (BipartiteData, Loader, Batch, MLP, EdgeModel, SModel, TModel,  # noqa: F401
                  GlobalModel, Block, GNN)
from .train import softfloor, loss_function  # noqa: F401
from .optim import FusedAdam  # noqa: F401

__version__ = "0.1.0"
