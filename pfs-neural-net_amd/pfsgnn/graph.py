"""Drop-in for the reference ``src/graph.py``: fiber-galaxy property data ->
BipartiteData graphs, built on the device.

``to_Graph`` (graph.py:14-67) builds every fiber -> class edge of a complete
bipartite graph with Python loops and then sorts them by source id with
``torch.argsort``.  Here the edge_index is written in that sorted
(fiber-major) order directly into HBM by one kernel
(``pfsgnn_build_complete``, include/pfsgnn.h); the node / edge / global
feature tables are device tensors.  ``torch.argsort`` is not stable, so the
reference's order of a fiber's classes is implementation-defined
(``graphs/graph-0.pt`` holds one such order); the edge *set* per fiber, the
features and the graph's shape are the same, and every pfsgnn op accepts
either order (pfsgnn_layout_analyze).
"""
import os

import numpy as np
import torch

from . import config
from .gnn import BipartiteData, backend


def pad_properties(utils, fdim=None):
    """graph.py:77: class properties padded with zero columns up to Fdim."""
    fdim = config.Fdim if fdim is None else fdim
    utils = np.asarray(utils, dtype=np.float64)
    if utils.ndim == 1:
        utils = utils[:, None]
    if utils.shape[1] > fdim:
        raise ValueError(f"{utils.shape[1]} property columns exceed Fdim={fdim}")
    return np.hstack((utils, np.zeros((utils.shape[0], fdim - utils.shape[1]))))


def to_Graph(properties, nfibers=None, fdim=None):
    """graph.py:14-67.  properties [NCLASSES, F]: one feature row per class.
    Returns BipartiteData(edge_index [2, NFIBERS*NCLASSES] sorted by fiber,
    x_s zeros [NFIBERS, Fdim], x_t properties, edge_attr zeros [E, Fdim],
    u zeros [1, Fdim]) on the device."""
    nfibers = config.NFIBERS if nfibers is None else int(nfibers)
    fdim = config.Fdim if fdim is None else int(fdim)
    props = torch.as_tensor(np.asarray(properties), dtype=torch.float)
    if props.dim() != 2:
        raise ValueError("properties must be [NCLASSES, F]")
    nclasses = props.shape[0]
    dev = config.device
    edge_index = backend().build_complete(1, nfibers, nclasses, order=0)
    x_s = torch.zeros(nfibers, fdim, dtype=torch.float, device=dev)
    x_t = props.to(dev)
    edge_attr = torch.zeros(nfibers * nclasses, fdim, dtype=torch.float, device=dev)
    u = torch.zeros(1, fdim, dtype=torch.float, device=dev)
    return BipartiteData(edge_index, x_s, x_t, edge_attr, u)


def main(ngraph=1, datafile=None, outdir="../graphs"):
    """graph.py:70-83: load the utility properties, pad them to Fdim, build
    and save ``ngraph`` graphs.  Saved as a dict of tensors (loadable with
    ``torch.load(..., weights_only=True)``) rather than a pickled PyG object."""
    utils = np.loadtxt(config.datafile if datafile is None else datafile)
    props = pad_properties(utils)
    os.makedirs(outdir, exist_ok=True)
    paths = []
    for igraph in range(ngraph):
        g = to_Graph(props)
        path = os.path.join(outdir, f"graph-{igraph}.pt")
        torch.save({k: getattr(g, k).cpu() for k in ("edge_index", "x_s", "x_t", "x_e", "x_u")},
                   path)
        paths.append(path)
    return paths


if __name__ == "__main__":
    main()
