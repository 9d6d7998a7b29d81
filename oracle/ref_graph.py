"""CPU restatement of the reference graph builders.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

* ``to_graph``  -- graph.py:14-67 (``to_Graph``): complete fiber->class edges,
  class-major construction, then sorted by source id.  The reference sorts
  with ``torch.argsort`` (unstable, graph.py:49), so the order of a fiber's
  edges is implementation-defined: ``graphs/graph-0.pt`` holds one such
  order (e.g. fiber 0 -> classes 1,11,10,9,8,7,0,6,...).  This restatement
  uses a stable sort; tests compare edge *sets* per fiber with graph-0 and
  use graph-0's own edge_index verbatim for order-sensitive parity.
* ``train_graph`` -- train.py:88-104: x_s = fiber counter, x_t = class_info,
  ``torch.cartesian_prod`` edges (fiber-major), x_e ~ U[lo, hi), u = 0.
"""
import numpy as np
import torch


def to_graph(properties, nfibers, fdim):
    properties = np.asarray(properties, dtype=np.float64)
    nclasses = properties.shape[0]
    e_s = np.tile(np.arange(nfibers), nclasses)          # graph.py:41-45 (class-major)
    e_t = np.repeat(np.arange(nclasses), nfibers)
    edge_index = torch.tensor(np.stack([e_s, e_t]), dtype=torch.long)
    order = torch.argsort(edge_index[0], stable=True)   # graph.py:49 (stable here)
    edge_index = edge_index[:, order]
    edge_attr = torch.zeros(edge_index.shape[1], fdim)  # graph.py:46-50
    x_s = torch.zeros(nfibers, fdim)                    # graph.py:54
    x_t = torch.tensor(properties, dtype=torch.float)   # graph.py:55
    u = torch.zeros(1, fdim)                            # graph.py:56
    return edge_index, x_s, x_t, edge_attr, u


def pad_properties(utils, fdim):
    """graph.py:77 (``np.hstack`` with zeros up to Fdim columns)."""
    utils = np.asarray(utils, dtype=np.float64)
    return np.hstack((utils, np.zeros((utils.shape[0], fdim - utils.shape[1]))))


def train_graph(class_info, nfibers, fdim, lo=2.0, hi=10.0, generator=None):
    """train.py:88-104 on the CPU."""
    class_info = torch.as_tensor(class_info, dtype=torch.float)
    nclasses = class_info.shape[0]
    x_t = class_info                                                            # train.py:89
    x_s = torch.arange(nfibers, dtype=torch.float).reshape(-1, 1)               # train.py:91
    edge_index = torch.cartesian_prod(torch.arange(nfibers), torch.arange(nclasses)).T  # :94
    x_e = lo + (hi - lo) * torch.rand(size=(nfibers * nclasses, fdim), generator=generator)  # :100
    x_u = torch.zeros(1, fdim)                                                  # train.py:101
    return edge_index, x_s, x_t, x_e, x_u
