"""Restatement of ``torch_scatter.scatter`` as used by the reference.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

The reference imports ``from torch_scatter import scatter, scatter_mean``
(gnn.py:4, train.py:4).  torch_scatter (pinned by the reference README to the
``torch-2.7.0`` wheel index) is not installed in this image, so its published
semantics are restated here:

* ``scatter(src, index, dim=0, dim_size=N, reduce='sum')``: ``out[i] = sum of
  src[j] with index[j] == i``; rows with no entries are 0.
* ``reduce='mean'``: the sum divided by ``count.clamp(min=1)`` (torch_scatter
  ``scatter_mean``), so empty rows are 0, not NaN.

Call sites this covers: gnn.py:140-144 (SModel mean/var/skew/kurt over
source nodes), gnn.py:190 (TModel sum over target nodes), train.py:48
(n_prime per class), train.py:61 (fiber_time per fiber).
"""
import torch


def scatter_sum(src, index, dim_size):
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    return out.index_add(0, index, src)


def scatter_mean(src, index, dim_size):
    total = scatter_sum(src, index, dim_size)
    ones = torch.ones(index.shape[0], dtype=src.dtype, device=src.device)
    count = scatter_sum(ones, index, dim_size).clamp(min=1)
    if src.dim() > 1:
        count = count.view((-1,) + (1,) * (src.dim() - 1))
    return total / count


def scatter(src, index, dim_size, reduce="sum"):
    if reduce == "sum":
        return scatter_sum(src, index, dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim_size)
    raise ValueError(reduce)
