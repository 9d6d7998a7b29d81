"""CPU restatement of the reference training objective (``src/train.py``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

``softfloor`` follows train.py:21-27 except that its uniform noise is an
explicit argument (the reference draws ``torch.rand_like`` inside; the
product draws it from a counter-based generator, and the tests hand the same
numbers to both).  ``loss_function`` follows train.py:29-80 for one graph in
the fiber-major complete layout train.py builds (train.py:94, whose edge order
train.py:40 and :67 rely on); a batch of G such graphs is the sum of the G
per-graph losses (identical to the reference for G == 1).
"""
import math

import torch
import torch.nn as nn

from .ref_scatter import scatter


def softfloor(x, sharpness=20, noiselevel=0.3, uniform=None):
    """train.py:21-27.  ``uniform`` stands in for ``torch.rand_like(x)``."""
    if uniform is None:
        uniform = torch.rand_like(x)
    noise = noiselevel * (uniform - 0.5)
    x = x + noise
    sharpness = x.new_tensor(sharpness)
    pi = x.new_tensor(math.pi)
    r = torch.where(sharpness == 0, torch.tensor(0.0, dtype=x.dtype), torch.exp(-1 / sharpness))
    return x + 1 / pi * (torch.arctan(r * torch.sin(2 * pi * x) / (1 - r * torch.cos(2 * pi * x)))
                         - torch.arctan(r / (torch.ones_like(r) - r)))


def loss_function(gnn, x_e, class_info, G, NF, NC, pclass=0.1, pfiber=1.0, sharpness=0.5,
                  total_time=42.0, nfields=10, wutils=2000.0, wvar=1.0, uniform=None):
    """train.py:29-80 (finaloutput=True branch values are returned too).

    ``x_e``: final edge features [G*NF*NC, F] in fiber-major order.
    ``class_info``: [G*NC, >=2] (col 0 = T_i hours per visit, col 1 = N_i).
    Returns (loss, per-graph dict of diagnostics)."""
    time = gnn.edge_prediction(x_e, scale=total_time / NC).squeeze(-1)  # train.py:42
    ci = class_info.reshape(G, NC, -1)
    losses = []
    diag = {"utils": [], "n_prime": [], "fiber_time": [], "variance": []}
    for g in range(G):
        t = time[g * NF * NC:(g + 1) * NF * NC]
        T_i = ci[g, :, 0].unsqueeze(0).expand(NF, -1).reshape(-1)           # train.py:39-40
        N_i = ci[g, :, 1] / nfields                                          # train.py:41
        visited = t / T_i                                                    # train.py:43
        u = None if uniform is None else uniform[g * NF * NC:(g + 1) * NF * NC]
        galaxies = softfloor(visited, sharpness, uniform=u)                  # train.py:46
        galaxies = torch.maximum(torch.full_like(galaxies, 0.0), galaxies)  # train.py:47
        tgt = torch.arange(NC).repeat(NF)
        src = torch.arange(NF).repeat_interleave(NC)
        n_prime = scatter(galaxies, tgt, NC, reduce="sum")                   # train.py:48
        tt = galaxies * T_i                                                  # train.py:49
        completeness = n_prime / N_i                                         # train.py:53
        totutils = torch.min(completeness)                                   # train.py:54
        class_over = torch.relu(n_prime - N_i)                               # train.py:57
        class_penalty = pclass * torch.sum(class_over ** 2)
        fiber_time = scatter(tt, src, NF, reduce="sum")                      # train.py:61
        overtime = fiber_time - total_time
        leaky = nn.LeakyReLU(negative_slope=0.1)
        fiber_penalty = pfiber * torch.sum(leaky(overtime) ** 2)             # train.py:64
        Time = tt.reshape(NF, NC)                                            # train.py:67
        variance = torch.sum(torch.var(Time, dim=0))                         # train.py:68
        loss = -wutils * totutils + fiber_penalty + class_penalty - wvar * variance  # train.py:71
        losses.append(loss)
        diag["utils"].append(totutils.detach())
        diag["n_prime"].append(n_prime.detach())
        diag["fiber_time"].append(fiber_time.detach())
        diag["variance"].append(variance.detach())
    return torch.stack(losses).sum(), diag
