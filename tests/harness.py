"""Shared builders for parity tests (test infrastructure)."""
import numpy as np
import torch

from oracle.ref_gnn import GNN as OracleGNN, Graph as OracleGraph


def canonical_edges(G, NF, NC):
    """train.py's fiber-major edge order (g*NF + f)*NC + c (train.py:94, batched)."""
    e = torch.arange(G * NF * NC)
    src = e // NC
    tgt = (e // (NF * NC)) * NC + e % NC
    return torch.stack([src, tgt])


def to_canonical(x, G, NF, NC):
    """Fiber-major [E, F] edge tensor -> the kernels' class-major channel-major [F, E]
    (canonical e = (g*NC + c)*NF + f)."""
    F = x.shape[1]
    return x.reshape(G, NF, NC, F).permute(3, 0, 2, 1).reshape(F, -1).contiguous()


def from_canonical(xc, G, NF, NC):
    """Inverse of to_canonical."""
    F = xc.shape[0]
    return xc.reshape(F, G, NC, NF).permute(1, 3, 2, 0).reshape(-1, F).contiguous()


def make_problem(G, NF, NC, F=10, B=2, Fs=1, Ft=2, T=12, seed=0, dtype=torch.float64, normed=True):
    """Random model + batched train.py-style inputs (train.py:88-104)."""
    gen = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    model = OracleGNN(B=B, Fdim=F, T=T, F_s=Fs, F_t=Ft, normed=normed).to(dtype)
    with torch.no_grad():
        for name, prm in model.named_parameters():
            if name.endswith("norm.weight"):
                prm.copy_(0.5 + torch.rand(prm.shape, generator=gen, dtype=dtype))
            elif name.endswith("norm.bias"):
                prm.copy_(0.3 * torch.randn(prm.shape, generator=gen, dtype=dtype))
    xs = torch.arange(NF, dtype=dtype).repeat(G).reshape(-1, 1)
    if Fs > 1:
        xs = torch.cat([xs, torch.randn(G * NF, Fs - 1, generator=gen, dtype=dtype)], 1)
    Ti = torch.randint(2, 13, (G * NC, 1), generator=gen).to(dtype)
    Ni = torch.randint(100, 2000, (G * NC, 1), generator=gen).to(dtype)
    xt = torch.cat([Ti, Ni], 1)
    if Ft > 2:
        xt = torch.cat([xt, torch.randn(G * NC, Ft - 2, generator=gen, dtype=dtype)], 1)
    xe = 2.0 + 8.0 * torch.rand(G * NF * NC, F, generator=gen, dtype=dtype)
    u = 0.1 * torch.randn(G, F, generator=gen, dtype=dtype)
    ei = canonical_edges(G, NF, NC)
    s_batch = torch.arange(G).repeat_interleave(NF)
    t_batch = torch.arange(G).repeat_interleave(NC)
    graph = OracleGraph(ei, xs, xt, xe, u, s_batch if G > 1 else None, t_batch if G > 1 else None)
    return model, graph
