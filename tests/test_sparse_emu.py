"""General (non-complete) bipartite graphs: the engine's sparse composition
(pfsgnn/sparse.py) on the emulated op set vs the autograd oracle (CPU, float64).

The reference runs on any edge_index (gnn.py:7-47); the oracle (oracle/ref_gnn.py)
takes one as is.  Cases cover ragged fiber/class degrees, empty fibers and
classes (the reference's scatter-mean gives 0 there, gnn.py:140-151),
repeated (fiber, class) pairs, a caller edge order that is neither fiber- nor
class-sorted, and batches of several graphs.  The objective is a fixed random
linear functional of every GNN output (x_s, x_t, x_e, u) -- train.py's own
loss indexes edges by position and needs complete graphs (train.py:40, :67).
"""
import copy

import pytest
import torch

from emu_backend import Dims, EmuBackend
from harness import make_problem
from oracle.ref_gnn import Graph as OracleGraph
from pfsgnn.engine import Engine


def sparse_edges(G, NF, NC, density, gen, dup=0, empty_fiber=True, empty_class=True):
    """Random edge_index of G graphs: each (f, c) kept with prob ``density``,
    ``dup`` repeated pairs, fiber 1 / class 0 of graph 0 optionally edgeless,
    shuffled caller order."""
    src, tgt = [], []
    for g in range(G):
        keep = torch.rand(NF, NC, generator=gen) < density
        keep[:, -1] = True                      # no class empty by accident
        keep[0, :] = True
        if g == 0 and empty_fiber:
            keep[1, :] = False
        if g == 0 and empty_class:
            keep[:, 0] = False
        f, c = torch.nonzero(keep, as_tuple=True)
        src.append(g * NF + f)
        tgt.append(g * NC + c)
    src, tgt = torch.cat(src), torch.cat(tgt)
    if dup:
        j = torch.randint(0, src.numel(), (dup,), generator=gen)
        src, tgt = torch.cat([src, src[j]]), torch.cat([tgt, tgt[j]])
    p = torch.randperm(src.numel(), generator=gen)
    return torch.stack([src[p], tgt[p]])


def sparse_problem(G, NF, NC, density, F=10, B=2, seed=0, dup=0, normed=True):
    model, graph = make_problem(G, NF, NC, F=F, B=B, seed=seed, normed=normed)
    gen = torch.Generator().manual_seed(seed + 100)
    ei = sparse_edges(G, NF, NC, density, gen, dup=dup)
    E = ei.shape[1]
    xe = 2.0 + 8.0 * torch.rand(E, F, generator=gen, dtype=torch.float64)
    graph = OracleGraph(ei, graph.x_s, graph.x_t, xe, graph.x_u, graph.s_batch, graph.t_batch)
    return model, graph, gen


def run_sparse(G, NF, NC, density, B=2, seed=0, dup=0, normed=True, F=10):
    model, graph, gen = sparse_problem(G, NF, NC, density, F=F, B=B, seed=seed, dup=dup,
                                       normed=normed)
    E = graph.edge_index.shape[1]
    ws, wt = torch.randn(G * NF, F, generator=gen, dtype=torch.float64), \
        torch.randn(G * NC, F, generator=gen, dtype=torch.float64)
    we, wu = torch.randn(E, F, generator=gen, dtype=torch.float64), \
        torch.randn(G, F, generator=gen, dtype=torch.float64)
    ref = copy.deepcopy(model)
    ref.train()
    out = ref(graph)
    loss_o = (out.x_s * ws).sum() + (out.x_t * wt).sum() + (out.x_e * we).sum() + (out.x_u * wu).sum()
    loss_o.backward()

    be = EmuBackend()
    sp = be.sparse_layout(graph.edge_index, G, NF, NC)
    d = Dims(G, NF, NC, F, sp=sp)
    assert d.E == E
    eng = Engine(be, F=F, B=B, Fs=1, Ft=2, T=12, normed=normed)
    P = {k: v.detach().clone() for k, v in model.named_parameters()}
    Gr = {k: torch.zeros_like(v) for k, v in P.items()}
    BN = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
    pos = sp.user_of                                      # caller edge at each position
    ctx = eng.forward(P, BN, d, graph.x_s.t().contiguous(), graph.x_t.t().contiguous(),
                      graph.x_e[pos].t().contiguous(), graph.x_u.t().contiguous())
    eng.backward(P, Gr, ctx, g_xe_out=we[pos].t().contiguous(), g_xs_out=ws.t().contiguous(),
                 g_xt_out=wt.t().contiguous(), g_u_out=wu.t().contiguous())
    xs, xt, xe3, u = ctx["out"]
    xe = be.edge_apply(d, *xe3)
    xe_user = torch.empty(E, F, dtype=torch.float64)
    xe_user[pos] = xe.t()
    return ref, out, (xs, xt, xe_user, u), Gr, BN


CASES = [(1, 9, 5, 0.6, 2, 0), (2, 7, 6, 0.5, 1, 3), (3, 6, 8, 0.4, 2, 5), (1, 12, 4, 0.9, 2, 0)]


@pytest.mark.parametrize("G,NF,NC,density,B,dup", CASES)
def test_sparse_engine_matches_oracle_fp64(G, NF, NC, density, B, dup):
    ref, out, (xs, xt, xe, u), Gr, BN = run_sparse(G, NF, NC, density, B=B, dup=dup)
    assert torch.allclose(xs.t(), out.x_s, rtol=1e-9, atol=1e-9)
    assert torch.allclose(xt.t(), out.x_t, rtol=1e-9, atol=1e-9)
    assert torch.allclose(xe, out.x_e, rtol=1e-9, atol=1e-9)
    assert torch.allclose(u.t(), out.x_u, rtol=1e-9, atol=1e-9)
    for name, prm in ref.named_parameters():
        gref = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        err = (Gr[name] - gref).abs().max().item()
        assert err <= 1e-8 * max(gref.abs().max().item(), 1.0), (name, err)
    for k, v in ref.state_dict().items():
        if "running" in k:
            assert torch.allclose(BN[k], v, rtol=1e-9, atol=1e-9), k


def test_sparse_engine_unnormed_fp64():
    ref, out, (xs, xt, xe, u), Gr, _ = run_sparse(2, 6, 5, 0.5, B=2, normed=False, dup=2)
    assert torch.allclose(xe, out.x_e, rtol=1e-9, atol=1e-9)
    for name, prm in ref.named_parameters():
        gref = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        assert (Gr[name] - gref).abs().max().item() <= 1e-8 * max(gref.abs().max().item(), 1.0), name


def test_sparse_layout_emulation():
    """CSR invariants of the layout (the HIP kernel is checked against this in
    tests/test_gpu_sparse.py)."""
    gen = torch.Generator().manual_seed(7)
    ei = sparse_edges(3, 5, 4, 0.5, gen, dup=4)
    sp = EmuBackend().sparse_layout(ei, 3, 5, 4)
    src, tgt = ei[0][sp.user_of], ei[1][sp.user_of]
    assert torch.equal(src, sp.src_p) and torch.equal(tgt, sp.tgt_p)
    assert bool((src[1:] >= src[:-1]).all())                  # sorted by fiber
    assert torch.equal(torch.sort(sp.user_of).values, torch.arange(ei.shape[1]))
    for f in range(15):                                      # stable: caller order within a fiber
        run = sp.user_of[sp.fib_ptr[f]:sp.fib_ptr[f + 1]]
        assert bool((run[1:] > run[:-1]).all())
        assert bool((src[sp.fib_ptr[f]:sp.fib_ptr[f + 1]] == f).all())
    for c in range(12):
        run = sp.cls_ord[sp.cls_ptr[c]:sp.cls_ptr[c + 1]]
        assert bool((tgt[run] == c).all()) and bool((run[1:] > run[:-1]).all())
    assert sp.fib_ptr[1] == sp.fib_ptr[2]                     # fiber 1 of graph 0 is empty
    with pytest.raises(ValueError):
        EmuBackend().sparse_layout(torch.tensor([[0], [5]]), 2, 3, 4)   # crosses graphs
