"""Data-parallel equivalence of the REAL model on CPU (gloo, world_size 2).

pfsgnn.GNN + pfsgnn.train.loss_function + backward run on the test emulation
of the op set (tests/emu_backend.py, installed as the backend, float32, with
config.device patched to the CPU), through the real _FlatMixin flat
parameter / gradient buffers and pfsgnn.distributed.  Rank r trains on graph
r of a 2-graph batch (train.py's per-process graph, sharded); after
allreduce_gradients every rank must hold 1/2 x the single-process gradient of
the 2-graph batch (the batch loss is the sum of the per-graph losses), and a
torch.optim.Adam step (train.py:141) must leave identical parameters on both
ranks.  With BatchNorm (normed=True) the forward normalises with per-rank
statistics (no SyncBN, as DDP), so only the buffer broadcast is checked there.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

G, NF, NC, B = 2, 12, 5, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "pfs-neural-net_amd")]
    import pfsgnn
    from pfsgnn import config, gnn
    from emu_backend import EmuBackend
    config.device = torch.device("cpu")
    gnn._BACKEND = EmuBackend(torch.float32)
    gnn._ParamMixin._check_device = lambda self: None      # float32 CPU parameters
    return pfsgnn


def _graphs(normed):
    from harness import make_problem
    model, graph = make_problem(G, NF, NC, B=B, seed=3, normed=normed, dtype=torch.float32)
    return model, graph


def _step(pfsgnn, model, data_parts, normed):
    from pfsgnn.train import loss_function
    gnn = pfsgnn.GNN(B=B, Fdim=10, T=12, F_s=1, F_t=2, normed=normed)
    gnn.load_state_dict(model.state_dict())
    gnn.train()
    ei, xs, xt, xe, xu = data_parts
    data = pfsgnn.BipartiteData(ei, xs, xt, xe, xu)
    gnn.zero_grad()
    out = gnn(data)
    loss, _ = loss_function(out, xt, pclass=0.1, pfiber=0.1, sharpness=10.0, seed=7, noiselevel=0.0)
    loss.backward()
    return gnn, loss


def _part(graph, g):
    """Graph g of the batch as a stand-alone graph (train.py's fiber-major order)."""
    E1 = NF * NC
    e = torch.arange(E1)
    ei = torch.stack([e // NC, e % NC])
    sl = slice(g * E1, (g + 1) * E1)
    return (ei, graph.x_s[g * NF:(g + 1) * NF], graph.x_t[g * NC:(g + 1) * NC], graph.x_e[sl],
            graph.x_u[g:g + 1])


def _worker(rank, world, port, out, normed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    pfsgnn = _setup()
    from pfsgnn.distributed import allreduce_gradients, broadcast_parameters, init_from_env, sync_buffers
    init_from_env(backend="gloo")
    model, graph = _graphs(normed)
    gnn, loss = _step(pfsgnn, model, _part(graph, rank), normed)
    broadcast_parameters(gnn)           # identical already; exercises the flat-buffer path
    allreduce_gradients(gnn)
    flat, gflat = gnn.flat_parameters()
    g_after = gflat.clone()
    opt = torch.optim.Adam(gnn.parameters(), lr=1e-2)
    opt.step()
    sync_buffers(gnn)
    out[rank] = (g_after, flat.clone(), {k: v.clone() for k, v in gnn.state_dict().items()},
                 float(loss.detach()))
    dist.barrier()
    dist.destroy_process_group()


def _run(normed):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out, normed), nprocs=2, join=True)
    return out[0], out[1]


def test_dp_gradients_equal_half_the_union_batch():
    (g0, p0, sd0, l0), (g1, p1, sd1, l1) = _run(normed=False)
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "pfs-neural-net_amd")]
    from pfsgnn import config, gnn as gnn_mod
    saved = (config.device, gnn_mod._BACKEND, gnn_mod._ParamMixin._check_device)
    try:                      # the single-process union batch, in this process
        pfsgnn = _setup()
        model, graph = _graphs(False)
        gnn, loss = _step(pfsgnn, model, (graph.edge_index, graph.x_s, graph.x_t, graph.x_e,
                                          graph.x_u), False)
        _, gu = gnn.flat_parameters()
        gu = gu.clone()
        loss = float(loss.detach())
    finally:
        config.device, gnn_mod._BACKEND, gnn_mod._ParamMixin._check_device = saved
    assert abs(l0 + l1 - loss) <= 1e-4 * abs(loss)
    assert torch.equal(g0, g1)                                  # one all-reduce, same result
    err = (g0 - 0.5 * gu).abs().max().item()
    assert err <= 1e-4 * gu.abs().max().item(), err
    assert torch.equal(p0, p1)                                  # Adam from identical grads
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


def test_dp_batchnorm_buffers_follow_rank0():
    (g0, p0, sd0, _), (g1, p1, sd1, _) = _run(normed=True)
    assert torch.equal(g0, g1) and torch.equal(p0, p1)
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k                   # running stats broadcast from rank 0
