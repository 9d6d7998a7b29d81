"""Data-parallel host logic on CPU: world_size 2 over gloo (127.0.0.1).

Covers pfsgnn.distributed: parameter broadcast from rank 0 and the single
mean all-reduce of the flat gradient buffer, for both the flat-buffer path
(what pfsgnn.GNN exposes) and the per-parameter path.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FlatModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("bn_running", torch.zeros(3))
        self.flat = torch.zeros(8)
        self.gflat = torch.zeros(8)

    def flat_parameters(self):
        return self.flat, self.gflat


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "pfs-neural-net_amd")]
    from pfsgnn.distributed import allreduce_gradients, broadcast_parameters, init_from_env
    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    m = FlatModel()
    m.flat.fill_(rank + 1.0)
    m.bn_running.fill_(10.0 * (rank + 1))
    broadcast_parameters(m)
    m.gflat.copy_(torch.arange(8.0) * (rank + 1))
    allreduce_gradients(m)
    lin = torch.nn.Linear(3, 2)
    torch.manual_seed(rank)
    for p in lin.parameters():
        p.data.normal_()
        p.grad = torch.full_like(p, float(rank))
    broadcast_parameters(lin)
    allreduce_gradients(lin)
    out[rank] = (m.flat.clone(), m.bn_running.clone(), m.gflat.clone(), lin.weight.data.clone(),
                 lin.weight.grad.clone())
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_and_broadcast_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    f0, b0, g0, w0, gw0 = out[0]
    f1, b1, g1, w1, gw1 = out[1]
    assert torch.equal(f0, torch.ones(8)) and torch.equal(f1, torch.ones(8))   # rank 0's params
    assert torch.equal(b0, b1) and b1[0] == 10.0
    expect = torch.arange(8.0) * 1.5                                           # mean of 1x and 2x
    assert torch.allclose(g0, expect) and torch.allclose(g1, expect)
    assert torch.equal(w0, w1)
    assert torch.allclose(gw0, torch.full_like(gw0, 0.5)) and torch.allclose(gw1, gw0)
