"""Data-parallel training over the GPUs of one node (one process per GPU).

The reference trains one graph per process (train.py); the batch of graphs
shards across ranks with no data-path collective: every rank runs the fused
step on its own graphs, and the only exchange is ONE all-reduce (mean) of the
flat gradient buffer (~40k floats for the reference model) per step, over
RCCL (backend "nccl" on ROCm) on xGMI -- it is latency-bound, so a single
bucket is the right size.

BatchNorm: the batch statistics a forward normalises with are per rank (no
SyncBN), as under torch DDP.  The running statistics (and
num_batches_tracked) follow DDP's default ``broadcast_buffers=True``: rank
0's buffers are broadcast to every rank once per step (``sync_buffers``, one
collective on a packed buffer), so eval-mode inference and checkpoints do not
depend on the rank.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return dist.get_rank() if dist.is_initialized() else 0, world
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def broadcast_parameters(model, src=0):
    """Rank `src`'s parameters and BatchNorm buffers to every rank (start of training)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    flat = model.flat_parameters()[0] if hasattr(model, "flat_parameters") else None
    if flat is not None:
        dist.broadcast(flat, src)
    else:
        for p in model.parameters():
            dist.broadcast(p.data, src)
    for b in model.buffers():
        dist.broadcast(b, src)


def sync_buffers(model, src=0):
    """DDP's broadcast_buffers=True: every rank takes rank `src`'s BatchNorm
    running statistics and batch counters (one broadcast of a packed buffer)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    bufs = [b for b in model.buffers()]
    if not bufs:
        return
    fl = [b for b in bufs if b.dtype == torch.float32]
    it = [b for b in bufs if b.dtype != torch.float32]
    for group in (fl, it):
        if not group:
            continue
        packed = torch.cat([b.reshape(-1) for b in group])
        dist.broadcast(packed, src)
        off = 0
        for b in group:
            n = b.numel()
            b.copy_(packed[off:off + n].view_as(b))
            off += n


def allreduce_gradients(model):
    """Mean of the gradients over ranks: one collective on the flat grad buffer."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    world = dist.get_world_size()
    if hasattr(model, "flat_parameters"):
        _, g = model.flat_parameters()
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        g.div_(world)
        return
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)
