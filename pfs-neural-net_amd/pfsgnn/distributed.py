"""Data-parallel training over the GPUs of one node (one process per GPU).

The reference trains one graph per process (train.py); the batch of graphs
shards across ranks with no data-path collective: every rank runs the fused
step on its own graphs, and the only exchange is ONE all-reduce (mean) of the
flat gradient buffer (~40k floats for the reference model) per step, over
RCCL (backend "nccl" on ROCm) on xGMI -- it is latency-bound, so a single
bucket is the right size.

BatchNorm: the batch statistics a forward normalises with are per rank (no
SyncBN), as under torch DDP.  The running statistics (and
num_batches_tracked) follow DDP's default ``broadcast_buffers=True``: at the
start of every step, before the forward (where DDP does it), rank 0's buffers
are broadcast to every rank (``sync_buffers``: the float buffers live in one
packed tensor, so it is one collective plus one for the int64 counters), so
eval-mode inference and checkpoints do not depend on the rank.
"""
import os

import torch
import torch.distributed as dist

# PFSGNN_DIST_FORCE=1: run the collectives even in a world of one rank (a
# process group of one member: RCCL still launches its kernels, which is how
# bench.py rehearses capturing them into the step's HIP graph on one GPU)
_FORCE = os.environ.get("PFSGNN_DIST_FORCE") == "1"


def _active():
    return dist.is_initialized() and (dist.get_world_size() > 1 or _FORCE)


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
    if not _active():
        return
    flat = model.flat_parameters()[0] if hasattr(model, "flat_parameters") else None
    if flat is not None:
        dist.broadcast(flat, src)
    else:
        for p in model.parameters():
            dist.broadcast(p.data, src)
    for b in model.buffers():
        dist.broadcast(b, src)


def _packed(model, names, dtype):
    """One tensor holding every `dtype` buffer of `model` in `names` order, the
    module buffers re-pointed at views of it (kept while they stay views)."""
    key = "_pf_bufpack_" + str(dtype).split(".")[-1]
    bufs = dict(model.named_buffers())
    cache = model.__dict__.get(key)
    if cache is not None and cache[0] == names:
        flat, offs = cache[1], cache[2]
        if all(bufs[n].data_ptr() == flat.data_ptr() + flat.element_size() * o
               and bufs[n].device == flat.device for n, o in zip(names, offs)):
            return flat
    # int64 counters of pfsgnn.GNN are already one tensor (GNN._bump_batches)
    nbt = model.__dict__.get("_pf_nbt")
    if dtype == torch.int64 and nbt is not None:
        flat = nbt[1]
        offs = [(bufs[n].data_ptr() - flat.data_ptr()) // 8 for n in names]
        if all(0 <= o < flat.numel() for o in offs) and len(set(offs)) == len(offs) == flat.numel():
            model.__dict__[key] = (names, flat, offs)
            return flat
    flat = torch.cat([bufs[n].detach().reshape(-1) for n in names]).contiguous()
    offs, o = [], 0
    for n in names:
        b = bufs[n]
        mod = model.get_submodule(n.rsplit(".", 1)[0]) if "." in n else model
        mod._buffers[n.rsplit(".", 1)[-1]] = flat[o:o + b.numel()].view_as(b)
        offs.append(o)
        o += b.numel()
    model.__dict__[key] = (names, flat, offs)
    return flat


def sync_buffers(model, src=0):
    """DDP's broadcast_buffers=True: every rank takes rank `src`'s BatchNorm
    running statistics and batch counters.  Call it at the start of a step,
    before the forward, as DDP does (the forward then reads and updates the
    same buffers on every rank)."""
    if not _active():
        return
    groups = {}
    for n, b in model.named_buffers():
        groups.setdefault(b.dtype, []).append(n)
    for dtype, names in groups.items():
        dist.broadcast(_packed(model, tuple(names), dtype), src)


def allreduce_gradients(model):
    """Mean of the gradients over ranks: one collective on the flat grad buffer."""
    if not _active():
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
