"""Drop-in for the reference ``src/train.py`` objective and training loop.

``loss_function`` (train.py:29-80) runs fused over the edges in
``libpfsgnn.so``: decoder_e (gnn.py:307) + softplus + ``softfloor``
(train.py:21) + the per-class / per-fiber scatters + penalties, with the
backward as one more fused pass that hands the last message-passing block
its edge gradient.  The loss reads the GNN's lazy final edge state directly
(``graph._pf``), so the normalised edge features are never re-read.

softfloor's noise: the reference draws ``torch.rand_like`` (train.py:22);
here the uniforms come from a counter-based hash of (seed, edge id) computed
in-kernel (``pfsgnn_common.h: pf_uniform``), with the per-call seed drawn from
torch's global CPU generator -- so ``torch.manual_seed`` governs it as it
governs the reference, a step is reproducible, and no RNG state lives on the
device.
"""
import math
import os
import sys

import numpy as np
import torch

from . import config
from .engine import Dims
from .gnn import GNN, BipartiteData, backend

_SEED_SPACE = (1 << 62)


def draw_seed():
    return int(torch.randint(0, _SEED_SPACE, (1,)).item())


def softfloor(x, sharpness=20, noiselevel=0.3):
    """train.py:21-27 on an arbitrary tensor (utility; the training objective
    uses the fused in-kernel version).  Elementwise torch on the device."""
    noise = noiselevel * (torch.rand_like(x) - 0.5)
    x = x + noise
    sharpness = x.new_tensor(sharpness)
    pi = x.new_tensor(np.pi)
    r = torch.where(sharpness == 0, torch.tensor(0.0, device=x.device), torch.exp(-1 / sharpness))
    return x + 1 / pi * (torch.arctan(r * torch.sin(2 * pi * x) / (1 - r * torch.cos(2 * pi * x)))
                         - torch.arctan(r / (torch.ones_like(r) - r)))


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, anchor, model, d, ectx, xe3, ci, sharpness, seed, pclass, pfiber,
                want_time, noiselevel):
        ctx.set_materialize_grads(False)   # the diagnostics get no gradient: no zero fills
        eng = model._engine()
        P = model._flat_params()
        loss, diag, lctx = eng.loss_forward(P, d, xe3, ci, sharpness, seed, pclass=pclass,
                                            pfiber=pfiber, total_time=float(config.TOTAL_TIME),
                                            nfields=float(config.NFIELDS), wutils=config.wutils,
                                            wvar=config.wvar, want_time=want_time,
                                            noiselevel=noiselevel)
        ctx.pf = (model, d, ectx, lctx)
        outs = (diag["utils"], diag["n_prime"], diag["fiber_time"], diag["variance"])
        ctx.mark_non_differentiable(*outs)
        if diag["time"] is not None:
            ctx.mark_non_differentiable(diag["time"])
        return (loss,) + outs + ((diag["time"],) if diag["time"] is not None else ())

    @staticmethod
    def backward(ctx, g_loss, *unused):
        model, d, ectx, lctx = ctx.pf
        if g_loss is None:
            return (None,) * 13
        eng = model._engine()
        P, Gr = model._flat_params(), model._recording_grads()
        prev = ectx.get("g_xe_canonical")
        # the final edge BatchNorm's backward sums come out of the same pass when
        # this loss is the edge state's only consumer so far
        bns = eng.loss_bnstat(ectx) if prev is None else None
        out = eng.loss_backward(P, Gr, lctx, gscale=g_loss, bnstat=bns)
        gc, part = out if bns is not None else (out, None)
        model._mark_live(Gr.used)
        # hand the canonical [F, E] gradient straight to the GNN's backward
        # (gnn._GNNFn.backward); the edge-state token gets none
        if prev is None:
            ectx["g_xe_canonical"] = gc
            if part is not None:
                ectx["g_xe_bn_part"] = part
        else:
            ectx["g_xe_canonical"] = prev + gc
            ectx.pop("g_xe_bn_part", None)
        return (None,) * 13


def _class_info_cm(class_info, d):
    ci = class_info.to(device=config.device, dtype=torch.float32)
    if ci.dim() != 2 or ci.size(0) != d.NT or ci.size(1) < 2:
        raise ValueError(f"class_info must be [G*NC, >=2] = [{d.NT}, >=2]; got {tuple(ci.shape)}")
    return ci[:, :2].t().contiguous()


def loss_function(graph, class_info, pclass=0.1, pfiber=1.0, sharpness=0.5, finaloutput=False,
                  *, gnn=None, seed=None, noiselevel=0.3):
    """train.py:29-80.  ``graph`` is the output of ``GNN.forward``; ``class_info``
    is [NC, 2] (T_i, N_i) per class -- [G*NC, 2] for a batch of G graphs, whose
    loss is the sum of the per-graph losses.  The reference reads the model
    from a global ``gnn`` (train.py:42); here it comes with the graph (or
    ``gnn=``).  Edge order must be the fiber-major layout train.py builds
    (train.py:94), on which train.py:40 and :67 rely.  ``seed`` (softfloor's
    noise): None draws one from torch's CPU generator; an int; or a device
    int64 tensor read in-kernel (a captured step then draws fresh noise per
    replay when the tensor is advanced on the device).  ``noiselevel`` is
    softfloor's (train.py:21, fixed at 0.3 by the reference's call)."""
    pf = graph.__dict__.get("_pf")
    if pf is None or graph.__dict__.get("_pf_replaced"):
        raise NotImplementedError("loss_function needs the BipartiteData returned by "
                                  "pfsgnn.GNN.forward (the fused loss reads its edge state)")
    model, d, lay, token, xe3, ectx = pf
    if token is None:
        # eval-mode forward: the loss is inference-only (no backward through it)
        if torch.is_grad_enabled():
            raise NotImplementedError("loss_function on an eval-mode GNN.forward runs under "
                                      "torch.no_grad() only (train.py:108 trains in train mode)")
        token = xe3[0].new_empty(())
    if gnn is not None and gnn is not model:
        raise ValueError("graph was produced by a different GNN than `gnn`")
    if not lay.fiber_major:
        raise NotImplementedError("train.py's objective indexes edges by position "
                                  "(train.py:40, :67): it needs the fiber-major edge order")
    ci = _class_info_cm(class_info, d)
    if seed is None:
        seed = draw_seed()
    elif not isinstance(seed, torch.Tensor):
        seed = int(seed)
    outs = _LossFn.apply(token, model.encoder_s[0].weight, model, d, ectx, xe3, ci, float(sharpness),
                         seed, float(pclass), float(pfiber), bool(finaloutput), float(noiselevel))
    loss, utils_g, n_prime, fiber_time, variance = outs[:5]
    if not finaloutput:
        return loss, utils_g.sum() if d.G > 1 else utils_g[0]
    time = outs[5]
    Ni = ci[1] / config.NFIELDS
    comp = (n_prime / Ni).detach().cpu().numpy()
    fibers = fiber_time.detach().cpu().numpy()
    utils = utils_g.sum() if d.G > 1 else utils_g[0]
    var = variance.sum() if d.G > 1 else variance[0]
    return loss, utils, comp, n_prime, fibers, time, var


# ---------------------------------------------------------------- training
def complete_graph(class_info, nfibers, fdim, lo=2.0, hi=10.0):
    """train.py:88-104: fiber counter x_s, class_info x_t, fiber-major complete
    edges, x_e ~ U[lo, hi), u = 0."""
    class_info = torch.as_tensor(class_info, dtype=torch.float, device=config.device)
    nclasses = class_info.shape[0]
    x_s = torch.arange(nfibers, dtype=torch.float, device=config.device).reshape(-1, 1)
    # torch.cartesian_prod's fiber-major order, built on the device
    edge_index = backend().build_complete(1, nfibers, nclasses, order=0)
    x_e = lo + (hi - lo) * torch.rand(size=(nfibers * nclasses, fdim)).to(config.device)
    x_u = torch.zeros(1, fdim).to(config.device)
    return BipartiteData(edge_index=edge_index, x_s=x_s, x_t=class_info, x_e=x_e, x_u=x_u)


def main(argv=None):
    """train.py:82-165 (training + checkpointing; the plotting of train.py:168-305
    is not part of the hot path and is skipped)."""
    from .optim import FusedAdam
    argv = sys.argv[1:] if argv is None else argv
    idx = int(os.environ.get("SLURM_ARRAY_TASK_ID", 0))
    ID = str(idx)
    class_info = torch.tensor(np.loadtxt(config.datafile), dtype=torch.float, device=config.device)
    NF, NC = config.NFIBERS, class_info.shape[0]
    graph = complete_graph(class_info, NF, config.Fdim)
    gnn = GNN(Fdim=config.Fdim, B=3, F_s=1, F_t=class_info.shape[1], T=NC).to(config.device)
    gnn.train()
    optimizer = FusedAdam(gnn.parameters(), lr=config.lr)
    nepochs = config.nepochs
    start_epoch = 0
    if argv:
        ck = torch.load(argv[0], map_location=config.device, weights_only=True)
        gnn.load_state_dict(ck["model_state"])
        optimizer.load_state_dict(ck["optim_state"])
        start_epoch = ck["epoch"] + 1
    best_utility = 0.0
    for epoch in range(start_epoch, nepochs):
        gnn.zero_grad()
        graph_ = gnn(graph)
        sharp = config.sharps[0] + (config.sharps[1] - config.sharps[0]) * epoch / nepochs
        loss, utility, comp, _, fiber_time, time, variance = loss_function(
            graph_, class_info, pclass=config.pclass, pfiber=config.pfiber, sharpness=sharp,
            finaloutput=True)
        loss.backward()
        optimizer.step()
        if float(utility) > best_utility and sharp > config.min_sharp:
            best_utility = float(utility)
            torch.save({"epoch": epoch, "model_state": gnn.state_dict(),
                        "optim_state": optimizer.state_dict()}, config.checkpoint_path + ID + ".pth")
    torch.save({"epoch": nepochs, "model_state": gnn.state_dict(),
                "optim_state": optimizer.state_dict()}, config.checkpoint_path + ID + ".pth")


if __name__ == "__main__":
    main()
