"""Resume from the reference's optimizer state (train.py:126-132, 141).

``params/model_gnn_0.pth`` holds the torch.optim.Adam state that trained the
shipped weights (tests/golden/ckpt_adam.npz: 80 of 109 parameters with state,
step 40000, lr 5e-4).  train.py resumes a run with
``optimizer.load_state_dict(checkpoint['optim_state'])``; pfsgnn's train.main
does the same into ``pfsgnn.FusedAdam``.  Here both optimizers load that state
over the same weights, take the same gradients -- those of one train.py step
(2000 fibers x 12 classes, B = 3, sharpness 20*39999/40000) through the real
pfsgnn.GNN + loss_function backward, whose live set must be the 80 indices
with state -- and step twice.  Parameters and both moments must agree with
torch.optim.Adam's, for FusedAdam in both modes (per-parameter host step
counts, and ``capturable=True``: one device step count, the form bench.py
graph-captures), and the 29 parameters without state must stay untouched.

Agreement bar: FusedAdam forms torch's double scalars (1 - beta1, 1 - beta2,
lr / bias_correction1, sqrt(bias_correction2)) once in fp32 and applies them in
the order of torch's DEVICE kernels (the reference trains on a GPU), fused
multiply-adds included.  On the GPU (test_gpu_adam_resume.py, against
torch.optim.Adam on the same device) moments and parameters must then agree
bit for bit.  torch's CPU kernels round differently (no fused multiply-add in
addcmul_, (value * m) / denom in addcdiv_), so here, against torch's CPU
Adam, moments and parameters must agree within 2 fp32 ulps.

This module runs on the CPU through the test emulation of the op set
(tests/emu_backend.py, float32, with EmuBackend.adam restating pfsgnn_adam);
tests/test_gpu_adam_resume.py runs the same check on the HIP library.
"""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SHARP = 20.0 * 39999 / 40000


def optim_state_dict():
    """ckpt_adam.npz back in torch.optim.Adam's state_dict format (as saved by
    train.py:154-165)."""
    z = np.load(os.path.join(GOLD, "ckpt_adam.npz"))
    idx = [int(i) for i in z["indices"]]
    state = {i: {"step": torch.tensor(float(s)),
                 "exp_avg": torch.as_tensor(z[f"exp_avg_{i}"]).float(),
                 "exp_avg_sq": torch.as_tensor(z[f"exp_avg_sq_{i}"]).float()}
             for i, s in zip(idx, z["step"])}
    group = {"lr": float(z["lr"]), "betas": tuple(float(b) for b in z["betas"]),
             "eps": float(z["eps"]), "weight_decay": float(z["weight_decay"]), "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
             "fused": None, "params": list(range(int(z["n_params"])))}
    return {"state": state, "param_groups": [group]}, idx


def model_state(device):
    z = np.load(os.path.join(GOLD, "ckpt_params.npz"))
    return {k: torch.as_tensor(z[k]).to(device) for k in z.files if k != "epoch"}


def train_step_grads(pfsgnn, device, seed=1234):
    """One train.py step's gradients through the real GNN + fused loss."""
    from oracle.ref_graph import train_graph
    from pfsgnn.train import loss_function
    classes = np.load(os.path.join(GOLD, "classes.npz"))["increasing"]
    ei, xs, xt, xe, u = train_graph(classes, 2000, 10, generator=torch.Generator().manual_seed(7))
    gnn = pfsgnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2)
    gnn.load_state_dict(model_state("cpu"))
    gnn = gnn.to(device)
    gnn.train()
    data = pfsgnn.BipartiteData(ei.to(device), xs.to(device), xt.to(device), xe.to(device),
                                u.to(device))
    gnn.zero_grad()
    out = gnn(data)
    loss, _ = loss_function(out, xt.to(device), pclass=0.1, pfiber=0.1, sharpness=SHARP,
                            seed=seed)
    loss.backward()
    return gnn


def run_resume(pfsgnn, device, capturable, steps=2):
    """(ours, torch's) per-parameter (value, exp_avg, exp_avg_sq) after `steps`
    optimizer steps from the checkpoint state, plus the live set."""
    from pfsgnn.optim import FusedAdam, _is_live
    sd, idx = optim_state_dict()
    gnn = train_step_grads(pfsgnn, device)
    params = list(gnn.parameters())
    live = [i for i, p in enumerate(params) if _is_live(p)]
    grads = [p.grad.detach().clone() if _is_live(p) else None for p in params]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    p0 = [p.detach().clone() for p in params]
    opt = FusedAdam(params, lr=sd["param_groups"][0]["lr"], capturable=capturable)
    opt.load_state_dict(sd)
    ropt = torch.optim.Adam(ref, lr=sd["param_groups"][0]["lr"])
    ropt.load_state_dict(sd)
    for _ in range(steps):
        opt.step()
        for r, g in zip(ref, grads):
            r.grad = None if g is None else g.clone()
        ropt.step()
    ours = [(p.detach(), opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"]) for p in params]
    theirs = [(r.detach(), ropt.state[r]["exp_avg"] if r in ropt.state else None,
               ropt.state[r]["exp_avg_sq"] if r in ropt.state else None) for r in ref]
    return ours, theirs, live, idx, p0


def _ulps(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    ulp = (torch.finfo(torch.float32).eps * b.abs()).clamp_min(1e-45)
    return ((a - b).abs() / ulp).max().item()


def check_resume(ours, theirs, live, idx, p0, max_ulp):
    """max_ulp = 0: bitwise.  Returns the worst (param, moment) ulp distance."""
    assert live == idx, "the backward's live set is not the checkpoint's Adam state indices"
    worst_p = worst_m = 0.0
    for i, ((p, m, v), (rp, rm, rv), q0) in enumerate(zip(ours, theirs, p0)):
        if i not in idx:
            assert rm is None
            assert torch.equal(p.cpu(), q0.cpu()), f"param {i} without Adam state moved"
            continue
        dm = max(_ulps(m, rm), _ulps(v, rv))
        dp = _ulps(p, rp)
        worst_p, worst_m = max(worst_p, dp), max(worst_m, dm)
        assert dm <= max_ulp, f"param {i}: moments {dm:.2f} ulp from torch's"
        assert dp <= max_ulp, f"param {i}: value {dp:.2f} ulp from torch's"
        assert not torch.equal(p.cpu(), q0.cpu()), f"param {i} with state did not move"
    return worst_p, worst_m


@pytest.fixture(scope="module")
def emu_pfsgnn():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "pfs-neural-net_amd")]
    import pfsgnn
    from pfsgnn import config, gnn as gnn_mod
    from emu_backend import EmuBackend
    saved = (config.device, gnn_mod._BACKEND, gnn_mod._ParamMixin._check_device)
    config.device = torch.device("cpu")
    gnn_mod._BACKEND = EmuBackend(torch.float32)
    gnn_mod._ParamMixin._check_device = lambda self: None
    yield pfsgnn
    config.device, gnn_mod._BACKEND, gnn_mod._ParamMixin._check_device = saved


@pytest.mark.parametrize("capturable", [False, True])
def test_resume_from_reference_adam_state(emu_pfsgnn, capturable):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    wp, wm = check_resume(*run_resume(emu_pfsgnn, "cpu", capturable), max_ulp=2)
    print(f"capturable={capturable}: worst difference vs torch CPU Adam: parameters "
          f"{wp:.2f} ulp, moments {wm:.2f} ulp")


def test_torch_side_gradient_marks_a_parameter_live(emu_pfsgnn):
    """a parameter the fused backward leaves dead (decoder_s under
    train.py's loss) but that a torch-side term of the loss reaches (here an
    L2 penalty on its weights) must be updated by FusedAdam as torch.optim.Adam
    updates it (its .grad is not None there)."""
    from pfsgnn.optim import FusedAdam, _is_live
    from pfsgnn.train import loss_function
    from oracle.ref_graph import train_graph
    pfsgnn = emu_pfsgnn
    classes = np.load(os.path.join(GOLD, "classes.npz"))["increasing"]
    ei, xs, xt, xe, u = train_graph(classes, 200, 10, generator=torch.Generator().manual_seed(3))
    gnn = pfsgnn.GNN(B=2, Fdim=10, T=12, F_s=1, F_t=2)
    gnn.train()
    names = [n for n, _ in gnn.named_parameters()]
    params = list(gnn.parameters())
    opt = FusedAdam(params, lr=1e-2)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    ropt = torch.optim.Adam(ref, lr=1e-2)
    gnn.zero_grad()
    out = gnn(pfsgnn.BipartiteData(ei, xs, xt, xe, u))
    loss, _ = loss_function(out, xt, pclass=0.1, pfiber=0.1, sharpness=10.0, seed=3)
    pen = gnn.decoder_s[0].weight
    (loss + 1e-3 * (pen * pen).sum()).backward()
    live = {n for n, p in zip(names, params) if _is_live(p)}
    assert "decoder_s.0.weight" in live and "decoder_s.2.weight" not in live
    for r, p in zip(ref, params):
        r.grad = p.grad.detach().clone() if _is_live(p) else None
    i = names.index("decoder_s.0.weight")
    before = params[i].detach().clone()
    opt.step()
    ropt.step()
    for n, p, r in zip(names, params, ref):
        assert torch.allclose(p.detach(), r.detach(), rtol=1e-6, atol=1e-7), n
    assert not torch.equal(params[i].detach(), before)       # the penalised weight moved
