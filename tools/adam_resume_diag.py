"""Diagnostic for tests/test_gpu_adam_resume.py: where does FusedAdam's step
differ from torch.optim.Adam's on the device?  One step from the checkpoint
state; prints the differing elements with their inputs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pfs-neural-net_amd")]

import pfsgnn  # noqa: E402
from pfsgnn.optim import FusedAdam, _is_live  # noqa: E402
from test_adam_resume import optim_state_dict, train_step_grads  # noqa: E402

sd, idx = optim_state_dict()
gnn = train_step_grads(pfsgnn, "cuda")
params = list(gnn.parameters())
names = [n for n, _ in gnn.named_parameters()]
grads = [p.grad.detach().clone() if _is_live(p) else None for p in params]
ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
p0 = [p.detach().clone() for p in params]
m0 = {i: sd["state"][i]["exp_avg"].clone() for i in idx}
v0 = {i: sd["state"][i]["exp_avg_sq"].clone() for i in idx}
opt = FusedAdam(params, lr=5e-4)
opt.load_state_dict(sd)
ropt = torch.optim.Adam(ref, lr=5e-4)
ropt.load_state_dict(sd)
opt.step()
for r, g in zip(ref, grads):
    r.grad = None if g is None else g.clone()
ropt.step()
for i in idx:
    a, b = params[i].detach().cpu(), ref[i].detach().cpu()
    bad = (a != b).nonzero().flatten() if a.dim() == 1 else (a.reshape(-1) != b.reshape(-1)).nonzero().flatten()
    if bad.numel():
        print(f"param {i} {names[i]}: {bad.numel()} of {a.numel()} elements differ")
        for e in bad[:6].tolist():
            f = lambda t: t.reshape(-1)[e].item()  # noqa: E731
            print(f"  [{e}] p0={f(p0[i].cpu())!r} g={f(grads[i].cpu())!r} m0={f(m0[i])!r} v0={f(v0[i])!r} "
                  f"m={f(opt.state[params[i]]['exp_avg'].cpu())!r} v={f(opt.state[params[i]]['exp_avg_sq'].cpu())!r} "
                  f"ours={f(a)!r} torch={f(b)!r}")
print("done")
