"""Engine orchestration + hand-derived backward vs the autograd oracle (CPU, float64).

The engine (product orchestration) is driven by the torch-CPU emulation of
the op set (tests/emu_backend.py); the oracle is the literal restatement of
the reference (oracle/).  In float64 the two must agree to ~1e-9: any error
in the fused algebra (split first Linear, post-sum second Linear, double
BatchNorm, moment gradients, loss gradients) shows up far above that.
"""
import copy

import pytest
import torch

from emu_backend import EmuBackend, Dims
from harness import from_canonical, make_problem, to_canonical
from noise_ref import uniform_numpy
from oracle.ref_train import loss_function as oracle_loss
from pfsgnn.engine import Engine, param_names


def run_pair(G, NF, NC, F=10, B=2, normed=True, sharp=12.0, seed=0, loss_bn=False):
    model, graph = make_problem(G, NF, NC, F=F, B=B, seed=seed, normed=normed)
    ref = copy.deepcopy(model)
    ref.train()
    # ---- oracle
    out = ref(graph)
    uni = torch.as_tensor(uniform_numpy(1234, G * NF * NC), dtype=torch.float64)
    loss_o, diag_o = oracle_loss(ref, out.x_e, graph.x_t, G, NF, NC, pclass=0.1, pfiber=0.1,
                                 sharpness=sharp, uniform=uni)
    loss_o.backward()
    # ---- engine + emulated ops
    be = EmuBackend()
    eng = Engine(be, F=F, B=B, Fs=1, Ft=2, T=12, normed=normed)
    P = {k: v.detach().clone() for k, v in model.named_parameters()}
    Gr = {k: torch.zeros_like(v) for k, v in P.items()}
    BN = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
    d = Dims(G, NF, NC, F)
    ctx = eng.forward(P, BN, d, graph.x_s.t().contiguous(), graph.x_t.t().contiguous(),
                      to_canonical(graph.x_e, G, NF, NC), graph.x_u.t().contiguous())
    loss_e, diag_e, lctx = eng.loss_forward(P, d, ctx["out"][2], graph.x_t.t().contiguous(), sharp,
                                           1234, pclass=0.1, pfiber=0.1)
    if loss_bn:   # the loss backward also makes the last edge BatchNorm's sums
        bns = eng.loss_bnstat(ctx)
        assert bns is not None
        g_next, ctx["g_xe_bn_part"] = eng.loss_backward(P, Gr, lctx, bnstat=bns)
    else:
        g_next = eng.loss_backward(P, Gr, lctx)
    eng.backward(P, Gr, ctx, g_xe_out=g_next)
    assert "g_xe_bn_part" not in ctx
    return ref, out, loss_o, ctx, loss_e, P, Gr, BN, be


@pytest.mark.parametrize("G,NF,NC,B,loss_bn", [(1, 9, 5, 2, False), (2, 6, 4, 1, False),
                                               (3, 5, 7, 2, False), (2, 6, 4, 1, True),
                                               (3, 5, 7, 2, True)])
def test_engine_matches_oracle_fp64(G, NF, NC, B, loss_bn):
    ref, out, loss_o, ctx, loss_e, P, Gr, BN, be = run_pair(G, NF, NC, B=B, loss_bn=loss_bn)
    xs, xt, xe3, u = ctx["out"]
    xe = be.edge_apply(ctx["d"], *xe3)
    assert torch.allclose(xs.t(), out.x_s, rtol=1e-9, atol=1e-9)
    assert torch.allclose(xt.t(), out.x_t, rtol=1e-9, atol=1e-9)
    assert torch.allclose(from_canonical(xe, G, NF, NC), out.x_e, rtol=1e-9, atol=1e-9)
    assert torch.allclose(u.t(), out.x_u, rtol=1e-9, atol=1e-9)
    assert torch.allclose(loss_e, loss_o, rtol=1e-10, atol=1e-8)
    names = param_names(B)
    assert set(names) == set(P.keys())
    for name, prm in ref.named_parameters():
        gref = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        scale = gref.abs().max().item() + 1e-12
        err = (Gr[name] - gref).abs().max().item()
        assert err <= 1e-8 * max(scale, 1.0), (name, err, scale)
    for k, v in ref.state_dict().items():
        if "running" in k:
            assert torch.allclose(BN[k], v, rtol=1e-9, atol=1e-9), k


def test_engine_unnormed_fp64():
    ref, out, loss_o, ctx, loss_e, P, Gr, BN, be = run_pair(2, 6, 5, B=2, normed=False)
    assert torch.allclose(loss_e, loss_o, rtol=1e-10, atol=1e-8)
    for name, prm in ref.named_parameters():
        gref = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        assert (Gr[name] - gref).abs().max().item() <= 1e-8 * max(gref.abs().max().item(), 1.0), name


@pytest.mark.parametrize("G,NF,NC,B", [(1, 9, 5, 2), (2, 6, 4, 1)])
def test_engine_eval_mode_fp64(G, NF, NC, B):
    """Eval-mode forward (every BatchNorm1d on running statistics, none
    updated) vs the oracle in ``eval()``; running stats are first moved off
    their init values by one training forward so the affine is non-trivial."""
    model, graph = make_problem(G, NF, NC, B=B, seed=3)
    model.train()
    with torch.no_grad():
        model(graph)
    ref = copy.deepcopy(model).eval()
    with torch.no_grad():
        out = ref(graph)
    be = EmuBackend()
    eng = Engine(be, F=10, B=B, Fs=1, Ft=2, T=12, normed=True)
    P = {k: v.detach().clone() for k, v in model.named_parameters()}
    BN = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
    BN0 = {k: v.clone() for k, v in BN.items()}
    d = Dims(G, NF, NC, 10)
    ctx = eng.forward(P, BN, d, graph.x_s.t().contiguous(), graph.x_t.t().contiguous(),
                      to_canonical(graph.x_e, G, NF, NC), graph.x_u.t().contiguous(),
                      training=False)
    xs, xt, xe3, u = ctx["out"]
    xe = be.edge_apply(d, *xe3)
    assert torch.allclose(xs.t(), out.x_s, rtol=1e-9, atol=1e-9)
    assert torch.allclose(xt.t(), out.x_t, rtol=1e-9, atol=1e-9)
    assert torch.allclose(from_canonical(xe, G, NF, NC), out.x_e, rtol=1e-9, atol=1e-9)
    assert torch.allclose(u.t(), out.x_u, rtol=1e-9, atol=1e-9)
    for k in BN:
        assert torch.equal(BN[k], BN0[k]), k
    with pytest.raises(NotImplementedError):   # an inference-only context
        eng.backward(P, {k: torch.zeros_like(v) for k, v in P.items()}, ctx,
                     g_xe_out=torch.zeros_like(xe))


@pytest.mark.parametrize("G,NF,NC,B,normed", [(1, 9, 5, 2, True), (2, 6, 4, 1, True),
                                              (3, 5, 7, 2, True), (2, 6, 5, 2, False)])
def test_engine_eval_mode_backward_fp64(G, NF, NC, B, normed):
    """gnn.eval() under autograd (the reference trains nothing in eval, but its
    backward works: BatchNorm on running statistics is an affine map, round()
    the identity, gnn.py:101/154/192/321-325): the engine's eval forward with
    want_grad + the train.py loss + backward vs the oracle in eval() in fp64."""
    model, graph = make_problem(G, NF, NC, B=B, seed=11, normed=normed)
    model.train()
    with torch.no_grad():
        model(graph)                     # running stats off their init values
    ref = copy.deepcopy(model).eval()
    sharp = 9.0
    out = ref(graph)
    uni = torch.as_tensor(uniform_numpy(4321, G * NF * NC), dtype=torch.float64)
    loss_o, _ = oracle_loss(ref, out.x_e, graph.x_t, G, NF, NC, pclass=0.1, pfiber=0.1,
                            sharpness=sharp, uniform=uni)
    loss_o.backward()
    be = EmuBackend()
    eng = Engine(be, F=10, B=B, Fs=1, Ft=2, T=12, normed=normed)
    P = {k: v.detach().clone() for k, v in model.named_parameters()}
    Gr = {k: torch.zeros_like(v) for k, v in P.items()}
    BN = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
    BN0 = {k: v.clone() for k, v in BN.items()}
    d = Dims(G, NF, NC, 10)
    ctx = eng.forward(P, BN, d, graph.x_s.t().contiguous(), graph.x_t.t().contiguous(),
                      to_canonical(graph.x_e, G, NF, NC), graph.x_u.t().contiguous(),
                      training=False, want_grad=True)
    loss_e, _, lctx = eng.loss_forward(P, d, ctx["out"][2], graph.x_t.t().contiguous(), sharp,
                                       4321, pclass=0.1, pfiber=0.1)
    eng.backward(P, Gr, ctx, g_xe_out=eng.loss_backward(P, Gr, lctx))
    assert torch.allclose(loss_e, loss_o, rtol=1e-10, atol=1e-8)
    for name, prm in ref.named_parameters():
        gref = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        scale = gref.abs().max().item() + 1e-12
        err = (Gr[name] - gref).abs().max().item()
        assert err <= 1e-8 * max(scale, 1.0), (name, err, scale)
    for k in BN:
        assert torch.equal(BN[k], BN0[k]), k
