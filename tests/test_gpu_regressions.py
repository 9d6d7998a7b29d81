"""Regression tests for host-side hazards of the HIP path (round-1 advisor
findings): stale per-tensor caches, buffers re-allocated under a captured
graph, weight decay on parameters the reference leaves without a gradient,
and NaN propagation through the completeness min."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

from harness import make_problem  # noqa: E402


def _hip_model(model, B):
    import pfsgnn
    gnn = pfsgnn.GNN(B=B, Fdim=10, T=12, F_s=1, F_t=2).cuda()
    gnn.load_state_dict({k: v.float() for k, v in model.state_dict().items()})
    gnn.train()
    return gnn


def _step(gnn, data, ci, seed=3):
    from pfsgnn.train import loss_function
    gnn.zero_grad()
    out = gnn(data)
    loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=8.0, seed=seed)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), out.x_e.detach().clone(), torch.cat([p.grad.reshape(-1) for p in gnn.parameters()]).clone()


def test_same_shape_batches_never_hit_stale_caches():
    """A new batch of the same shape whose tensors land on recycled allocator
    blocks must be re-analysed (edge_index) and re-converted (x_e)."""
    import pfsgnn
    from pfsgnn import gnn as G_
    G, NF, NC = 2, 40, 12
    model, graph = make_problem(G, NF, NC, B=2, seed=1)
    ci = graph.x_t.float().cuda()
    gen = torch.Generator().manual_seed(5)
    results = []
    for it in range(3):
        # a fresh random edge order and fresh x_e every iteration, same shapes
        perm = torch.randperm(G * NF * NC, generator=gen)
        ei = graph.edge_index[:, perm].cuda()
        xe = (2.0 + 8.0 * torch.rand(G * NF * NC, 10, generator=gen)).cuda()
        data = pfsgnn.BipartiteData(ei, graph.x_s.float(), graph.x_t.float(), xe, graph.x_u.float())
        gnn = _hip_model(model, 2)
        out = gnn(data)
        xe_out = out.x_e.detach().clone()
        # ground truth for this batch: caches cleared
        G_._LAYOUT_CACHE.clear()
        G_._EDGE_CACHE.clear()
        gnn2 = _hip_model(model, 2)
        ref = gnn2(data).x_e.detach().clone()
        assert torch.equal(xe_out, ref), it
        results.append(xe_out)
        del data, ei, xe, out, gnn, gnn2
    assert not torch.equal(results[0], results[1])


def test_replay_survives_workspace_growth():
    """Eager calls on a larger batch after capture grow the workspace / arena;
    the captured graph must keep writing into memory it still owns."""
    import pfsgnn
    model, graph = make_problem(1, 64, 16, B=2, seed=2)
    gnn = _hip_model(model, 2)
    data = pfsgnn.BipartiteData(graph.edge_index, graph.x_s.float(), graph.x_t.float(),
                                graph.x_e.float(), graph.x_u.float())
    ci = graph.x_t.float().cuda()
    sd = copy.deepcopy(gnn.state_dict())
    from pfsgnn.train import loss_function

    def fb():
        gnn.zero_grad()
        out = gnn(data)
        loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=8.0, seed=4)
        loss.backward()
        return loss

    fb()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fb()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static = fb()
    g.replay()
    torch.cuda.synchronize()
    want_loss = static.clone()
    want_grad = torch.cat([p.grad.reshape(-1) for p in gnn.parameters()]).clone()
    # a much larger eager batch forces every scratch buffer to grow
    big_model, big = make_problem(4, 700, 128, B=2, seed=3)
    gbig = _hip_model(big_model, 2)
    _step(gbig, pfsgnn.BipartiteData(big.edge_index, big.x_s.float(), big.x_t.float(),
                                     big.x_e.float(), big.x_u.float()), big.x_t.float().cuda())
    torch.cuda.empty_cache()
    junk = torch.full((64 << 20,), float("nan"), device="cuda")   # reuse freed blocks
    gnn.load_state_dict(sd)
    g.replay()
    torch.cuda.synchronize()
    del junk
    assert torch.equal(static, want_loss)
    got = torch.cat([p.grad.reshape(-1) for p in gnn.parameters()])
    assert torch.equal(got, want_grad)


def test_fused_adam_weight_decay_skips_gradless_parameters():
    """torch.optim.Adam skips parameters whose .grad is None (decoder_s and the
    last block's S/T/Global models under the train.py loss)."""
    import pfsgnn
    model, graph = make_problem(1, 48, 12, B=2, seed=6)
    gnn = _hip_model(model, 2)
    data = pfsgnn.BipartiteData(graph.edge_index, graph.x_s.float(), graph.x_t.float(),
                                graph.x_e.float(), graph.x_u.float())
    ci = graph.x_t.float().cuda()
    opt = pfsgnn.FusedAdam(gnn.parameters(), lr=1e-2, weight_decay=0.05)
    ref_params = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in gnn.named_parameters()}
    ropt = torch.optim.Adam(list(ref_params.values()), lr=1e-2, weight_decay=0.05)
    for it in range(2):
        _step(gnn, data, ci, seed=10 + it)
        live = {n for n, p in gnn.named_parameters() if getattr(p, "_pf_live", True)}
        assert "decoder_s.0.weight" not in live and "mpb.1.s_model.norm.weight" not in live
        assert "decoder_e.0.weight" in live and "mpb.0.s_model.norm.weight" in live
        for n, p in gnn.named_parameters():
            ref_params[n].grad = p.grad.detach().cpu().clone() if n in live else None
        opt.step()
        ropt.step()
    for n, p in gnn.named_parameters():
        torch.testing.assert_close(p.detach().cpu(), ref_params[n].detach(), rtol=1e-5, atol=1e-6,
                                   msg=n)


def test_completeness_min_propagates_nan():
    """train.py:53-54: torch.min over a completeness containing 0/0 is NaN."""
    from pfsgnn.engine import Dims
    from pfsgnn.gnn import backend
    be = backend()
    d = Dims(1, 8, 4, 10)
    n_prime = torch.tensor([3.0, 0.0, 5.0, 1.0], device="cuda")
    ci = torch.tensor([[2.0, 2.0, 2.0, 2.0], [10.0, 0.0, 10.0, 10.0]], device="cuda")
    fiber_time = torch.full((8,), 40.0, device="cuda")
    tvar = torch.ones(4, device="cuda")
    loss, utils, variance, Gn, Gf, Gv = be.loss_finalize(d, n_prime, fiber_time, tvar, ci, 0.1,
                                                         0.1, 42.0, 10.0, 2000.0, 1.0)
    torch.cuda.synchronize()
    assert torch.isnan(utils).all().item() and torch.isnan(loss).all().item()
    comp = n_prime.cpu() / (ci[1].cpu() / 10.0)
    assert torch.isnan(torch.min(comp))


def test_fused_adam_tracks_live_sets_like_torch_adam():
    """GNN.node_prediction / edge_prediction run decoder_s /
    decoder_e through the module-level MLP autograd function, whose backward
    must mark the decoder parameters live, and a parameter whose gradient
    comes and goes keeps torch.optim.Adam's per-parameter step count and is
    left untouched (no moment decay, no weight decay) on steps without one.
    Steps alternate between the fused train.py loss and a loss on
    node_prediction(out.x_s) + the unfused edge_prediction(out.x_e), so the
    live set changes every step; weight decay on."""
    import pfsgnn
    from pfsgnn.train import loss_function
    model, graph = make_problem(1, 48, 12, B=2, seed=6)
    gnn = _hip_model(model, 2)
    data = pfsgnn.BipartiteData(graph.edge_index, graph.x_s.float(), graph.x_t.float(),
                                graph.x_e.float(), graph.x_u.float())
    ci = graph.x_t.float().cuda()
    opt = pfsgnn.FusedAdam(gnn.parameters(), lr=1e-2, weight_decay=0.05)
    ref_params = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in gnn.named_parameters()}
    ropt = torch.optim.Adam(list(ref_params.values()), lr=1e-2, weight_decay=0.05)
    for it in range(4):
        opt.zero_grad()
        gnn.zero_grad()
        out = gnn(data)
        if it % 2 == 0:
            loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=10.0, seed=20 + it)
        else:
            pred = gnn.node_prediction(out.x_s)
            loss = (pred * torch.linspace(-1, 1, pred.shape[1], device="cuda")).sum() \
                + 1e-3 * gnn.edge_prediction(out.x_e).sum()
        loss.backward()
        torch.cuda.synchronize()
        live = {n for n, p in gnn.named_parameters() if p._pf_live}
        if it % 2 == 0:
            assert "decoder_s.0.weight" not in live and "decoder_e.0.weight" in live
        else:
            assert "decoder_s.0.weight" in live and "decoder_e.2.bias" in live
        for n, p in gnn.named_parameters():
            ref_params[n].grad = p.grad.detach().cpu().clone() if n in live else None
        opt.step()
        ropt.step()
    for n, p in gnn.named_parameters():
        torch.testing.assert_close(p.detach().cpu(), ref_params[n].detach(), rtol=1e-5, atol=1e-6,
                                   msg=n)
