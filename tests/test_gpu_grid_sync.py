"""The device-wide barrier of the fused class-side launches (k_class_tail_fwd,
k_class_bwd; csrc/pfsgnn_mlp.hip grid_sync) in both of its forms: the default
sc1 hand-off (relaxed agent-scope counter, sc1 stores and loads of the handed-
over partials) and the acq_rel form (release arrival, acquire poll).  The
barrier only orders, so two training steps under either form must give bitwise
the same loss, gradients, parameters and BatchNorm buffers, at a grid of ~200
workgroups (24 graphs x 128 classes).  And no barrier may have timed out."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _two_steps(fenced):
    import pfsgnn
    from pfsgnn import native
    from pfsgnn.train import loss_function
    native.set_grid_sync_fenced(fenced)
    try:
        G, NF, NC, F = 24, 300, 128, 10
        torch.manual_seed(0)
        gnn = pfsgnn.GNN(B=3, Fdim=F, T=NC, F_s=1, F_t=2).cuda()
        gnn.train()
        gen = torch.Generator().manual_seed(5)
        ci = torch.cat([torch.randint(2, 13, (G * NC, 1), generator=gen).float(),
                        torch.randint(1000, 100000, (G * NC, 1), generator=gen).float()], 1)
        e = torch.arange(G * NF * NC)
        ei = torch.stack([e // NC, (e // (NF * NC)) * NC + e % NC])
        data = pfsgnn.BipartiteData(ei, torch.arange(NF, dtype=torch.float).repeat(G).reshape(-1, 1),
                                    ci, 2.0 + 8.0 * torch.rand(G * NF * NC, F, generator=gen),
                                    torch.zeros(G, F))
        ci = ci.cuda()
        opt = pfsgnn.FusedAdam(gnn.parameters(), lr=1e-3)
        losses, grads = [], None
        for s in range(2):
            gnn.zero_grad()
            out = gnn(data)
            loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=8.0, seed=11 + s)
            loss.backward()
            grads = torch.cat([p.grad.reshape(-1) for p in gnn.parameters() if p.grad is not None])
            opt.step()
            losses.append(loss.detach())
        torch.cuda.synchronize()
        params = torch.cat([p.detach().reshape(-1) for p in gnn.parameters()])
        bufs = torch.cat([b.detach().double().reshape(-1) for b in gnn.buffers()])
        return torch.stack(losses).cpu(), grads.cpu(), params.cpu(), bufs.cpu()
    finally:
        native.set_grid_sync_fenced(False)


def test_grid_sync_forms_bitwise_equal():
    from pfsgnn import native
    a = _two_steps(False)
    b = _two_steps(True)
    for x, y, what in zip(a, b, ("loss", "grads", "params", "buffers")):
        assert torch.isfinite(x).all(), what
        assert torch.equal(x, y), what
    assert native.sync_faults() == 0
