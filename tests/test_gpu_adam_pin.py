"""The reference-state pin of tests/test_adam_pin.py on the HIP path: the
product's training step (pfsgnn.GNN + pfsgnn.train.loss_function, through
libpfsgnn.so) at the reference's trained weights against the reference's own
Adam state (params/model_gnn_0.pth's optim_state).

* exact: the parameters the fused backward marks live (the ones FusedAdam
  updates, ``p._pf_live``) are the 80 indices the reference's Adam kept
  state for;
* statistical: the mean gradient over the same 32 seeded draws of train.py's
  edge features and softfloor noise as the oracle's test (the product's own
  counter-based generator, which the oracle's test reproduces bit for bit)
  points against Adam's momentum in Adam's normalised coordinates, with the
  bounds the oracle is held to.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from test_adam_pin import (NDRAW, NOISE_SEED0, SHARP, adam_state, direction_stats, draw,  # noqa: E402
                           matches_adam, model_state)


def test_hip_gradients_match_reference_adam_state():
    import pfsgnn
    from pfsgnn.train import loss_function
    gnn = pfsgnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2).cuda()
    gnn.load_state_dict(model_state())
    gnn.train()
    _, idx = adam_state()
    grads = []
    for d in range(NDRAW):
        ei, xs, xt, xe, u, _ = draw(d)
        data = pfsgnn.BipartiteData(ei, xs.float(), xt.float(), xe.float(), u.float())
        gnn.zero_grad()
        out = gnn(data)
        loss, _ = loss_function(out, xt.float().cuda(), pclass=0.1, pfiber=0.1, sharpness=SHARP,
                                seed=NOISE_SEED0 + d)
        loss.backward()
        params = list(gnn.parameters())
        live = [i for i, p in enumerate(params) if getattr(p, "_pf_live", False)]
        assert live == idx, (d, live)
        grads.append([p.grad.detach().double().cpu().clone() for p in params])
    torch.cuda.synchronize()
    stats = direction_stats(grads)
    print("HIP path vs Adam state: global cos %+.3f, tensor-normalised cos %+.3f" % stats)
    assert matches_adam(stats), stats
