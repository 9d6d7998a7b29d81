"""Pin the loss and the backward with the reference's own optimizer state (CPU).

``params/model_gnn_0.pth`` holds, beside the trained weights, the state of the
torch.optim.Adam that trained them (train.py:154-165, extracted weights-only
into tests/golden/ckpt_adam.npz by make_golden.py): the step count (40000),
the indices of the parameters that have state, and per parameter ``exp_avg``
(m: the 10-step EMA of its gradients, beta1 = 0.9) and ``exp_avg_sq`` (v: the
1000-step EMA of the squared gradients).  Two checks follow from it:

* exact: Adam keeps state for exactly the parameters whose ``.grad`` the
  reference's backward set (torch.optim.Adam skips ``grad is None``), so the
  oracle's set of parameters with a gradient under train.py's loss must be
  those 80 of 109 indices.  The 29 without state are decoder_s and block 2's
  s_model / t_model / global_model: dead under train.py's loss (only x_e
  reaches it, gnn.py:307-312, train.py:42).
* statistical: at the trained weights theta_T (sharpness 20 * 39999/40000,
  train.py:137) the gradient, averaged over softfloor noise and train.py's
  random edge features, points along the momentum m -- here AGAINST it: the
  trained weights oscillate about a minimum, and after a step the gradient
  pulls back along the direction just travelled (cos < 0).  Compared in
  Adam's own normalised coordinates (g / sqrt(v), m / sqrt(v)):
    - ``global``: cosine over every parameter element with state;
    - ``tensor``: the same after scaling each tensor to unit rms, so the
      large-gradient tensors do not dominate.
  The mean runs over 32 draws of train.py's edge features and of softfloor's
  noise (the product's generator, seeds 1000..1031); fewer draws leave the
  statistic dominated by the noise (16 draws: oracle tensor cosines from
  -0.33 to +0.17 over three noise seeds).  With 32 draws the oracle reaches
  global -0.66 / tensor -0.61 (and -0.59/-0.58, -0.57/-0.55 with noise seeds
  5000.., 9000..); the bounds are -0.55 / -0.50, both required.  Three
  plausible mis-restatements miss them at every one of those seeds
  (measured; global / tensor at seed 1000): pfiber = 1.0, the loss_function
  signature default instead of the 0.1 train.py passes (-0.46 / -0.52);
  the variance term's sign flipped (-0.52 / -0.37); GlobalModel's RMSNorm
  applied once instead of twice (+0.47 / -0.03).

The draws are seeded, so the statistic is deterministic; the margins are
what the mutants show.  tests/test_gpu_adam_pin.py runs the same check on the
HIP path's gradients, with the same noise.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_gnn
from oracle.ref_graph import train_graph
from oracle.ref_train import loss_function

GOLD = os.path.join(os.path.dirname(__file__), "golden")
NDRAW = 32
SHARP = 20.0 * 39999 / 40000            # train.py:137 at the last epoch
GLOBAL_BOUND, TENSOR_BOUND = -0.55, -0.50


def adam_state():
    z = np.load(os.path.join(GOLD, "ckpt_adam.npz"))
    idx = [int(i) for i in z["indices"]]
    return z, idx


def model_state():
    z = np.load(os.path.join(GOLD, "ckpt_params.npz"))
    return {k: torch.as_tensor(z[k]) for k in z.files if k != "epoch"}


NOISE_SEED0 = 1000


def draw(d, noise0=None):
    """train.py's graph (train.py:88-104: x_e ~ U(2, 10)) and softfloor's
    uniforms for draw d: the product's in-kernel generator with seed
    noise0 + d (tests/noise_ref.py reproduces it bit for bit), so the oracle
    here and the HIP path (tests/test_gpu_adam_pin.py) see the same noise."""
    from noise_ref import uniform_numpy
    classes = np.load(os.path.join(GOLD, "classes.npz"))["increasing"]
    ei, xs, xt, xe, u = train_graph(classes, 2000, 10, generator=torch.Generator().manual_seed(d))
    seed = (NOISE_SEED0 if noise0 is None else noise0) + d
    uni = torch.as_tensor(uniform_numpy(seed, 24000), dtype=torch.float64)
    return ei, xs, xt, xe, u, uni


def oracle_grads(ndraw=NDRAW, pfiber=0.1, wvar=1.0, global_cls=None, noise0=None):
    """Per draw, the list of parameter gradients (None where autograd gave none)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    orig = ref_gnn.GlobalModel
    if global_cls is not None:
        ref_gnn.GlobalModel = global_cls
    try:
        m = ref_gnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2).double()
    finally:
        ref_gnn.GlobalModel = orig
    m.load_state_dict(model_state())
    m.train()
    out_g = []
    for d in range(ndraw):
        ei, xs, xt, xe, u, uni = draw(d, noise0)
        g = ref_gnn.Graph(ei, xs.double(), xt.double(), xe.double(), u.double())
        m.zero_grad(set_to_none=True)
        out = m(g)
        loss, _ = loss_function(m, out.x_e, g.x_t, 1, 2000, 12, pclass=0.1, pfiber=pfiber, wvar=wvar,
                                sharpness=SHARP, uniform=uni)
        loss.backward()
        out_g.append([None if p.grad is None else p.grad.detach().double().clone()
                      for p in m.parameters()])
    return out_g


def direction_stats(grads):
    """(global, tensor-normalised) cosine between the mean gradient and Adam's
    momentum, both in Adam's normalised coordinates (divided by sqrt(v))."""
    z, idx = adam_state()
    us, ws = [], []
    for i in idx:
        g = torch.stack([torch.as_tensor(d[i]).double().cpu() for d in grads]).mean(0).reshape(-1)
        m = torch.as_tensor(z[f"exp_avg_{i}"]).double().reshape(-1)
        v = torch.as_tensor(z[f"exp_avg_sq_{i}"]).double().reshape(-1).sqrt()
        ok = v > 1e-30
        us.append(g[ok] / v[ok])
        ws.append(m[ok] / v[ok])

    def cos(a, b):
        return float(torch.nn.functional.cosine_similarity(a, b, dim=0))

    unit = lambda x: x / (x.pow(2).mean().sqrt() + 1e-300)  # noqa: E731
    return (cos(torch.cat(us), torch.cat(ws)),
            cos(torch.cat([unit(x) for x in us]), torch.cat([unit(x) for x in ws])))


def matches_adam(stats):
    return stats[0] <= GLOBAL_BOUND and stats[1] <= TENSOR_BOUND


@pytest.fixture(scope="module")
def oracle_g():
    return oracle_grads()


def test_adam_state_fixture():
    z, idx = adam_state()
    assert int(z["n_params"]) == 109 and len(idx) == 80
    assert (z["step"] == 40000).all()
    assert float(z["lr"]) == 5e-4 and float(z["weight_decay"]) == 0.0     # config.py lr, Adam()
    assert tuple(z["betas"]) == (0.9, 0.999)


def test_live_parameters_are_the_adam_state_indices(oracle_g):
    """Exact: the parameters the oracle's backward gives a gradient are the
    ones the reference's Adam kept state for."""
    _, idx = adam_state()
    live = [i for i, g in enumerate(oracle_g[0]) if g is not None]
    assert live == idx
    names = [n for n, _ in ref_gnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2).named_parameters()]
    dead = {names[i].split(".")[0] if names[i].startswith("decoder") else ".".join(names[i].split(".")[:3])
            for i in range(109) if i not in idx}
    assert dead == {"decoder_s", "mpb.2.s_model", "mpb.2.t_model", "mpb.2.global_model"}


def test_gradient_direction_matches_adam_momentum(oracle_g):
    stats = direction_stats(oracle_g)
    print("oracle vs Adam state: global cos %+.3f, tensor-normalised cos %+.3f" % stats)
    assert matches_adam(stats), stats


class _SingleRMSGlobal(ref_gnn.GlobalModel):
    """Mutation: RMSNorm applied once (what gnn.py:223 *looks* like)."""

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None, t_batch=None):
        h = torch.cat([u, x_s.mean(0, keepdim=True), x_t.mean(0, keepdim=True)], -1)
        return self.norm(self[2](self[1](self[0](h))))


@pytest.mark.parametrize("mutant", ["pfiber_default", "variance_sign", "single_rmsnorm"])
def test_adam_pin_rejects_mutants(mutant):
    kw = {"pfiber_default": dict(pfiber=1.0), "variance_sign": dict(wvar=-1.0),
          "single_rmsnorm": dict(global_cls=_SingleRMSGlobal)}[mutant]
    stats = direction_stats(oracle_grads(**kw))
    print(f"{mutant}: global cos {stats[0]:+.3f}, tensor-normalised cos {stats[1]:+.3f}")
    assert not matches_adam(stats), stats
