"""Pin the CPU oracle against the reference's own shipped fixtures (CPU only).

The reference cannot run here (torch_geometric / torch_scatter absent), so no
output vectors of it exist.  Its shipped data pins the oracle instead:
* graphs/graph-0.pt (raw storages, tests/golden/graph0.npz): the graph builder;
* params/model_gnn_0.pth + models/model_gnn_0.pth (tests/golden/ckpt_*.npz):
  the module tree (keys, shapes, order) and -- through the BatchNorm running
  statistics the reference's training run recorded -- the forward wiring.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_gnn
from oracle.ref_graph import pad_properties, to_graph, train_graph

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_ckpt(name):
    z = np.load(os.path.join(GOLD, name))
    return {k: torch.as_tensor(z[k]) for k in z.files if k != "epoch"}


# ------------------------------------------------------------------ graph-0
def test_graph0_is_to_graph_of_increasing_txt():
    z = np.load(os.path.join(GOLD, "graph0.npz"))
    ei = z["edge_index"].astype(np.int64)
    assert ei.shape == (2, 24000)
    src, tgt = ei
    assert (np.diff(src) >= 0).all(), "graph.py:49 sorts edges by source"
    for f in range(2000):
        assert sorted(tgt[f * 12:(f + 1) * 12].tolist()) == list(range(12))
    classes = np.load(os.path.join(GOLD, "classes.npz"))
    props = pad_properties(classes["increasing"], 10)          # config.datafile, graph.py:76-77
    assert np.array_equal(z["x_t"], props.astype(np.float32))
    assert tuple(z["x_s_shape"]) == (2000, 10) and float(z["x_s_absmax"]) == 0.0
    assert tuple(z["x_e_shape"]) == (24000, 10) and float(z["x_e_absmax"]) == 0.0
    assert tuple(z["u_shape"]) == (1, 10) and float(z["u_absmax"]) == 0.0
    ei2, xs, xt, xe, u = to_graph(props, 2000, 10)
    a = {(int(s), int(t)) for s, t in ei.T}
    b = {(int(s), int(t)) for s, t in ei2.numpy().T}
    assert a == b
    assert np.array_equal(xt.numpy(), z["x_t"])


def test_graph0_edge_order_is_not_canonical():
    """graph-0 lists each fiber's classes in (unstable) argsort order: the HIP
    path must honour edge_index, not assume c = e % NC."""
    z = np.load(os.path.join(GOLD, "graph0.npz"))
    tgt = z["edge_index"][1].astype(np.int64)
    assert (tgt != np.tile(np.arange(12), 2000)).any()


# ------------------------------------------------------------------ checkpoint
@pytest.mark.parametrize("name", ["ckpt_params.npz", "ckpt_models.npz"])
def test_checkpoint_keys_match_oracle_and_product(name):
    sd = load_ckpt(name)
    mo = ref_gnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2)
    assert list(mo.state_dict().keys()) == list(sd.keys())
    for k, v in mo.state_dict().items():
        assert tuple(v.shape) == tuple(sd[k].shape), k
    import pfsgnn
    from pfsgnn.engine import param_names
    mp = pfsgnn.GNN(B=3, Fdim=10, T=12, F_s=1, F_t=2)
    assert list(mp.state_dict().keys()) == list(sd.keys())
    assert [n for n, _ in mp.named_parameters()] == param_names(3)
    missing, unexpected = mp.load_state_dict(sd, strict=True)
    assert not missing and not unexpected


def _bn_pin(model_cls, sd, seed=0):
    classes = np.load(os.path.join(GOLD, "classes.npz"))
    ei, xs, xt, xe, u = train_graph(classes["increasing"], 2000, 10,
                                    generator=torch.Generator().manual_seed(seed))
    m = model_cls(B=3, Fdim=10, T=12, F_s=1, F_t=2).double()
    m.load_state_dict(sd)
    m.train()
    calls = {}
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.register_forward_hook(
                lambda mod, i, o, name=name: calls.setdefault(name, []).append(
                    (i[0].mean(0), i[0].var(0))))
    with torch.no_grad():
        m(ref_gnn.Graph(ei, xs.double(), xt.double(), xe.double(), u.double()))
    err = {}
    for name, cl in calls.items():
        mom = 0.1
        if len(cl) == 2:     # two updates per step: steady state of the EMA
            a, b = (1 - mom) * mom, mom
            pm = (a * cl[0][0] + b * cl[1][0]) / (a + b)
            pv = (a * cl[0][1] + b * cl[1][1]) / (a + b)
        else:
            pm, pv = cl[0]
        rm, rv = sd[name + ".running_mean"].double(), sd[name + ".running_var"].double()
        err[name] = max(((pm - rm).abs() / rv.sqrt()).max().item(), ((pv - rv).abs() / rv).max().item())
    return err


@pytest.mark.parametrize("name", ["ckpt_params.npz", "ckpt_models.npz"])
def test_bn_running_stats_pin_forward_wiring(name):
    """The oracle forward, run with the reference's trained weights on the
    train.py graph, reproduces the BatchNorm running statistics the reference's
    own run recorded: EdgeModel norms (applied twice per step, hence
    num_batches_tracked = 2 x epochs) to < 5 %, SModel/TModel norms to < 25 %
    (their statistics are sharper functions of the last steps' weights)."""
    sd = load_ckpt(name)
    if name == "ckpt_params.npz":
        assert int(sd["mpb.0.edge_model.norm.num_batches_tracked"]) == 2 * int(
            sd["mpb.0.s_model.norm.num_batches_tracked"])
    err = _bn_pin(ref_gnn.GNN, sd)
    for k, v in err.items():
        bound = 0.05 if "edge_model" in k else 0.25
        assert v < bound, (k, v)


class _SingleNormEdge(ref_gnn.EdgeModel):
    """Mutation: BatchNorm applied once (what the reference's code *looks* like)."""

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None):
        src, tgt = edge_index
        h = torch.cat([x_s[src], x_t[tgt], edge_attr, u.expand(edge_attr.size(0), -1)], dim=-1)
        return self.norm(self[2](self[1](self[0](h))))


class _SwappedEdge(ref_gnn.EdgeModel):
    """Mutation: source/target features swapped in the concatenation."""

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None):
        src, tgt = edge_index
        h = torch.cat([x_t[tgt], x_s[src], edge_attr, u.expand(edge_attr.size(0), -1)], dim=-1)
        return self.norm(torch.nn.Sequential.forward(self, h))


@pytest.mark.parametrize("mutant", [_SingleNormEdge, _SwappedEdge])
def test_bn_pin_rejects_wrong_wiring(mutant, monkeypatch):
    sd = load_ckpt("ckpt_params.npz")
    monkeypatch.setattr(ref_gnn, "EdgeModel", mutant)
    err = _bn_pin(ref_gnn.GNN, sd)
    worst_edge = max(v for k, v in err.items() if "edge_model" in k)
    assert worst_edge > 0.3, err
