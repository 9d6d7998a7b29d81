"""Full training-step parity at Fdim 8 and 16 on complete graphs.

The complete-graph step has fused backward forms that the Fdim-10 parity cases
cover but the sparse Fdim-8/16 cases do not reach (the sliced path keeps them
off):
  * node_mlp_2's backward forming SModel's moment coefficients in its epilogue
    (pfsgnn_mlp_bwd_pre's coef; engine._mom_epi_ok accepts Fdim 8, where the
    message width 2F = 16 leaves only lane group 0 of the epilogue active);
  * SModel's BatchNorm backward sums made by TModel's fiber reduction
    (target_bwd(bn_sums=...), mlp_bwd(bn_part=...));
  * the last block's EdgeModel BatchNorm sums made by the loss backward.
Each case runs with those forms on (the default) and off (PFSGNN_MOM_EPI=0,
PFSGNN_FIBER_BN_SUMS=0, PFSGNN_LOSS_BN_SUMS=0: the separate launches), and
both are held to the fp64 oracle with test_gpu_parity's bar; NF is not a
multiple of 64 so the last fiber group of every edge block is ragged."""
import pytest
import torch

from harness import make_problem
from test_gpu_parity import check, oracle_step, ours_step

pytestmark = pytest.mark.gpu

UNFUSED = {"PFSGNN_MOM_EPI": "0", "PFSGNN_FIBER_BN_SUMS": "0", "PFSGNN_LOSS_BN_SUMS": "0"}


@pytest.mark.parametrize("path", ["mfma", "mfma32"])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("F,G,NF,NC,B", [(8, 2, 70, 12, 2), (8, 1, 130, 20, 3), (16, 2, 70, 12, 2)])
def test_fdim_training_step_matches_oracle(F, G, NF, NC, B, fused, path, monkeypatch):
    import pfsgnn
    if not fused:
        for k, v in UNFUSED.items():
            monkeypatch.setenv(k, v)
    prev = pfsgnn.get_edge_path()
    pfsgnn.set_edge_path(path)
    try:
        model, graph = make_problem(G, NF, NC, F=F, B=B, seed=F + NF + NC)
        seed, sharp = 500 + NC, 8.0
        m64, o64, l64 = oracle_step(model, graph, G, NF, NC, seed, sharp, torch.float64)
        ref32 = [oracle_step(model, graph, G, NF, NC, seed, sharp, torch.float32, reverse=rv)
                 for rv in (False, True)]
        gnn, out, loss = ours_step(model, graph, G, NF, NC, B, seed, sharp, F=F)
        check("loss", loss, l64, [r[2] for r in ref32])
        for nm in ("x_e", "x_s", "x_t", "x_u"):
            check(nm, getattr(out, nm), getattr(o64, nm), [getattr(r[1], nm) for r in ref32])
        p64 = dict(m64.named_parameters())
        p32s = [dict(r[0].named_parameters()) for r in ref32]
        for name, p in gnn.named_parameters():
            r64 = p64[name].grad if p64[name].grad is not None else torch.zeros_like(p64[name])
            r32 = [q[name].grad if q[name].grad is not None else torch.zeros_like(q[name])
                   for q in p32s]
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            check("grad " + name, g, r64, r32)
        b64 = m64.state_dict()
        b32s = [r[0].state_dict() for r in ref32]
        for k, v in gnn.state_dict().items():
            if "running" in k:
                check(k, v.double(), b64[k].double(), [b[k].double() for b in b32s])
    finally:
        pfsgnn.set_edge_path(prev)
