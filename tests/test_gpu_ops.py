"""Op-level parity: every HIP op of libpfsgnn.so vs the same op emulated in
float64 torch on identical inputs (tests/emu_backend.py), at several batch
geometries (NC below / at / above a wave, non-power-of-two NC, several graphs).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from emu_backend import EmuBackend, Dims as EDims  # noqa: E402

GEOMS = [(1, 37, 12), (2, 50, 16), (1, 9, 128), (3, 21, 5), (2, 7, 200), (1, 33, 64)]


@pytest.fixture(scope="module")
def hb():
    from pfsgnn.native import HipBackend
    return HipBackend()


def r(*shape, scale=1.0, off=0.0, gen=None):
    return (torch.randn(*shape, generator=gen, dtype=torch.float64) * scale + off)


def cuda(t):
    return None if t is None else t.to(torch.float32).cuda().contiguous()


def cpu(t):
    return None if t is None else t.detach().double().cpu()


def close(a, b, rtol=2e-4, atol=1e-5, name=""):
    a, b = cpu(a), cpu(b)
    scale = b.abs().max().item() if b.numel() else 1.0
    err = (a - b).abs().max().item() if b.numel() else 0.0
    assert err <= atol + rtol * max(scale, 1e-30), f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def dims(G, NF, NC, F=10):
    from pfsgnn.engine import Dims
    return Dims(G, NF, NC, F), EDims(G, NF, NC, F)


@pytest.fixture(params=["mfma", "mfma32", "valu", "bf16x3", "bf16x6"])
def prec(request):
    import pfsgnn
    prev = pfsgnn.get_edge_path()
    pfsgnn.set_edge_path(request.param)
    yield request.param
    pfsgnn.set_edge_path(prev)


# (+ blocks of one and of two classes: the edge_mlp_bwd class pipeline's
# shortest streams, class_stream_pipe)
EDGE_CASES = [(G, NF, NC, 10) for G, NF, NC in GEOMS] + [(2, 50, 16, 8), (1, 33, 64, 8),
                                                         (2, 50, 16, 16), (1, 70, 24, 16),
                                                         (1, 9, 1, 10), (2, 30, 2, 10)]


@pytest.mark.parametrize("G,NF,NC,F", EDGE_CASES)
def test_edge_ops(hb, prec, G, NF, NC, F):
    """Every per-edge kernel on every fp32-class path (fp32 VALU, MFMA, the
    bf16x3 contractions) against the float64 emulation, at every supported
    Fdim (the bf16 paths are built for Fdim 10)."""
    if prec == "bf16x3" and F != 10:
        pytest.skip("bf16x3 is instantiated for Fdim 10 (bf16x6 runs the mfma arithmetic there)")
    gen = torch.Generator().manual_seed(G * 1000 + NF * 10 + NC + F)
    # Inputs on a grid on which every FIRST-layer pre-activation is computed exactly
    # by every path (fp64 emulation, fp32 fmaf chains, fp32 MFMA, and bf16x3,
    # whose hi + lo split holds a 16-bit significand exactly): weights
    # bf16-exact (multiples of 1/64, |w| < 2), edge inputs with <= 16 significant
    # bits, node parts on a 1/256 grid, sums below 2^24 grid units.  LeakyReLU's
    # slope then switches on the same edges in every path; on random data an edge
    # whose pre-activation lies within rounding of 0 takes the other slope in one
    # path (a kink flip: an O(1) change of that edge's gradient, not an error).
    def q(t, step):
        return torch.round(t / step) * step
    emu = EmuBackend()
    d, de = dims(G, NF, NC, F)
    E, NS, NT = d.E, d.NS, d.NT
    xe = q(r(F, E, scale=2, off=3, gen=gen), 1 / 16)
    xsc, xsh = q(r(F, gen=gen) * 0.5 + 1, 1 / 16), q(r(F, gen=gen), 1 / 16)
    Ps, Pt = q(r(4 * F, NS, gen=gen), 1 / 256), q(r(4 * F, NT, gen=gen), 1 / 256)
    W1, W2, b2 = q(r(4 * F, 4 * F, scale=0.3, gen=gen), 1 / 64), r(F, 4 * F, scale=0.3, gen=gen), r(F, gen=gen)
    # edge_mlp_fwd
    y_h, mu_h, var_h = hb.edge_mlp_fwd(d, cuda(xe), cuda(xsc), cuda(xsh), cuda(Ps), cuda(Pt), cuda(W1), cuda(W2), cuda(b2))
    y_e, mu_e, var_e = emu.edge_mlp_fwd(de, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
    close(y_h, y_e, name="y"); close(mu_h, mu_e, name="mu"); close(var_h, var_e, name="var")
    y = q(y_e, 1 / 4)
    sc, sh = q(r(F, gen=gen) * 0.3 + 1, 1 / 8), q(r(F, gen=gen), 1 / 8)
    # source_fwd
    Qt = q(r(2 * F, NT, gen=gen), 1 / 256)
    Ws1, Ws2, bs2 = q(r(2 * F, 2 * F, scale=0.3, gen=gen), 1 / 64), r(2 * F, 2 * F, scale=0.3, gen=gen), r(2 * F, gen=gen)
    hs_h = torch.zeros(8 * F, NS, device="cuda")
    hs_e = torch.zeros(8 * F, NS, dtype=torch.float64)
    mom_h = hb.source_fwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Qt), cuda(Ws1), cuda(Ws2), cuda(bs2), hs_h)
    mom_e = emu.source_fwd(de, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_e)
    for i, nm in enumerate(["mean", "c2", "c3", "c4"]):
        close(mom_h[i], mom_e[i], rtol=1e-3, name=nm)
    close(hs_h, hs_e, rtol=2e-3, atol=1e-3, name="hs")
    # target_fwd / bwd
    Rs, Wt1 = q(r(2 * F, NS, gen=gen), 1 / 256), q(r(2 * F, 2 * F, scale=0.3, gen=gen), 1 / 64)
    close(hb.target_fwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Rs), cuda(Wt1)),
          emu.target_fwd(de, y, sc, sh, Rs, Wt1), name="hsum")
    g_hsum = r(2 * F, NT, gen=gen)
    dWt1_h = torch.zeros(2 * F, 2 * F, device="cuda")
    dWt1_e = torch.zeros(2 * F, 2 * F, dtype=torch.float64)
    GzT_h, gxe_h = hb.target_bwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Rs), cuda(Wt1), cuda(g_hsum), dWt1_h, want_gxe=True)
    GzT_e, gxe_e = emu.target_bwd(de, y, sc, sh, Rs, Wt1, g_hsum, dWt1_e, want_gxe=True)
    close(GzT_h, GzT_e, name="GzT"); close(gxe_h, gxe_e, name="gxeT"); close(dWt1_h, dWt1_e, name="dWt1")
    # source_bwd (with T part, g_next, BN sums)
    mean = r(2 * F, NS, gen=gen)
    coef = r(4, 2 * F, NS, gen=gen) * torch.tensor([1, 0.3, 0.1, 0.03], dtype=torch.float64)[:, None, None]
    g_next = r(F, E, gen=gen)
    mu1, inv1 = r(F, gen=gen), r(F, gen=gen).abs() + 0.5
    grads_h = [torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, device="cuda")]
    grads_e = [torch.zeros(2 * F, 2 * F, dtype=torch.float64), torch.zeros(2 * F, 2 * F, dtype=torch.float64), torch.zeros(2 * F, dtype=torch.float64)]
    out_h = hb.source_bwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Qt), cuda(Ws1), cuda(Ws2), cuda(bs2), cuda(mean), cuda(coef),
                          (cuda(Rs), cuda(Wt1), cuda(g_hsum)), cuda(g_next), (cuda(mu1), cuda(inv1)), *grads_h)
    out_e = emu.source_bwd(de, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, (Rs, Wt1, g_hsum), g_next, (mu1, inv1), *grads_e)
    for a, b, nm in zip(out_h, out_e, ["g_tot", "GzS", "Sg", "Sgx"]):
        close(a, b, rtol=5e-4, name=nm)
    for a, b, nm in zip(grads_h, grads_e, ["dWs1", "dWs2", "dbs2"]):
        close(a, b, rtol=5e-4, name=nm)
    # source_bwd without optional parts
    out_h = hb.source_bwd(d, cuda(y), None, None, cuda(Qt), cuda(Ws1), cuda(Ws2), cuda(bs2), cuda(mean), cuda(coef),
                          None, None, None, *[g.zero_() for g in grads_h])
    out_e = emu.source_bwd(de, y, None, None, Qt, Ws1, Ws2, bs2, mean, coef, None, None, None, *[g.zero_() for g in grads_e])
    close(out_h[0], out_e[0], rtol=5e-4, name="g_tot(bare)")
    close(out_h[1], out_e[1], rtol=5e-4, name="GzS(bare)")
    # edge bn sums
    Sg_h, Sgx_h = hb.edge_bn_grad_sums(d, cuda(g_next), cuda(y), cuda(mu1), cuda(inv1))
    Sg_e, Sgx_e = emu.edge_bn_grad_sums(de, g_next, y, mu1, inv1)
    close(Sg_h, Sg_e, name="Sg"); close(Sgx_h, Sgx_e, name="Sgx")
    # edge_mlp_bwd
    alpha, gam0, gam1 = r(F, gen=gen), r(F, gen=gen) * 0.1, r(F, gen=gen) * 0.1
    gh = [torch.zeros(4 * F, 4 * F, device="cuda"), torch.zeros(F, 4 * F, device="cuda"), torch.zeros(F, device="cuda")]
    ge = [torch.zeros(4 * F, 4 * F, dtype=torch.float64), torch.zeros(F, 4 * F, dtype=torch.float64), torch.zeros(F, dtype=torch.float64)]
    oh = hb.edge_mlp_bwd(d, cuda(g_next), cuda(alpha), cuda(gam0), cuda(gam1), cuda(y), cuda(xe), cuda(xsc), cuda(xsh),
                         cuda(Ps), cuda(Pt), cuda(W1), cuda(W2), *gh, want_gxe=True)
    oe = emu.edge_mlp_bwd(de, g_next, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2, *ge, want_gxe=True)
    for a, b, nm in zip(oh, oe, ["gxe", "GzEs", "GzEt"]):
        close(a, b, rtol=5e-4, name=nm)
    for a, b, nm in zip(gh, ge, ["dW1", "dW2", "db2"]):
        close(a, b, rtol=5e-4, name=nm)


@pytest.mark.parametrize("G,NF,NC", [(1, 37, 12), (2, 50, 16), (3, 700, 4), (4, 1001, 3)])
def test_concat_node_ops(hb, G, NF, NC):
    """lin_cat / wgrad_cat (the in-place torch.cat inputs of gnn.py:100/153/191/220):
    per-node blocks, a per-graph broadcast block and non-contiguous weight columns,
    against the emulation (which materialises the concatenation)."""
    gen = torch.Generator().manual_seed(11)
    emu = EmuBackend()
    N = G * NF
    for rows, M in [((10, 80, 10), 100), ((10, 10), 40), ((3, 5, 7, 2), 20)]:
        cols, c = [], 0
        for k in rows:
            cols.append(c)
            c += k + 1  # a gap column between blocks: weight columns are not contiguous
        K = c
        segs_e = []
        for i, k in enumerate(rows):
            bc = i == len(rows) - 1
            segs_e.append((r(k, G if bc else N, gen=gen), cols[i], bc))
        segs_h = [(cuda(X), col, bc) for X, col, bc in segs_e]
        W, b = r(M, K + 2, gen=gen), r(M, gen=gen)
        close(hb.lin_cat(cuda(W), segs_h, N, b=cuda(b), act_in=True, bscale=2.0),
              emu.lin_cat(W, segs_e, N, b=b, act_in=True, bscale=2.0), name=f"lin_cat{rows}")
        dY = r(M, N, gen=gen)
        dW_h, db_h = torch.zeros(M, K + 2, device="cuda"), torch.zeros(M, device="cuda")
        dW_e, db_e = torch.zeros(M, K + 2, dtype=torch.float64), torch.zeros(M, dtype=torch.float64)
        hb.wgrad_cat(cuda(dY), segs_h, dW_h, db=db_h, act_in=True, dbscale=0.5)
        emu.wgrad_cat(dY, segs_e, dW_e, db=db_e, act_in=True, dbscale=0.5)
        close(dW_h, dW_e, name=f"wgrad_cat{rows}"); close(db_h, db_e, name="db_cat")
        assert (dW_h[:, [cl - 1 for cl in cols[1:]]] == 0).all(), "gap columns written"


@pytest.mark.parametrize("G,NF,NC", [(1, 37, 12), (2, 50, 16), (1, 9, 128), (3, 700, 4)])
def test_node_ops(hb, G, NF, NC):
    gen = torch.Generator().manual_seed(7)
    emu = EmuBackend()
    N = G * NF
    for (M, K) in [(10, 1), (40, 10), (100, 100), (10, 100), (3, 7)]:
        W, X, b = r(M, K + 3, gen=gen), r(K, N, gen=gen), r(M, gen=gen)
        close(hb.lin(cuda(W), 2, K, cuda(X), b=cuda(b), act_in=True, bscale=3.0),
              emu.lin(W, 2, K, X, b=b, act_in=True, bscale=3.0), name=f"lin{M}x{K}")
        dY, Z = r(M, N, gen=gen), r(K, N, gen=gen)
        close(hb.lin_t(cuda(W), 2, K, cuda(dY), z=cuda(Z)), emu.lin_t(W, 2, K, dY, z=Z), name="lin_t")
        dW_h, db_h = torch.zeros(M, K + 3, device="cuda"), torch.zeros(M, device="cuda")
        dW_e, db_e = torch.zeros(M, K + 3, dtype=torch.float64), torch.zeros(M, dtype=torch.float64)
        hb.wgrad(cuda(dY), cuda(X), dW_h, col0=2, db=db_h, act_in=True, dbscale=2.0)
        emu.wgrad(dY, X, dW_e, col0=2, db=db_e, act_in=True, dbscale=2.0)
        close(dW_h, dW_e, name="wgrad"); close(db_h, db_e, name="db")
    C = 10
    X = r(C, N, scale=3, off=5, gen=gen)
    gamma, beta = r(C, gen=gen).abs() + 0.5, r(C, gen=gen)
    rm_h, rv_h = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    rm_e, rv_e = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    Yh, muh, varh = hb.bn_fwd(cuda(X), cuda(gamma), cuda(beta), rm_h, rv_h, 0.1, 1e-5)
    Ye, mue, vare = emu.bn_fwd(X, gamma, beta, rm_e, rv_e, 0.1, 1e-5)
    close(Yh, Ye, name="bn"); close(rm_h, rm_e, name="rm"); close(rv_h, rv_e, name="rv")
    dY = r(C, N, gen=gen)
    dg_h, dbt_h = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dg_e, dbt_e = torch.zeros(C, dtype=torch.float64), torch.zeros(C, dtype=torch.float64)
    close(hb.bn_bwd(cuda(dY), cuda(X), muh, varh, cuda(gamma), 1e-5, dg_h, dbt_h),
          emu.bn_bwd(dY, X, mue, vare, gamma, 1e-5, dg_e, dbt_e), rtol=1e-3, name="bn_bwd")
    close(dg_h, dg_e, name="dgamma"); close(dbt_h, dbt_e, name="dbeta")
    close(hb.graph_reduce(cuda(X), G, mean=True), emu.graph_reduce(X, G, mean=True), name="greduce")
    src = r(C, G, gen=gen)
    oh, oe = cuda(X), X.clone()
    hb.graph_bcast_add(oh, cuda(src), 0.5)
    emu.graph_bcast_add(oe, src, 0.5)
    close(oh, oe, name="bcast")
    U = r(C, G, gen=gen)
    w = r(C, gen=gen).abs() + 0.5
    eps = float(torch.finfo(torch.float32).eps)
    Yh, sh_ = hb.rms2_fwd(cuda(U), cuda(w), eps)
    Ye, se_ = emu.rms2_fwd(U, w, eps)
    close(Yh, Ye, name="rms2")
    dw_h, dw_e = torch.zeros(C, device="cuda"), torch.zeros(C, dtype=torch.float64)
    dU = r(C, G, gen=gen)
    close(hb.rms2_bwd(cuda(dU), cuda(U), cuda(w), sh_, eps, dw_h), emu.rms2_bwd(dU, U, w, se_, eps, dw_e),
          rtol=1e-3, name="rms2_bwd")
    close(dw_h, dw_e, rtol=1e-3, name="rms_dw")
    mom = torch.stack([r(20, N, gen=gen), r(20, N, gen=gen).abs() + 0.1, r(20, N, gen=gen) * 0.1, r(20, N, gen=gen).abs()])
    gst = r(80, N, gen=gen)
    close(hb.moment_coef(cuda(mom), cuda(gst), NC), emu.moment_coef(mom, gst, NC), rtol=1e-3, name="coef")
    mu1, var1 = r(C, gen=gen), r(C, gen=gen).abs() + 0.1
    a = hb.bn2_finalize(cuda(mu1), cuda(var1), cuda(gamma), cuda(beta), None, None, 1000, 0.1, 1e-5)
    b = emu.bn2_finalize(mu1, var1, gamma, beta, None, None, 1000, 0.1, 1e-5)
    for x, yv in zip(a, b):
        close(x, yv, name="bn2")
    Sg, Sgx = r(C, gen=gen), r(C, gen=gen)
    dgh, dbh = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dge, dbe = torch.zeros(C, dtype=torch.float64), torch.zeros(C, dtype=torch.float64)
    a = hb.bn2_bwd_coef(cuda(Sg), cuda(Sgx), cuda(mu1), cuda(var1), cuda(gamma), 1000, 1e-5, dgh, dbh)
    b = emu.bn2_bwd_coef(Sg, Sgx, mu1, var1, gamma, 1000, 1e-5, dge, dbe)
    for x, yv in zip(list(a) + [dgh, dbh], list(b) + [dge, dbe]):
        close(x, yv, name="bn2bwd")


@pytest.mark.parametrize("G,NF,NC", [(1, 37, 12), (2, 50, 16), (1, 9, 128)])
def test_loss_ops(hb, G, NF, NC):
    F = 10
    gen = torch.Generator().manual_seed(11)
    emu = EmuBackend()
    d, de = dims(G, NF, NC, F)
    y = r(F, d.E, gen=gen)
    sc, sh = r(F, gen=gen) * 0.3 + 1, r(F, gen=gen)
    Wd1, bd1, Wd2, bd2 = r(F, F, scale=0.3, gen=gen), r(F, gen=gen), r(1, F, scale=0.5, gen=gen), r(1, gen=gen) + 1.0
    Ti = torch.randint(2, 13, (d.NT,), generator=gen).double()
    Ni = torch.randint(100, 2000, (d.NT,), generator=gen).double()
    ci = torch.stack([Ti, Ni])
    for sharp in [0.0, 12.0]:
        args = (Wd1, bd1, Wd2, bd2, ci, 42.0 / NC, sharp, 0.3, 99)
        oh = hb.loss_fwd(d, cuda(y), cuda(sc), cuda(sh), *[cuda(a) if isinstance(a, torch.Tensor) else a for a in args], want_time=True)
        oe = emu.loss_fwd(de, y, sc, sh, *args, want_time=True)
        for a, b, nm in zip(oh, oe, ["n_prime", "fiber_time", "tmean", "tvar", "tt"]):
            close(a, b, rtol=1e-3, atol=1e-4, name=nm)
        fh = hb.loss_finalize(d, oh[0], oh[1], oh[3], cuda(ci), 0.1, 0.1, 42.0, 10.0, 2000.0, 1.0)
        fe = emu.loss_finalize(de, oe[0], oe[1], oe[3], ci, 0.1, 0.1, 42.0, 10.0, 2000.0, 1.0)
        for a, b, nm in zip(fh, fe, ["loss", "utils", "variance", "Gn", "Gf", "Gv"]):
            close(a, b, rtol=1e-3, atol=1e-4, name=nm)
        gh = [torch.zeros(F, F, device="cuda"), torch.zeros(F, device="cuda"), torch.zeros(1, F, device="cuda"), torch.zeros(1, device="cuda")]
        ge = [torch.zeros(F, F, dtype=torch.float64), torch.zeros(F, dtype=torch.float64), torch.zeros(1, F, dtype=torch.float64), torch.zeros(1, dtype=torch.float64)]
        gxh = hb.loss_bwd(d, cuda(y), cuda(sc), cuda(sh), *[cuda(a) if isinstance(a, torch.Tensor) else a for a in args],
                          fh[3], fh[4], fh[5], oh[2], 1.0, *gh)
        gxe = emu.loss_bwd(de, y, sc, sh, *args, fe[3], fe[4], fe[5], oe[2], 1.0, *ge)
        close(gxh, gxe, rtol=2e-3, atol=1e-4, name="loss gxe")
        for a, b, nm in zip(gh, ge, ["dWd1", "dbd1", "dWd2", "dbd2"]):
            close(a, b, rtol=2e-3, atol=1e-4, name=nm)
        # the BatchNorm-sums arm (pfsgnn_loss_bwd_bn): the same gradient, bitwise,
        # plus per-block partials of sum g and sum g (y - mu1) inv1
        mu1, var1 = r(F, gen=gen), r(F, gen=gen).abs() + 0.5
        inv1 = 1.0 / torch.sqrt(var1 + 1e-5)
        gh2 = [torch.zeros_like(t) for t in gh]
        gxh2, part = hb.loss_bwd(d, cuda(y), cuda(sc), cuda(sh),
                                 *[cuda(a) if isinstance(a, torch.Tensor) else a for a in args],
                                 fh[3], fh[4], fh[5], oh[2], 1.0, *gh2, bn=(cuda(mu1), cuda(inv1)))
        assert torch.equal(gxh2, gxh)
        for a, b in zip(gh2, gh):
            assert torch.equal(a, b)
        # (about the HIP gradient itself, so only the sums' rounding is compared)
        Sg, Sgx = emu.edge_bn_grad_sums(de, cpu(gxh), cpu(cuda(y)), mu1, inv1)
        S = part.double().sum(0).cpu()
        mag = cpu(gxh).abs().sum(1).max().item()   # fp32 summation error scale
        close(S[:F], Sg, rtol=0, atol=1e-5 * mag, name="loss bn Sg")
        close(S[F:], Sgx, rtol=0, atol=1e-5 * mag * (inv1.max().item() * 6), name="loss bn Sgx")
        gamma = r(F, gen=gen)
        dgh, dbh = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")
        dgh2, dbh2 = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")
        a1 = hb.bn2_bwd_coef_part(part, cuda(mu1), cuda(var1), cuda(gamma), d.E, 1e-5, dgh, dbh)
        a2 = hb.bn2_bwd_coef(part[:, :F].sum(0), part[:, F:].sum(0), cuda(mu1), cuda(var1),
                             cuda(gamma), d.E, 1e-5, dgh2, dbh2)
        for x, yv in zip(list(a1) + [dgh, dbh], list(a2) + [dgh2, dbh2]):
            close(x, yv, rtol=1e-4, atol=1e-6, name="bn2 coef part")


def test_noise_bit_exact(hb):
    """The in-kernel softfloor uniforms equal tests/noise_ref.py bit for bit."""
    from noise_ref import uniform_numpy
    F, G, NF, NC = 8, 1, 16, 16
    d, _ = dims(G, NF, NC, F)
    y = torch.zeros(F, d.E, device="cuda")
    # decoder = 0 -> pred = bd2 = 0 -> time = log(2)*scale ; choose scale so time/T = 0
    z = torch.zeros
    Wd1, bd1, Wd2, bd2 = z(F, F, device="cuda"), z(F, device="cuda"), z(1, F, device="cuda"), torch.full((1,), -1e4, device="cuda")
    ci = torch.stack([torch.ones(NC), torch.full((NC,), 1e9)]).cuda()
    out = hb.loss_fwd(d, y, None, None, Wd1, bd1, Wd2, bd2, ci, 1.0, 0.0, 1.0, 4242, want_time=True)
    tt = out[4].cpu().double()
    u = torch.as_tensor(uniform_numpy(4242, d.E)).double()
    expect = torch.clamp(u - 0.5, min=0.0)      # time = softplus(-1e4) ~ 0; sharpness 0 -> identity
    assert torch.allclose(tt, expect, atol=1e-6)


def test_adam_matches_torch(hb):
    from pfsgnn.optim import FusedAdam
    torch.manual_seed(0)
    ps = [torch.randn(17, 5, device="cuda", requires_grad=True), torch.randn(33, device="cuda", requires_grad=True)]
    qs = [p.detach().clone().requires_grad_() for p in ps]
    o1 = FusedAdam(ps, lr=5e-4, weight_decay=0.01)
    o2 = torch.optim.Adam(qs, lr=5e-4, weight_decay=0.01)
    for it in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad = g.clone()
            q.grad = g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, rtol=1e-6, atol=1e-7), (p - q).abs().max()


@pytest.mark.parametrize("G,NF,NC", [(1, 37, 12), (3, 21, 5), (2, 7, 200)])
def test_layout_modes(hb, G, NF, NC):
    """layout_analyze classifies the caller's edge order and the three conversion
    modes (permutation / fiber-major arithmetic / identity) agree with the
    harness's explicit index maps, bit-exactly."""
    from harness import canonical_edges, from_canonical, to_canonical
    from pfsgnn.gnn import Layout
    F = 10
    E = G * NF * NC
    gen = torch.Generator().manual_seed(NF + NC)
    x = torch.randn(E, F, generator=gen)
    ei_fm = canonical_edges(G, NF, NC)
    xc_ref = to_canonical(x, G, NF, NC)
    # fiber-major (train.py's order)
    perm, complete, fm, ident = hb.layout_analyze(ei_fm.cuda(), G, NF, NC)
    assert complete and fm and not ident
    for lay in (Layout(G, NF, NC, Layout.FIBER_MAJOR), Layout(G, NF, NC, Layout.PERM, perm)):
        xc = hb.edges_to_canonical(x.cuda(), lay)
        assert torch.equal(xc.cpu(), xc_ref)
        back = hb.edges_from_canonical(xc, None, None, lay, rowmajor=True)
        assert torch.equal(back.cpu(), x)
    # arbitrary order
    p = torch.randperm(E, generator=gen)
    perm, complete, fm, ident = hb.layout_analyze(ei_fm[:, p].contiguous().cuda(), G, NF, NC)
    assert complete and not fm and not ident
    lay = Layout(G, NF, NC, Layout.PERM, perm)
    xc = hb.edges_to_canonical(x[p].contiguous().cuda(), lay)
    assert torch.equal(xc.cpu(), xc_ref)
    sc, sh = torch.rand(F, generator=gen) + 0.5, torch.randn(F, generator=gen)
    out = hb.edges_from_canonical(xc, sc.cuda(), sh.cuda(), lay, rowmajor=True).cpu()
    assert torch.allclose(out, (x * sc + sh)[p], rtol=1e-6, atol=1e-6)
    # canonical (class-major) order
    ei_cm = ei_fm.t().reshape(G, NF, NC, 2).permute(0, 2, 1, 3).reshape(E, 2).t().contiguous()
    perm, complete, fm, ident = hb.layout_analyze(ei_cm.cuda(), G, NF, NC)
    assert complete and ident
    assert torch.equal(perm.cpu(), torch.arange(E, dtype=torch.int32))
    # incomplete / duplicated / cross-graph
    bad = ei_fm.clone()
    bad[1, 0] = bad[1, 1]
    assert not hb.layout_analyze(bad.cuda(), G, NF, NC)[1]
    if G > 1:
        bad = ei_fm.clone()
        bad[1, 0] = NC * (G - 1)
        assert not hb.layout_analyze(bad.cuda(), G, NF, NC)[1]
    assert torch.equal(from_canonical(xc_ref, G, NF, NC), x)


# fused node MLP (+ BatchNorm1d): (K split into blocks, H, O, N, G, bn) -- the
# SModel / TModel / GlobalModel / encoder shapes at Fdim 8/10/16, N not a
# multiple of 64, per-graph u blocks, one wave-chunk and many
MLP_CASES = [
    ([10, 80, 10], 100, 10, 38 * 64 + 26, 16, True),     # SModel node_mlp_2, Fdim 10
    ([8, 64, 8], 80, 8, 1000, 4, True),                 # Fdim 8
    ([16, 32, 16], 64, 16, 777, 3, True),               # TModel node_mlp_2, Fdim 16
    ([12, 88, 12], 112, 16, 300, 4, True),              # the widest fused shape
    ([10, 20, 10], 40, 10, 2048, 16, True),             # TModel node_mlp_2
    ([10, 10, 10], 30, 10, 16, 16, False),              # GlobalModel MLP over G columns
    ([1], 10, 10, 5000, 1, False),                      # encoder_s
    ([2], 10, 10, 130, 1, False),                       # encoder_t
]


@pytest.mark.parametrize("blocks,H,O,N,G,bn", MLP_CASES)
def test_mlp_fused(hb, blocks, H, O, N, G, bn):
    """pfsgnn_mlp_fwd / pfsgnn_mlp_bwd (+ the BatchNorm1d) and the weight
    gradients taken from their saved tensors, vs the float64 emulation."""
    gen = torch.Generator().manual_seed(N + H + O)
    emu = EmuBackend()
    K = sum(blocks)
    last_pg = len(blocks) == 3 and G > 1 and N % G == 0 and N > G
    X = []
    col = 0
    for i, rows in enumerate(blocks):
        pg = last_pg and i == len(blocks) - 1
        X.append((r(rows, G if pg else N, gen=gen), col, pg))
        col += rows
    W1, b1 = r(H, K, scale=0.2, gen=gen), r(H, scale=0.3, gen=gen)
    W2, b2 = r(O, H, scale=0.2, gen=gen), r(O, gen=gen)
    g, bt = r(O, gen=gen) * 0.2 + 1, r(O, gen=gen) * 0.1
    rm, rv = r(O, gen=gen) * 0.1, r(O, gen=gen).abs() + 0.5
    dY = r(O, N, gen=gen)
    res = {}
    for be, conv in ((emu, lambda t: t.clone()), (hb, cuda)):
        segs = [(conv(t), c, pg) for t, c, pg in X]
        w = [conv(t) for t in (W1, b1, W2, b2)]
        bnp = (conv(g), conv(bt), conv(rm), conv(rv), 0.1, 1e-5) if bn else None
        Y, Z, Yp, mu, var = be.mlp_fwd(segs, N, *w, bn=bnp)
        dg, db = conv(torch.zeros(O)), conv(torch.zeros(O))
        bnb = (Yp, mu, var, bnp[0], 1e-5, dg, db) if bn else None
        outs, bufs = [], []
        for t, c, pg in X:
            buf = conv(torch.full((t.shape[0], N), 0.5))
            bufs.append(buf)
            outs.append((buf, t.shape[0], c == 0))      # first block accumulates
        dYp, dZ = be.mlp_bwd(conv(dY), Z, w[0], w[2], K, bn=bnb, outs=outs)
        dW1, db1 = conv(torch.zeros(H, K)), conv(torch.zeros(H))
        dW2, db2 = conv(torch.zeros(O, H)), conv(torch.zeros(O))
        be.wgrad(dYp, Z, dW2, db=db2, act_in=True)
        be.wgrad_cat(dZ, segs, dW1, db=db1)
        res[be.name] = dict(Y=Y, Z=Z, dYp=dYp, dZ=dZ, dW1=dW1, db1=db1, dW2=dW2, db2=db2,
                            **{f"dX{i}": b for i, b in enumerate(bufs)},
                            **({"mu": mu, "var": var, "rm": bnp[2], "rv": bnp[3], "dg": dg,
                                "db": db} if bn else {}))
    for k, v in res["emu"].items():
        atol = 1e-6
        if k in ("db2", "db"):
            # sums of the BatchNorm-backward gradient cancel to ~0 analytically:
            # judged against the fp32 rounding of the sum of |terms|
            atol += 1e-6 * res["emu"]["dYp"].abs().sum(1).max().item()
        close(res["hip"][k], v, rtol=5e-5, atol=atol, name=k)


def test_linear_batch_matches_single_launches():
    """pfsgnn_gemm_multi (node parts / input gradients batched) against the
    single-launch pfsgnn_lin_cat / pfsgnn_lin_t: bitwise equal."""
    from pfsgnn.gnn import backend
    hb = backend()
    g = torch.Generator().manual_seed(5)
    r = lambda *s: torch.randn(*s, generator=g).cuda()  # noqa: E731
    F, G, NS, NT = 10, 3, 3 * 301, 3 * 37
    W1, b1, Ws1, bs1 = r(4 * F, 4 * F), r(4 * F), r(2 * F, 2 * F), r(2 * F)
    xs, xt, u = r(F, NS), r(F, NT), r(F, G)
    outs = hb.linear_batch([("cat", W1, [(xs, 0, False)], NS, None),
                            ("cat", W1, [(xt, F, False), (u, 3 * F, True)], NT, b1),
                            ("cat", Ws1, [(xt, 0, False)], NT, bs1)])
    ref = [hb.lin(W1, 0, F, xs), hb.lin_cat(W1, [(xt, F, False), (u, 3 * F, True)], NT, b=b1),
           hb.lin(Ws1, 0, F, xt, b=bs1)]
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)
    gs, gt = r(4 * F, NS), r(4 * F, NT)
    ys, yt = r(F, NS), r(F, NT)
    ys2, yt2 = ys.clone(), yt.clone()
    hb.linear_batch([("t", W1, 0, F, gs, ys, True), ("t", W1, F, F, gt, yt, True)])
    hb.lin_t(W1, 0, F, gs, out=ys2, add=True)
    hb.lin_t(W1, F, F, gt, out=yt2, add=True)
    assert torch.equal(ys, ys2) and torch.equal(yt, yt2)


@pytest.mark.parametrize("G,n1,n2,F,normed", [(1, 37, 12, 10, True), (16, 2394, 128, 10, True),
                                                (3, 300, 7, 16, True), (5, 21, 5, 8, False)])
def test_global_fused(hb, G, n1, n2, F, normed):
    """pfsgnn_global_fwd / _bwd (the whole GlobalModel, gnn.py:208-223, one
    launch each) vs the composed emulation (graph means, MLP, RMSNorm x2)."""
    emu = EmuBackend()
    gen = torch.Generator().manual_seed(G * 7 + F)
    xs, xt, u = r(F, G * n1, gen=gen), r(F, G * n2, gen=gen), r(F, G, gen=gen)
    W1, b1 = r(3 * F, 3 * F, scale=0.3, gen=gen), r(3 * F, gen=gen)
    W2, b2 = r(F, 3 * F, scale=0.3, gen=gen), r(F, gen=gen)
    w = r(F, gen=gen).abs() + 0.5 if normed else None
    eps = float(torch.finfo(torch.float32).eps)
    oh = hb.global_fwd(cuda(xs), cuda(xt), cuda(u), cuda(W1), cuda(b1), cuda(W2), cuda(b2),
                       cuda(w), eps, G)
    oe = emu.global_fwd(xs, xt, u, W1, b1, W2, b2, w, eps, G)
    for a, b, nm in zip(oh[:4], oe[:4], ("Y", "means", "Z", "V")):
        close(a, b, name=nm)
    dY = r(F, G, gen=gen)
    gu_e, gxs_e, gxt_e = r(F, G, gen=gen), r(F, G * n1, gen=gen), r(F, G * n2, gen=gen)
    gu_h, gxs_h, gxt_h = cuda(gu_e), cuda(gxs_e), cuda(gxt_e)
    dw_h = torch.zeros(F, device="cuda") if normed else None
    dw_e = torch.zeros(F, dtype=torch.float64) if normed else None
    gh = hb.global_bwd(cuda(dY), oh[3], cuda(w), oh[4], eps, dw_h, oh[2], cuda(W1), cuda(W2),
                       gu_h, gxs_h, 1.0 / n1, gxt_h, 1.0 / n2)
    ge = emu.global_bwd(dY, oe[3], w, oe[4], eps, dw_e, oe[2], W1, W2, gu_e, gxs_e, 1.0 / n1,
                        gxt_e, 1.0 / n2)
    torch.cuda.synchronize()
    close(gh[0], ge[0], rtol=1e-3, name="gV"); close(gh[1], ge[1], rtol=1e-3, name="dZ")
    close(gu_h, gu_e, rtol=1e-3, name="g_u")
    close(gxs_h, gxs_e, rtol=1e-3, name="g_xs"); close(gxt_h, gxt_e, rtol=1e-3, name="g_xt")
    if normed:
        close(dw_h, dw_e, rtol=1e-3, name="dw")


@pytest.mark.parametrize("G,NF,NC,F", EDGE_CASES)
def test_edge_ops_node_epilogues(hb, G, NF, NC, F):
    """The node-side Linear epilogues of the edge ops' reductions (TModel's
    second Linear after the class sum; the first Linears' node-input gradients
    g_xs / g_xt / Vu) against the emulation's separate products, at every Fdim
    (reduction widths 16, 20, 32, 40, 64) and with KS = 1 and KS > 1 grids."""
    gen = torch.Generator().manual_seed(7 + G * 1000 + NF * 10 + NC + F)

    def q(t, step):
        return torch.round(t / step) * step
    emu = EmuBackend()
    d, de = dims(G, NF, NC, F)
    E, NS, NT = d.E, d.NS, d.NT
    y = q(r(F, E, scale=2, gen=gen), 1 / 4)
    sc, sh = q(r(F, gen=gen) * 0.3 + 1, 1 / 8), q(r(F, gen=gen), 1 / 8)
    # target_fwd + agg
    Rs, Wt1 = q(r(2 * F, NS, gen=gen), 1 / 256), q(r(2 * F, 2 * F, scale=0.3, gen=gen), 1 / 64)
    Wt2, bt2 = r(2 * F, 2 * F, scale=0.3, gen=gen), r(2 * F, gen=gen)
    hs_h, agg_h = hb.target_fwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Rs), cuda(Wt1),
                                agg=(cuda(Wt2), cuda(bt2), float(NF)))
    hs_e, agg_e = emu.target_fwd(de, y, sc, sh, Rs, Wt1, agg=(Wt2, bt2, float(NF)))
    close(hs_h, hs_e, name="hsum"); close(agg_h, agg_e, name="agg")
    # target_bwd + g_xs
    g_hsum = r(2 * F, NT, gen=gen)
    dW_h, dW_e = torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, 2 * F, dtype=torch.float64)
    gxs_e = r(F, NS, gen=gen)
    gxs_h = cuda(gxs_e)
    GzT_h, _ = hb.target_bwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Rs), cuda(Wt1), cuda(g_hsum), dW_h,
                             g_xs=gxs_h)
    GzT_e, _ = emu.target_bwd(de, y, sc, sh, Rs, Wt1, g_hsum, dW_e, g_xs=gxs_e)
    close(GzT_h, GzT_e, name="GzT"); close(gxs_h, gxs_e, rtol=5e-4, name="g_xs(T)")
    # source_bwd + g_xt
    Qt = q(r(2 * F, NT, gen=gen), 1 / 256)
    Ws1, Ws2, bs2 = q(r(2 * F, 2 * F, scale=0.3, gen=gen), 1 / 64), r(2 * F, 2 * F, scale=0.3, gen=gen), r(2 * F, gen=gen)
    mean = r(2 * F, NS, gen=gen)
    coef = r(4, 2 * F, NS, gen=gen) * torch.tensor([1, 0.3, 0.1, 0.03], dtype=torch.float64)[:, None, None]
    gr_h = [torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, device="cuda")]
    gr_e = [torch.zeros(2 * F, 2 * F, dtype=torch.float64), torch.zeros(2 * F, 2 * F, dtype=torch.float64), torch.zeros(2 * F, dtype=torch.float64)]
    gxt_e = r(F, NT, gen=gen)
    gxt_h = cuda(gxt_e)
    oh = hb.source_bwd(d, cuda(y), cuda(sc), cuda(sh), cuda(Qt), cuda(Ws1), cuda(Ws2), cuda(bs2), cuda(mean),
                       cuda(coef), None, None, None, *gr_h, g_xt=gxt_h)
    oe = emu.source_bwd(de, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, None, None, None, *gr_e, g_xt=gxt_e)
    close(oh[1], oe[1], rtol=5e-4, name="GzS"); close(gxt_h, gxt_e, rtol=5e-4, name="g_xt(S)")
    # edge_mlp_bwd + nodes
    xe = q(r(F, E, scale=2, off=3, gen=gen), 1 / 16)
    Ps, Pt = q(r(4 * F, NS, gen=gen), 1 / 256), q(r(4 * F, NT, gen=gen), 1 / 256)
    W1, W2 = q(r(4 * F, 4 * F, scale=0.3, gen=gen), 1 / 64), r(F, 4 * F, scale=0.3, gen=gen)
    g_tot = r(F, E, gen=gen)
    alpha, gam0, gam1 = r(F, gen=gen), r(F, gen=gen) * 0.1, r(F, gen=gen) * 0.1
    gh = [torch.zeros(4 * F, 4 * F, device="cuda"), torch.zeros(F, 4 * F, device="cuda"), torch.zeros(F, device="cuda")]
    ge = [torch.zeros(4 * F, 4 * F, dtype=torch.float64), torch.zeros(F, 4 * F, dtype=torch.float64), torch.zeros(F, dtype=torch.float64)]
    nxs_e, nxt_e = r(F, NS, gen=gen), r(F, NT, gen=gen)
    nxs_h, nxt_h = cuda(nxs_e), cuda(nxt_e)
    oh = hb.edge_mlp_bwd(d, cuda(g_tot), cuda(alpha), cuda(gam0), cuda(gam1), cuda(y), cuda(xe), None, None,
                         cuda(Ps), cuda(Pt), cuda(W1), cuda(W2), *gh, want_gxe=False, nodes=(nxs_h, nxt_h))
    oe = emu.edge_mlp_bwd(de, g_tot, alpha, gam0, gam1, y, xe, None, None, Ps, Pt, W1, W2, *ge, want_gxe=False,
                          nodes=(nxs_e, nxt_e))
    torch.cuda.synchronize()
    for a, b, nm in zip(oh[1:], oe[1:], ["GzEs", "GzEt", "Vu"]):
        close(a, b, rtol=5e-4, name=nm)
    close(nxs_h, nxs_e, rtol=5e-4, name="g_xs(E)"); close(nxt_h, nxt_e, rtol=5e-4, name="g_xt(E)")


def test_node_x3_policy(hb):
    """The node level's gradient chains and weight gradients follow the edge
    path (pf::node_x3): bf16x3 on the default `mfma` path, fp32 on the exact
    `mfma32` path.  SModel node_mlp_2's shape (100-wide, the RS backward and
    the <8, 8> weight gradient): mfma32 within 1e-5 of the float64 emulation,
    mfma within the 5e-5 bar and visibly coarser (the split path is live)."""
    import pfsgnn
    blocks, H, O, N, G = [10, 80, 10], 100, 10, 38 * 64 + 26, 16
    gen = torch.Generator().manual_seed(4242)
    K = sum(blocks)
    X, col = [], 0
    for rows in blocks:
        X.append((r(rows, N, gen=gen), col, False))
        col += rows
    W1, b1 = r(H, K, scale=0.2, gen=gen), r(H, scale=0.3, gen=gen)
    W2, b2 = r(O, H, scale=0.2, gen=gen), r(O, gen=gen)
    dY = r(O, N, gen=gen)
    emu = EmuBackend()

    def run(be, conv):
        segs = [(conv(t), c, pg) for t, c, pg in X]
        w = [conv(t) for t in (W1, b1, W2, b2)]
        Y, Z, Yp, mu, var = be.mlp_fwd(segs, N, *w, bn=None)
        outs = [(conv(torch.zeros(t.shape[0], N)), t.shape[0], False) for t, _, _ in X]
        dYp, dZ = be.mlp_bwd(conv(dY), Z, w[0], w[2], K, bn=None, outs=outs)
        dW1 = conv(torch.zeros(H, K))
        be.wgrad_cat(dZ, segs, dW1)
        return {"dZ": dZ, "dX1": outs[1][0], "dW1": dW1}

    ref = run(emu, lambda t: t.clone())
    prev = pfsgnn.get_edge_path()
    err = {}
    try:
        for path in ("mfma32", "mfma"):
            pfsgnn.set_edge_path(path)
            got = run(hb, cuda)
            err[path] = {k: ((cpu(got[k]) - v).abs().max() / v.abs().max()).item() for k, v in ref.items()}
    finally:
        pfsgnn.set_edge_path(prev)
    for k in ref:
        assert err["mfma32"][k] <= 1e-5, (k, err)
        assert err["mfma"][k] <= 5e-5, (k, err)
    assert err["mfma"]["dW1"] > 4 * err["mfma32"]["dW1"], err   # the bf16x3 weight gradient ran
    assert err["mfma"]["dX1"] > 4 * err["mfma32"]["dX1"], err   # the bf16x3 input-gradient chain ran
