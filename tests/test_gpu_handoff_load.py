"""edge_mlp_fwd's in-launch BatchNorm statistics (mom_finalize's hand-off,
pfsgnn_common.h last_arrival) under UNEVEN load.

The last-arriving block of each group of 64 Welford partials reads the other
blocks' partials inside the same launch.  MI355X_MICROARCH.md: a hand-off must
be tested under uneven load with the consumer's L1 warm -- an idle chip and
uniform load hide stale reads.  Here a second stream keeps a varying part of the
chip busy with GEMMs while the bench-geometry edge_mlp_fwd (3040 blocks,
several per CU) runs on the default stream, 24 times; every run's mu / var /
sc / sh / inv1 / running statistics must equal the idle run's bit for bit, and
the idle run must agree with the separate-launch form (no sync buffer:
k_moments_finalize) to float rounding of the double merge."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs():
    from pfsgnn.engine import Dims
    G, NF, NC, F = 16, 2394, 128, 10
    d = Dims(G, NF, NC, F)
    g = torch.Generator(device="cuda").manual_seed(3)
    c = lambda *s, sc=1.0, off=0.0: (torch.randn(*s, device="cuda", generator=g) * sc + off)  # noqa: E731
    t = dict(xe=c(F, d.E, sc=2, off=3), xsc=c(F, sc=0.5, off=1), xsh=c(F), Ps=c(4 * F, d.NS),
             Pt=c(4 * F, d.NT), W1=c(4 * F, 4 * F, sc=0.3), W2=c(F, 4 * F, sc=0.3), b2=c(F),
             gamma=c(F, sc=0.2, off=1), beta=c(F, sc=0.3), rm=c(F, sc=0.1), rv=c(F, sc=0.1, off=1).abs())
    return d, t


def _run(hb, d, t):
    rm, rv = t["rm"].clone(), t["rv"].clone()
    y, mu, var, sc, sh, inv1 = hb.edge_mlp_fwd_bn(
        d, t["xe"], t["xsc"], t["xsh"], t["Ps"], t["Pt"], t["W1"], t["W2"], t["b2"],
        (t["gamma"], t["beta"], rm, rv, 0.1, 1e-5))
    return dict(mu=mu, var=var, sc=sc, sh=sh, inv1=inv1, rm=rm, rv=rv)


def test_edge_stats_handoff_under_uneven_load():
    import pfsgnn  # noqa: F401
    from pfsgnn import native
    from pfsgnn.native import HipBackend
    hb = HipBackend()
    if native._SYNC is None:
        pytest.skip("PFSGNN_NO_HANDOFF=1: no in-launch hand-off to test")
    d, t = _inputs()
    ref = _run(hb, d, t)
    torch.cuda.synchronize()
    # the separate-launch form: no sync buffer -> k_moments_finalize
    native._call("pfsgnn_set_sync_buffer", None, 0)
    try:
        sep = _run(hb, d, t)
        torch.cuda.synchronize()
    finally:
        native._call("pfsgnn_set_sync_buffer", native._SYNC.data_ptr(), native._SYNC.numel())
    for k in ("mu", "var", "sc", "sh", "rm", "rv"):
        torch.testing.assert_close(ref[k], sep[k], rtol=2e-6, atol=1e-7, msg=lambda m: f"{k}: {m}")

    side = torch.cuda.Stream()
    mats = {n: torch.randn(n, n, device="cuda") for n in (1024, 2048, 4096)}
    sizes = [1024, 4096, 2048, 4096, 1024, 2048]
    for rep in range(24):
        n = sizes[rep % len(sizes)]
        a = mats[n]
        with torch.cuda.stream(side):   # the load: a varying number of busy CUs
            for _ in range(1 + rep % 3):
                a = torch.tanh(a @ mats[n] * (1.0 / n))
        got = _run(hb, d, t)            # default stream, concurrent with the load
        torch.cuda.synchronize()
        for k, v in ref.items():
            assert torch.equal(v, got[k]), \
                f"rep {rep} (load {n}): {k} differs from the idle run " \
                f"({int((v != got[k]).sum())} of {v.numel()} elements)"
