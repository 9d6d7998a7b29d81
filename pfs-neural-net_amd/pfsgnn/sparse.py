"""General (non-complete) bipartite graphs: the edge ops of ``pfsgnn.engine``
composed from gathers, node-level Linear kernels and segment reductions.

The reference runs on any ``edge_index`` (gnn.py:7-47): its per-edge MLPs read
``x_s[src]`` / ``x_t[tgt]`` (gnn.py:100, 136, 188) and its scatters reduce over
arbitrary fibers (gnn.py:140-144, ``reduce='mean'``) and classes (gnn.py:190,
``reduce='sum'``).  The fused edge kernels (pfsgnn_edge.hip / pfsgnn_mfma.hip)
assume G complete graphs; a batch that is not complete is laid out once by
``pfsgnn_sparse_layout`` (CSR by fiber and by class, include/pfsgnn.h) and
every engine edge op then runs here, with the same arguments and results as
the fused op it replaces:

* edge tensors are channel-major [C, E] in *position* order -- the caller's
  edges sorted stably by fiber, so each fiber's messages are one contiguous
  run (``fib_ptr``) and the per-fiber moments need no index;
* the first Linear of every per-edge MLP is split as in the fused path: the
  edge-feature part is one ``pfsgnn_lin_gather`` over E columns whose
  epilogue adds the node parts (Ps, Pt, Qt, Rs) gathered per edge;
* per-fiber and per-class sums are ``pfsgnn_segment_sum`` (one wave per
  segment, every channel in registers, fixed DPP tree: bitwise reproducible);
* TModel's ``scatter(MLP(msg), tgt, 'sum')`` keeps the second Linear after the
  sum, with its bias scaled by each class's degree (engine.target_fwd).

Intermediates the fused kernels recompute in registers (z1, zs, zt) are
recomputed here too, as [C, E] tables, so forward and backward keep the
fused path's saved state (y, sc, sh) and nothing else per edge.
"""
import weakref

import torch


class SparseGeo:
    """Layout of a general batch (outputs of pfsgnn_sparse_layout).

    src_p / tgt_p [E]: fiber / class of each position; user_of [E]: the
    caller's edge at each position; fib_ptr [NS+1]: CSR by fiber over
    positions; cls_ord [E] / cls_ptr [NT+1]: positions sorted stably by class
    and its CSR; deg_t [1, NT]: float class degrees (TModel's bias sum)."""

    def __init__(self, E, src_p, tgt_p, user_of, fib_ptr, cls_ord, cls_ptr, deg_t):
        self.E = int(E)
        self.src_p, self.tgt_p, self.user_of = src_p, tgt_p, user_of
        self.fib_ptr, self.cls_ord, self.cls_ptr = fib_ptr, cls_ord, cls_ptr
        self.deg_t = deg_t
        self.sl = None   # native.SlicedLayout when the fused sliced kernels run the batch

    @property
    def EP(self):
        """Edge-tensor columns: E positions, or the sliced layout's (padding included)."""
        return self.E if self.sl is None else self.sl.EP


class SparseEdgeOps:
    """The engine's edge op set (engine.Engine: edge_fwd / source_fwd /
    target_fwd and their backwards) for a general batch, on backend ``be``'s
    primitives.  Signatures mirror the backend's fused edge ops."""

    def __init__(self, be):
        self.be = be
        self._xcache = {}

    # ------------------------------------------------------------ helpers
    def _x(self, xe, sc, sh):
        """The lazy edge state materialised: xe_new = sc*y + sh per channel.
        Each state is read by up to five ops of a step (S/T forward, their
        backward, the next EdgeModel backward): it is materialised once and
        kept while its (y, sc, sh) tensors live (weak references)."""
        if sc is None:
            return xe
        key = (id(xe), id(sc), id(sh))
        hit = self._xcache.get(key)
        if hit is not None:
            ry, rs, rh, x, ver = hit
            if ry() is xe and rs() is sc and rh() is sh and ver == (xe._version, sc._version,
                                                                    sh._version):
                return x
        # drop the states that died (their x would otherwise stay allocated)
        self._xcache = {k: v for k, v in self._xcache.items()
                        if v[0]() is not None and v[1]() is not None and v[2]() is not None}
        x = self.be.affine_rows(xe, sc, sh)
        self._xcache[key] = (weakref.ref(xe), weakref.ref(sc), weakref.ref(sh), x,
                             (xe._version, sc._version, sh._version))
        return x

    def _z1(self, d, x, Ps, Pt, W1):
        """EdgeModel first Linear (gnn.py:100): Ps[:, src] + Pt[:, tgt] + W1[:, 2F:3F] x."""
        be, F, sp = self.be, d.F, d.sp
        return be.lin_gather(W1, 2 * F, F, x, [(Ps, sp.src_p), (Pt, sp.tgt_p)])

    def _zs(self, d, x, Qt, Ws1):
        """SModel node_mlp_1 first Linear (gnn.py:136): Qt[:, tgt] + Ws1[:, F:2F] x."""
        return self.be.lin_gather(Ws1, d.F, d.F, x, [(Qt, d.sp.tgt_p)])

    def _zt(self, d, x, Rs, Wt1):
        """TModel node_mlp_1 first Linear (gnn.py:188): Rs[:, src] + Wt1[:, F:2F] x."""
        return self.be.lin_gather(Wt1, d.F, d.F, x, [(Rs, d.sp.src_p)])

    # ------------------------------------------------------------ forward
    def edge_mlp_fwd(self, d, xe, xsc, xsh, Ps, Pt, W1, W2, b2):
        x = self._x(xe, xsc, xsh)
        z1 = self._z1(d, x, Ps, Pt, W1)
        y = self.be.lin(W2, 0, W2.shape[1], z1, b=b2, act_in=True)
        mu, var = self.be.rows_stats(y)
        return y, mu, var

    def source_fwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_out):
        x = self._x(y, sc, sh)
        zs = self._zs(d, x, Qt, Ws1)
        m = self.be.lin(Ws2, 0, Ws2.shape[1], zs, b=bs2, act_in=True)
        return self.be.segment_moments(m, d.sp.fib_ptr, d.NS, hs_out)

    def target_fwd(self, d, y, sc, sh, Rs, Wt1):
        x = self._x(y, sc, sh)
        zt = self._zt(d, x, Rs, Wt1)
        return self.be.segment_sum(zt, d.sp.cls_ord, d.sp.cls_ptr, d.NT, act=True)

    # ------------------------------------------------------------ backward
    def target_bwd(self, d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=False):
        be, F = self.be, d.F
        x = self._x(y, sc, sh)
        zt = self._zt(d, x, Rs, Wt1)
        gz = be.gather_cols(g_hsum, d.sp.tgt_p, mode=2, Z=zt)
        GzT = be.segment_sum(gz, None, d.sp.fib_ptr, d.NS)
        be.wgrad(gz, x, dWt1, col0=F)
        gxe = be.lin_t(Wt1, F, F, gz) if want_gxe else None
        return GzT, gxe

    def source_bwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next, bnstat,
                   dWs1, dWs2, dbs2):
        be, F, sp = self.be, d.F, d.sp
        x = self._x(y, sc, sh)
        zs = self._zs(d, x, Qt, Ws1)
        m = be.lin(Ws2, 0, Ws2.shape[1], zs, b=bs2, act_in=True)
        gm = be.segment_moment_grad(m, sp.src_p, mean, coef)
        be.wgrad(gm, zs, dWs2, db=dbs2, act_in=True)
        gz = be.lin_t(Ws2, 0, Ws2.shape[1], gm, z=zs)
        be.wgrad(gz, x, dWs1, col0=F)
        g = be.lin_t(Ws1, F, F, gz)
        GzS = be.segment_sum(gz, sp.cls_ord, sp.cls_ptr, d.NT)
        if tpart is not None:
            # TModel's per-edge input gradient (its node_mlp_1 reads the same x_e)
            Rs, Wt1, g_hsum = tpart
            zt = self._zt(d, x, Rs, Wt1)
            gzt = be.gather_cols(g_hsum, sp.tgt_p, mode=2, Z=zt)
            be.lin_t(Wt1, F, F, gzt, out=g, add=True)
        if g_next is not None:
            one = be.ones(F)
            be.rows_axpby(g_next, g, one, one, be.zeros(F), out=g)
        Sg = Sgx = None
        if bnstat is not None:
            Sg, Sgx = be.rows_bn_sums(g, y, *bnstat)
        return g, GzS, Sg, Sgx

    def edge_bn_grad_sums(self, d, g, y, mu1, inv1):
        return self.be.rows_bn_sums(g, y, mu1, inv1)

    def edge_mlp_bwd(self, d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2,
                     dW1, dW2, db2, want_gxe=True):
        be, F, sp = self.be, d.F, d.sp
        gy = be.rows_axpby(g_tot, y, alpha, gam1, gam0)
        x = self._x(xe, xsc, xsh)
        z1 = self._z1(d, x, Ps, Pt, W1)
        be.wgrad(gy, z1, dW2, db=db2, act_in=True)
        gz = be.lin_t(W2, 0, W2.shape[1], gy, z=z1)
        be.wgrad(gz, x, dW1, col0=2 * F)
        GzEs = be.segment_sum(gz, None, sp.fib_ptr, d.NS)
        GzEt = be.segment_sum(gz, sp.cls_ord, sp.cls_ptr, d.NT)
        gxe = be.lin_t(W1, 2 * F, F, gz) if want_gxe else None
        return gxe, GzEs, GzEt

    def edge_apply(self, d, y, sc, sh):
        return self.be.affine_rows(y, sc, sh) if sc is not None else y.clone()
