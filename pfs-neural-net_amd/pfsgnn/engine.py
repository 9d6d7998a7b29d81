"""Fused training-step engine for the bipartite fiber/class GNN.

This is the orchestration layer of the hot path.  It runs ``GNN.forward``
(gnn.py:280-305) and its backward -- which the reference gets from autograd
through ``torch.cat`` / ``torch_scatter`` / BatchNorm -- as a short, explicit
sequence of ops on a backend.  In the product the backend is
``native.HipBackend``: every op is a HIP kernel in ``libpfsgnn.so`` reached
through the C ABI in ``include/pfsgnn.h``.  (The test suite hands the same
engine a torch-CPU emulation of the op set to check every hand-derived
backward formula against the autograd oracle; the product never does.)

Layouts (DESIGN.md §Data layout): node tensors are channel-major ``[C, N]``;
edge tensors are channel-major ``[C, E]`` over the canonical class-major edge
order ``e = (g*NC + c)*NF + f`` of a batch of G complete bipartite graphs
(a general batch: its position order, edges sorted by fiber -- pfsgnn.sparse).
Edge state is kept *lazily*: an EdgeModel output is its pre-norm value ``y``
plus a per-channel affine ``(sc, sh)`` (xe_new = sc*y + sh) -- the triple
``xe3 = (y, sc, sh)``; consumers apply the affine on the fly, so inside the
stack the normalised edge tensor is never written to HBM.

Algebra used to cut per-edge work (all exact in real arithmetic):
* the first Linear of every per-edge MLP is split over its concatenated input
  (gnn.py:100/136/188): node parts are computed once per node (``Ps``, ``Pt``,
  ``Qt``, ``Rs``) and gathered; only the edge-feature part is per edge;
* TModel's ``scatter(MLP(msg), tgt, 'sum')`` (gnn.py:190) equals
  ``W2 @ scatter(lrelu(W1 msg + b1)) + NF*b2``: the second Linear runs after
  the per-class sum;
* the EdgeModel's BatchNorm runs twice (gnn.py:101 -- ``super().forward`` runs
  the Sequential's ``norm`` child, then ``self.norm`` again; the reference
  checkpoint's num_batches_tracked = 2 x epochs confirms it) and collapses to
  one affine forward and one per-channel coefficient triple backward;
* in backward, TModel's per-edge input gradient is recomputed inside the
  SModel edge pass, which also adds the downstream edge gradient and takes the
  edge BatchNorm's two gradient sums -- one pass instead of four.
"""
import os

import torch


class Dims:
    """Batch geometry: G graphs of NF fibers x NC classes, feature width F.
    ``sp``: None for complete bipartite graphs (E = G*NF*NC, the fused edge
    kernels), or the pfsgnn.sparse.SparseGeo of a general batch of E edges."""

    def __init__(self, G, NF, NC, F, sp=None):
        self.G, self.NF, self.NC, self.F = int(G), int(NF), int(NC), int(F)
        self.sp = sp
        self.E = self.G * self.NF * self.NC if sp is None else sp.E
        # columns of an edge tensor (a sliced general batch pads its fibers' runs)
        self.EP = self.E if sp is None else sp.EP
        self.NS = self.G * self.NF
        self.NT = self.G * self.NC

    def __repr__(self):
        kind = "" if self.sp is None else ", general"
        return f"Dims(G={self.G}, NF={self.NF}, NC={self.NC}, F={self.F}, E={self.E}{kind})"


def param_names(B, normed=True):
    """Parameter names in the reference's state_dict order (gnn.py:266-278)."""
    names = []

    def mlp(pre):
        names.extend([pre + ".0.weight", pre + ".0.bias", pre + ".2.weight", pre + ".2.bias"])

    mlp("encoder_s")
    mlp("encoder_t")
    for b in range(B):
        p = f"mpb.{b}."
        mlp(p + "edge_model")
        if normed:
            names.extend([p + "edge_model.norm.weight", p + "edge_model.norm.bias"])
        for m in ("s_model", "t_model"):
            mlp(p + m + ".node_mlp_1")
            mlp(p + m + ".node_mlp_2")
            if normed:
                names.extend([p + m + ".norm.weight", p + m + ".norm.bias"])
        mlp(p + "global_model")
        if normed:
            names.append(p + "global_model.norm.weight")
    mlp("decoder_e")
    mlp("decoder_s")
    return names


def _seg_n(segs):
    """Node count of a row-block list: the width of its first per-node block."""
    for X, _, bc in segs:
        if not bc:
            return X.shape[1]
    raise ValueError("a concatenated input needs at least one per-node block")


def _fused_mlp_ok(W1, W2, segs):
    """Shapes the fused node-MLP op takes (include/pfsgnn.h pfsgnn_mlp_fwd)."""
    K = sum(X.shape[0] for X, _, _ in segs)
    cols_in_order = all(col == sum(X.shape[0] for X, _, _ in segs[:i])
                        for i, (_, col, _) in enumerate(segs))
    return (W2.shape[0] <= 16 and W1.shape[0] <= 112 and K <= 112 and len(segs) <= 4
            and cols_in_order)


class Engine:
    def __init__(self, backend, F, B=0, Fs=1, Ft=1, T=1, normed=True, bn_eps=1e-5,
                 bn_momentum=0.1, rms_eps=None):
        self.be = backend
        self.F, self.B, self.Fs, self.Ft, self.T = F, B, Fs, Ft, T
        self.normed = normed
        self.bn_eps = bn_eps
        self.bn_momentum = bn_momentum
        self.rms_eps = rms_eps
        self.training = True
        # eval() with autograd: the forward saves what the backward needs
        # (BatchNorm on running statistics, gnn.py:101/154/192)
        self.want_grad = False

    # ================================================================= MLP
    def _bn_args(self, P, BN, bnkey):
        return (P[bnkey + "weight"], P[bnkey + "bias"], BN.get(bnkey + "running_mean"),
                BN.get(bnkey + "running_var"), self.bn_momentum, self.bn_eps)

    def _fused_tail_ok(self, P, d, pre_s, pre_t, pre_g):
        """The fused block tail (mlp_fwd_epi on SModel's node_mlp_2,
        target_global_fwd for TModel's node_mlp_2 + the GlobalModel): training
        with normalisation, on the HIP ops' shapes."""
        be, F = self.be, self.F
        if os.environ.get("PFSGNN_FUSED_TAIL", "1") == "0":   # A/B knob
            return False
        if not (self.training and self.normed and hasattr(be, "target_global_fwd") and F <= 16):
            return False
        def mlp_ok(pre):
            W1, W2 = P[pre + "0.weight"], P[pre + "2.weight"]
            return max(W1.shape) <= 112 and W2.shape[0] <= 16
        return (mlp_ok(pre_s + "node_mlp_2.") and mlp_ok(pre_t + "node_mlp_2.")
                and max(P[pre_g + "0.weight"].shape) <= 192)

    def mlp_fwd(self, P, pre, X, bnkey=None, BN=None, epi=None):
        """MLP (gnn.py:65): Linear -> LeakyReLU(0.1) -> Linear on [K, N], as ONE
        fused op, optionally followed by the module's BatchNorm1d (``bnkey``,
        gnn.py:154/192).  X is a tensor or, for the concatenated inputs of
        gnn.py:153/191/220, a list of row blocks ``(tensor, weight column,
        per_graph)`` read in place (a per_graph block is [rows, G], broadcast
        over each graph's nodes).  Returns (Y, saved); with ``epi`` (training
        BatchNorm only: [(W, col0, nk, b)]) -> (Y, saved, [W[:, col0:col0+O] Y + b])."""
        be = self.be
        W1, b1, W2, b2 = P[pre + "0.weight"], P[pre + "0.bias"], P[pre + "2.weight"], P[pre + "2.bias"]
        segs = X if isinstance(X, list) else [(X, 0, False)]
        N = _seg_n(segs)
        norm = bnkey is not None and self.normed
        if epi:
            assert norm and self.training and _fused_mlp_ok(W1, W2, segs)
            Y, Z, Yp, mu, var, outs = be.mlp_fwd_epi(segs, N, W1, b1, W2, b2,
                                                     self._bn_args(P, BN, bnkey), epi)
            return Y, (segs, Z, (Yp, mu, var, bnkey)), outs
        if not _fused_mlp_ok(W1, W2, segs):
            return self._mlp_fwd_ops(P, BN, pre, segs, N, bnkey if norm else None)
        if norm and self.training:
            Y, Z, Yp, mu, var = be.mlp_fwd(segs, N, W1, b1, W2, b2, bn=self._bn_args(P, BN, bnkey))
            return Y, (segs, Z, (Yp, mu, var, bnkey))
        Y, Z, _, _, _ = be.mlp_fwd(segs, N, W1, b1, W2, b2,
                                   save_z=self.training or self.want_grad)
        if norm:
            # eval: nn.BatchNorm1d on running statistics, applied once (gnn.py:154/192)
            rm, rv = BN[bnkey + "running_mean"], BN[bnkey + "running_var"]
            sc, sh = be.bn_eval_coef(P[bnkey + "weight"], P[bnkey + "bias"], rm, rv,
                                     self.bn_eps, 1)
            return be.affine_rows(Y, sc, sh), (segs, Z, ("eval", Y, bnkey, rm, rv))
        return Y, (segs, Z, None)

    def mlp_bwd(self, P, Gr, pre, dY, saved, outs=(), bn_part=None, mom_coef=None):
        """Backward of mlp_fwd: the input gradient goes to ``outs`` = [(tensor or
        None, rows, add)] over the K input rows (empty: none wanted); the weight
        gradients accumulate into Gr.  ``bn_part``: the BatchNorm's backward sums
        already made by dY's producer (_fiber_bn_sums)."""
        be = self.be
        if saved[0] == "ops":
            return self._mlp_bwd_ops(P, Gr, pre, dY, saved, outs)
        segs, Z, bns = saved
        W1, W2 = P[pre + "0.weight"], P[pre + "2.weight"]
        K = sum(X.shape[0] for X, _, _ in segs)
        bn = None
        if bns is not None and bns[0] == "eval":
            dY = self._bn_eval_bwd(P, Gr, bns[2], 1, dY, bns[1], bns[3], bns[4])
            bns = None
        if bns is not None:
            Yp, mu, var, key = bns
            bn = (Yp, mu, var, P[key + "weight"], self.bn_eps, Gr[key + "weight"], Gr[key + "bias"])
        kw = {"bn_part": bn_part} if bn_part is not None else {}
        if mom_coef is not None:
            kw["mom_coef"] = mom_coef
        dYp, dZ = be.mlp_bwd(dY, Z, W1, W2, K, bn=bn, outs=list(outs), **kw)
        be.wgrad(dYp, Z, Gr[pre + "2.weight"], db=Gr[pre + "2.bias"], act_in=True)
        be.wgrad_cat(dZ, segs, Gr[pre + "0.weight"], db=Gr[pre + "0.bias"])

    def _fiber_bn_sums(self, d, ss):
        """SModel's node_mlp_2 BatchNorm backward sums made by TModel's edge
        backward, whose epilogue finishes g_xs (pfsgnn_target_bwd_bn): the
        (Yp, mu, var, eps) to hand it, or None (then mlp_bwd sums them)."""
        sS = ss.get("sS")
        if (d.sp is not None or not self.normed or not getattr(self.be, "fiber_bn_sums", False)
                or os.environ.get("PFSGNN_FIBER_BN_SUMS", "1") == "0" or sS is None
                or sS[0] == "ops" or sS[2] is None or sS[2][0] == "eval"):
            return None
        Yp, mu, var, _ = sS[2]
        return (Yp, mu, var, self.bn_eps)

    def _bn_eval_bwd(self, P, Gr, key, times, dY, Yp, rm, rv):
        """Backward of an eval-mode BatchNorm1d (running statistics rm, rv; applied
        ``times`` times) at its input Yp: dgamma / dbeta accumulate into Gr and
        the input gradient scale * dY comes back (pfsgnn_bn_eval_bwd_coef)."""
        be = self.be
        g, b = P[key + "weight"], P[key + "bias"]
        inv, scale = be.bn_eval_bwd_coef(g, b, rm, rv, self.bn_eps, times)
        Sg, Sgx = be.rows_bn_sums(dY, Yp, rm, inv)
        be.bn_eval_bwd_coef(g, b, rm, rv, self.bn_eps, times, Sg, Sgx, Gr[key + "weight"],
                            Gr[key + "bias"])
        return be.affine_rows(dY, scale, be.zeros(scale.shape[0]))

    # MLPs outside the fused op's shapes (output > 16 or a width > 112: Fdim 16's
    # SModel node_mlp_2, a node_prediction decoder over many classes) run as
    # separate Linear ops
    def _mlp_fwd_ops(self, P, BN, pre, segs, N, bnkey):
        be = self.be
        W1, b1, W2, b2 = P[pre + "0.weight"], P[pre + "0.bias"], P[pre + "2.weight"], P[pre + "2.bias"]
        Z = be.lin_cat(W1, segs, N, b=b1)
        Y = be.lin(W2, 0, W2.shape[1], Z, b=b2, act_in=True)
        bns = None
        if bnkey is not None:
            if self.training:
                Yn, mu, var = be.bn_fwd(Y, P[bnkey + "weight"], P[bnkey + "bias"],
                                        BN.get(bnkey + "running_mean"), BN.get(bnkey + "running_var"),
                                        self.bn_momentum, self.bn_eps)
                bns = (Y, mu, var, bnkey)
                Y = Yn
            else:
                rm, rv = BN[bnkey + "running_mean"], BN[bnkey + "running_var"]
                sc, sh = be.bn_eval_coef(P[bnkey + "weight"], P[bnkey + "bias"], rm, rv,
                                         self.bn_eps, 1)
                bns = ("eval", Y, bnkey, rm, rv)
                Y = be.affine_rows(Y, sc, sh)
        return Y, ("ops", segs, Z, bns)

    def _mlp_bwd_ops(self, P, Gr, pre, dY, saved, outs):
        be = self.be
        _, segs, Z, bns = saved
        W1, W2 = P[pre + "0.weight"], P[pre + "2.weight"]
        if bns is not None and bns[0] == "eval":
            dY = self._bn_eval_bwd(P, Gr, bns[2], 1, dY, bns[1], bns[3], bns[4])
            bns = None
        if bns is not None:
            Yp, mu, var, key = bns
            dY = be.bn_bwd(dY, Yp, mu, var, P[key + "weight"], self.bn_eps, Gr[key + "weight"],
                           Gr[key + "bias"])
        be.wgrad(dY, Z, Gr[pre + "2.weight"], db=Gr[pre + "2.bias"], act_in=True)
        dZ = be.lin_t(W2, 0, W2.shape[1], dY, z=Z)
        be.wgrad_cat(dZ, segs, Gr[pre + "0.weight"], db=Gr[pre + "0.bias"])
        r = 0
        for t, rows, add in outs:
            if t is not None:
                be.lin_t(W1, r, rows, dZ, out=t, add=add)
            r += rows

    def _gu_add(self, X, G, g_u):
        """g_u += per-graph sums of X (a u[batch] gradient, gnn.py:100/153/191);
        inside a backward block they are batched into one launch (_gu_flush)."""
        pend = getattr(self, "_gu_pend", None)
        if pend is not None:
            pend.append((X, g_u))
        else:
            self.be.graph_reduce(X, G, out=g_u)

    def _gu_flush(self, G):
        pend, self._gu_pend = getattr(self, "_gu_pend", None) or [], []
        self._gu_flush_list(pend, G)

    def _gu_flush_list(self, pend, G):
        for i in range(0, len(pend), 4):
            part = pend[i:i + 4]
            assert all(t is part[0][1] for _, t in part)
            self.be.graph_reduce_multi([X for X, _ in part], G, part[0][1])

    def _rms_eps(self, t):
        return self.rms_eps if self.rms_eps is not None else torch.finfo(t.dtype).eps

    # ========================================================= model pieces
    # --- EdgeModel (gnn.py:86-101)
    def node_parts(self, P, d, pe, ps, xs, xt, u):
        """The node parts of a block's first per-edge Linear layers that depend
        only on the block's inputs -- EdgeModel's Ps, Pt (gnn.py:100) and
        SModel's Qt (gnn.py:136) -- as one batched launch."""
        F = self.F
        W1, b1 = P[pe + "0.weight"], P[pe + "0.bias"]
        Ws1, bs1 = P[ps + "node_mlp_1.0.weight"], P[ps + "node_mlp_1.0.bias"]
        if 4 * F > 64:
            return None
        return self.be.linear_batch([
            ("cat", W1, [(xs, 0, False)], d.NS, None),
            ("cat", W1, [(xt, F, False), (u, 3 * F, True)], d.NT, b1),
            ("cat", Ws1, [(xt, 0, False)], d.NT, bs1)])

    def edge_fwd(self, P, BN, d, pre, xs, xt, xe3, u, parts=None):
        be, F = self.be, self.F
        W1, b1 = P[pre + "0.weight"], P[pre + "0.bias"]
        W2, b2 = P[pre + "2.weight"], P[pre + "2.bias"]
        if parts is not None:
            Ps, Pt = parts
        else:
            Ps = be.lin(W1, 0, F, xs)
            Pt = be.lin_cat(W1, [(xt, F, False), (u, 3 * F, True)], d.NT, b=b1)
        if self.normed and self.training:
            # the double BatchNorm's finalize rides in the moments pass
            key = pre + "norm."
            y, mu1, var1, sc, sh, inv1 = be.edge_mlp_fwd_bn(
                d, xe3[0], xe3[1], xe3[2], Ps, Pt, W1, W2, b2,
                (P[key + "weight"], P[key + "bias"], BN.get(key + "running_mean"),
                 BN.get(key + "running_var"), self.bn_momentum, self.bn_eps))
            return dict(xs=xs, xt=xt, xe3=xe3, u=u, Ps=Ps, Pt=Pt, y=y, mu1=mu1, var1=var1,
                        sc=sc, sh=sh, inv1=inv1)
        y, mu1, var1 = be.edge_mlp_fwd(d, xe3[0], xe3[1], xe3[2], Ps, Pt, W1, W2, b2)
        if self.normed and not self.training:
            # eval: both BatchNorm applications (gnn.py:101) on running statistics
            key = pre + "norm."
            sc, sh = be.bn_eval_coef(P[key + "weight"], P[key + "bias"], BN[key + "running_mean"],
                                     BN[key + "running_var"], self.bn_eps, 2)
            return dict(xs=xs, xt=xt, xe3=xe3, u=u, Ps=Ps, Pt=Pt, y=y, mu1=mu1, var1=var1,
                        sc=sc, sh=sh, inv1=None, rm=BN[key + "running_mean"],
                        rv=BN[key + "running_var"])
        return dict(xs=xs, xt=xt, xe3=xe3, u=u, Ps=Ps, Pt=Pt, y=y, mu1=mu1, var1=var1,
                    sc=None, sh=None, inv1=None)

    def edge_bn_coef(self, P, Gr, d, pre, st, Sg, Sgx):
        """The double BatchNorm's backward coefficients from its gradient sums
        (taken about edge_bnstat's centre and scale)."""
        key = pre + "norm."
        if "rm" in st:      # eval: running statistics, an affine map applied twice
            _, scale = self.be.bn_eval_bwd_coef(P[key + "weight"], P[key + "bias"], st["rm"],
                                                st["rv"], self.bn_eps, 2, Sg, Sgx,
                                                Gr[key + "weight"], Gr[key + "bias"])
            z = self.be.zeros(scale.shape[0])
            return scale, z, z
        return self.be.bn2_bwd_coef(Sg, Sgx, st["mu1"], st["var1"], P[key + "weight"], d.E,
                                    self.bn_eps, Gr[key + "weight"], Gr[key + "bias"])

    def edge_bnstat(self, P, pre, st):
        """(centre, 1/scale) of the edge BatchNorm's gradient sums: the batch
        statistics in training, the running statistics in eval."""
        if "rm" in st:
            key = pre + "norm."
            inv, _ = self.be.bn_eval_bwd_coef(P[key + "weight"], P[key + "bias"], st["rm"],
                                              st["rv"], self.bn_eps, 2)
            return st["rm"], inv
        return st["mu1"], st["inv1"]

    def edge_bwd(self, P, Gr, d, pre, st, g_tot, bnc, want_gxe, g_xs, g_xt, g_u):
        """g_tot: d loss / d xe_new (canonical [F, E]); bnc: the BatchNorm's
        backward coefficients (alpha, gam0, gam1) (edge_bn_coef), None if unnormed.
        Adds the node-input gradients into g_xs / g_xt / g_u; returns d loss / d xe_in."""
        be, F, G = self.be, self.F, d.G
        if self.normed:
            alpha, gam0, gam1 = bnc
        else:
            alpha, gam0, gam1 = be.ones(F), be.zeros(F), be.zeros(F)
        W1, W2 = P[pre + "0.weight"], P[pre + "2.weight"]
        xe, xsc, xsh = st["xe3"]
        dW1 = Gr[pre + "0.weight"]
        # the node-input gradients g_xs += W1s^T GzEs, g_xt += W1t^T GzEt ride in
        # the op's per-fiber / per-class reductions; Vu = W1u^T GzEt per class
        g_xe, GzEs, GzEt, Vu = be.edge_mlp_bwd(d, g_tot, alpha, gam0, gam1, st["y"], xe, xsc, xsh,
                                               st["Ps"], st["Pt"], W1, W2, dW1,
                                               Gr[pre + "2.weight"], Gr[pre + "2.bias"],
                                               want_gxe=want_gxe, nodes=(g_xs, g_xt))
        be.wgrad(GzEs, st["xs"], dW1, col0=0)
        # x_t[tgt] and u[batch] columns in one pass (u's gradient sums over classes)
        be.wgrad_cat(GzEt, [(st["xt"], F, False), (st["u"], 3 * F, True)], dW1,
                     db=Gr[pre + "0.bias"])
        self._gu_add(Vu, G, g_u)             # g_u += W1u^T (sum of GzEt over each graph)
        return g_xe

    # --- SModel (gnn.py:123-154)
    def source_fwd(self, P, BN, d, pre, xs, xt, xe3, u, Qt=None, epi=None):
        """``epi`` (fused block tail): {name: (W, col0, nk, b)} linear maps of
        the new x_s done in its normalising pass, returned under their names."""
        be, F = self.be, self.F
        Ws1, bs1 = P[pre + "node_mlp_1.0.weight"], P[pre + "node_mlp_1.0.bias"]
        Ws2, bs2 = P[pre + "node_mlp_1.2.weight"], P[pre + "node_mlp_1.2.bias"]
        if Qt is None:
            Qt = be.lin(Ws1, 0, F, xt, b=bs1)
        hmom = be.empty(8 * F, d.NS)
        # the per-edge messages, kept for the backward (complete graphs on the
        # mfma paths; None where source_bwd recomputes them)
        msg = be.msg_cache(d) if (self.training or self.want_grad) and \
            hasattr(be, "msg_cache") else None
        if msg is not None:
            mom = be.source_fwd(d, xe3[0], xe3[1], xe3[2], Qt, Ws1, Ws2, bs2, hmom, msg=msg)
        else:
            mom = be.source_fwd(d, xe3[0], xe3[1], xe3[2], Qt, Ws1, Ws2, bs2, hmom)
        # node_mlp_2 input [x, mean, std, skew, kurt, u[batch]] (gnn.py:153), in place,
        # + its BatchNorm1d (gnn.py:154) in the same fused op
        hS = [(xs, 0, False), (hmom, F, False), (u, 9 * F, True)]
        st = dict(xs=xs, xt=xt, xe3=xe3, u=u, Qt=Qt, mom=mom, msg=msg)
        if epi:
            names = list(epi)
            xs_new, sS, outs = self.mlp_fwd(P, pre + "node_mlp_2.", hS, pre + "norm.", BN,
                                            epi=[epi[k] for k in names])
            st.update(zip(names, outs))
        else:
            xs_new, sS = self.mlp_fwd(P, pre + "node_mlp_2.", hS, pre + "norm.", BN)
        st.update(sS=sS, xs_new=xs_new)
        return st

    def _mom_epi_ok(self, d, st):
        """node_mlp_2's backward can turn the moment gradients into the
        coefficients itself (pfsgnn_mlp_bwd_pre's coef): complete graphs, the
        fused MLP in its wide register form, 16..20 message channels."""
        sS = st.get("sS")
        return (d.sp is None and getattr(self.be, "fiber_bn_sums", False)
                and self.F in (8, 10) and sS is not None and sS[0] != "ops"
                and os.environ.get("PFSGNN_MOM_EPI", "1") != "0"
                and os.environ.get("PFSGNN_MLP_BWD_RS", "1") != "0")

    def source_node_bwd(self, P, Gr, d, pre, st, g_xs_new, g_xs, g_u, bn_part=None):
        """Node half of the SModel backward; returns the per-fiber moment coefficients."""
        be, F, G = self.be, self.F, d.G
        gu = be.empty(F, d.NS)               # d loss / d u[batch], per fiber
        if self._mom_epi_ok(d, st):
            # d loss / d [mean, std, skew, kurt] never leaves the kernel: its
            # epilogue makes the coefficients (k_moment_coef's arithmetic)
            coef = be.empty(4, 2 * F, d.NS)
            self.mlp_bwd(P, Gr, pre + "node_mlp_2.", g_xs_new, st["sS"],
                         outs=[(g_xs, F, True), (None, 8 * F, False), (gu, F, False)],
                         bn_part=bn_part, mom_coef=(st["mom"], coef, F, d.NC))
            self._gu_add(gu, G, g_u)
            return coef
        gst = be.empty(8 * F, d.NS)          # d loss / d [mean, std, skew, kurt]
        self.mlp_bwd(P, Gr, pre + "node_mlp_2.", g_xs_new, st["sS"],
                     outs=[(g_xs, F, True), (gst, 8 * F, False), (gu, F, False)],
                     bn_part=bn_part)
        self._gu_add(gu, G, g_u)
        # messages per fiber: NC on complete graphs, the fiber degree otherwise
        return be.moment_coef(st["mom"], gst, d.NC if d.sp is None else d.sp.fib_ptr)

    def source_edge_bwd(self, P, Gr, d, pre, st, coef, tpart, g_next, bnstat, g_xt, se=None,
                        epre=None, tmask=None):
        """SModel edge backward; with the upstream EdgeModel's state ``se`` (and
        its prefix) the edge BatchNorm's backward coefficients come out of the
        same call -> (g_tot, (alpha, gam0, gam1)); else -> (g_tot, Sg, Sgx).
        ``tmask``: the TModel forward's mask for ``tpart`` (target_fwd)."""
        be, F = self.be, self.F
        Ws1, Ws2 = P[pre + "node_mlp_1.0.weight"], P[pre + "node_mlp_1.2.weight"]
        y, sc, sh = st["xe3"]
        bn2 = None
        if se is not None and bnstat is not None:
            key = epre + "norm."
            bn2 = (P[key + "weight"], se["var1"], d.E, self.bn_eps, Gr[key + "weight"],
                   Gr[key + "bias"])
        out = be.source_bwd(
            d, y, sc, sh, st["Qt"], Ws1, Ws2, P[pre + "node_mlp_1.2.bias"], st["mom"][0], coef,
            tpart, g_next, bnstat, Gr[pre + "node_mlp_1.0.weight"], Gr[pre + "node_mlp_1.2.weight"],
            Gr[pre + "node_mlp_1.2.bias"], bn2=bn2, g_xt=g_xt,  # + g_xt += Ws1x^T GzS
            **({"tmask": tmask} if tmask is not None and tpart is not None else {}),
            **({"msg": st["msg"]} if st.get("msg") is not None else {}))
        g_tot, GzS = out[0], out[1]
        be.wgrad(GzS, st["xt"], Gr[pre + "node_mlp_1.0.weight"], col0=0,
                 db=Gr[pre + "node_mlp_1.0.bias"])
        if bn2 is not None:
            return g_tot, out[4]
        return g_tot, out[2], out[3]

    # --- TModel (gnn.py:175-192)
    def target_fwd(self, P, BN, d, pre, xs, xt, xe3, u, Rs=None, glob=None):
        """``glob`` (fused block tail) = (GlobalModel prefix, next block's prefix
        or None): TModel's node_mlp_2 + BatchNorm and the GlobalModel run as one
        op (target_global_fwd); the GlobalModel's state comes back as ["su"] and
        the next block's class parts (Pt, Qt) as ["parts_t"]."""
        be, F = self.be, self.F
        Wt1, bt1 = P[pre + "node_mlp_1.0.weight"], P[pre + "node_mlp_1.0.bias"]
        Wt2, bt2 = P[pre + "node_mlp_1.2.weight"], P[pre + "node_mlp_1.2.bias"]
        if Rs is None:
            Rs = be.lin(Wt1, 0, F, xs, b=bt1)
        # the LeakyReLU mask of the per-edge layer, kept for the backward (MFMA
        # path; None where the backward recomputes it)
        tmask = be.tmask(d) if self.training and hasattr(be, "tmask") else None
        if glob is not None and d.sp is None and hasattr(be, "target_block_fwd") and \
                d.G * -(-d.NC // 32) <= 512 and d.NC <= 2048 and \
                os.environ.get("PFSGNN_CLASS_TAIL", "1") != "0":
            return self._target_block_fwd(P, BN, d, pre, xs, xt, xe3, u, Rs, tmask, glob)
        if d.sp is None:
            # the second Linear after the per-class sum, in the op's reduction epilogue
            hsum, agg = be.target_fwd(d, xe3[0], xe3[1], xe3[2], Rs, Wt1,
                                      agg=(Wt2, bt2, float(d.NF)),
                                      **({"tmask": tmask} if tmask is not None else {}))
        else:
            hsum = be.target_fwd(d, xe3[0], xe3[1], xe3[2], Rs, Wt1,
                                 **({"tmask": tmask} if tmask is not None else {}))
            # the bias of the summed messages is deg(c) * b2 (gnn.py:190)
            agg = be.lin(Wt2, 0, 2 * F, hsum)
            be.lin(bt2.view(-1, 1), 0, 1, d.sp.deg_t, out=agg, add=True)
        # node_mlp_2 input [x, agg, u[batch]] (gnn.py:191), in place, + BatchNorm1d
        hT = [(xt, 0, False), (agg, F, False), (u, 3 * F, True)]
        st = dict(xs=xs, xt=xt, xe3=xe3, u=u, Rs=Rs, hsum=hsum, tmask=tmask)
        if glob is None:
            xt_new, sT = self.mlp_fwd(P, pre + "node_mlp_2.", hT, pre + "norm.", BN)
            st.update(sT=sT, xt_new=xt_new)
            return st
        pg, pnext = glob
        m2 = pre + "node_mlp_2."
        w = P[pg + "norm.weight"]
        nxt = None
        if pnext is not None:
            pe, ps = pnext + "edge_model.", pnext + "s_model."
            nxt = (P[pe + "0.weight"], P[pe + "0.bias"], P[ps + "node_mlp_1.0.weight"],
                   P[ps + "node_mlp_1.0.bias"])
        r = be.target_global_fwd(hT, d.G, d.NC, P[m2 + "0.weight"], P[m2 + "0.bias"],
                                 P[m2 + "2.weight"], P[m2 + "2.bias"],
                                 self._bn_args(P, BN, pre + "norm."), xs, d.NF, u,
                                 P[pg + "0.weight"], P[pg + "0.bias"], P[pg + "2.weight"],
                                 P[pg + "2.bias"], w, self._rms_eps(u), nxt)
        st.update(sT=(hT, r["Z"], (r["Yp"], r["mu"], r["var"], pre + "norm.")), xt_new=r["xt"])
        st["su"] = dict(sU=([(u, 0, False), (r["means"], F, False)], r["gZ"], None), v=r["gV"],
                        rms=r["rms"], u_new=r["u"], fused=True)
        st["parts_t"] = (r["Pt"], r["Qt"])
        return st

    def _target_block_fwd(self, P, BN, d, pre, xs, xt, xe3, u, Rs, tmask, glob):
        """target_fwd's fused form on a complete batch: TModel's per-edge layer,
        then its class side, node_mlp_2 + BatchNorm, the GlobalModel and the next
        block's class parts in one launch (pfsgnn_target_block_fwd)."""
        be, F = self.be, self.F
        pg, pnext = glob
        m2 = pre + "node_mlp_2."
        nxt = None
        if pnext is not None:
            pe, ps = pnext + "edge_model.", pnext + "s_model."
            nxt = (P[pe + "0.weight"], P[pe + "0.bias"], P[ps + "node_mlp_1.0.weight"],
                   P[ps + "node_mlp_1.0.bias"])
        r = be.target_block_fwd(d, xe3[0], xe3[1], xe3[2], Rs, P[pre + "node_mlp_1.0.weight"],
                                P[pre + "node_mlp_1.2.weight"], P[pre + "node_mlp_1.2.bias"],
                                tmask, xt, u, P[m2 + "0.weight"], P[m2 + "0.bias"],
                                P[m2 + "2.weight"], P[m2 + "2.bias"],
                                self._bn_args(P, BN, pre + "norm."), xs, P[pg + "0.weight"],
                                P[pg + "0.bias"], P[pg + "2.weight"], P[pg + "2.bias"],
                                P[pg + "norm.weight"], self._rms_eps(u), nxt)
        hT = [(xt, 0, False), (r["agg"], F, False), (u, 3 * F, True)]
        st = dict(xs=xs, xt=xt, xe3=xe3, u=u, Rs=Rs, hsum=r["hsum"], tmask=tmask)
        st.update(sT=(hT, r["Z"], (r["Yp"], r["mu"], r["var"], pre + "norm.")), xt_new=r["xt"])
        st["su"] = dict(sU=([(u, 0, False), (r["means"], F, False)], r["gZ"], None), v=r["gV"],
                        rms=r["rms"], u_new=r["u"], fused=True)
        st["parts_t"] = (r["Pt"], r["Qt"])
        return st

    def _class_bwd_ok(self, d, su, stt):
        """The fused class backward's conditions: a complete batch, training
        BatchNorm, the fused forward tail's GlobalModel state."""
        sT = stt.get("sT")
        return (d.sp is None and self.normed and self.F in (8, 10, 16) and d.NC <= 1024
                and hasattr(self.be, "target_class_bwd") and su.get("fused")
                and sT is not None and sT[2] is not None and sT[2][0] != "eval"
                and os.environ.get("PFSGNN_CLASS_BWD", "1") != "0")

    def _class_bwd(self, P, Gr, d, p, su, stt, pend, g_u, g_xs_new, g_xt_new, g_xt_in, g_u_in):
        """global_bwd + target_node_bwd (and the block above's u-gradient flush)
        as one launch (pfsgnn_target_class_bwd); their weight gradients stay
        deferred jobs.  -> g_hsum."""
        be, F, G = self.be, self.F, d.G
        pg, pt = p + "global_model.", p + "t_model."
        m2 = pt + "node_mlp_2."
        segsU, Zg, _ = su["sU"]
        hT, ZT, (Yp, mu, var, key) = stt["sT"]
        w = P[pg + "norm.weight"]
        gH = P[pg + "0.weight"].shape[0]
        gV, gdZ, dwp = be.empty(F, G), be.empty(gH, G), be.empty(F, G)
        r = be.target_class_bwd(d, pend, g_u, su["v"], w, su["rms"], Zg, P[pg + "0.weight"],
                                P[pg + "2.weight"], gV, gdZ, dwp, g_u_in, g_xs_new, g_xt_new, Yp,
                                mu, var, P[key + "weight"], self.bn_eps, Gr[key + "weight"],
                                Gr[key + "bias"], ZT, P[m2 + "0.weight"], P[m2 + "2.weight"],
                                P[pt + "node_mlp_1.2.weight"], g_xt_in)
        be.wgrad(gV, Zg, Gr[pg + "2.weight"], db=Gr[pg + "2.bias"], act_in=True)
        be.wgrad_cat(gdZ, segsU, Gr[pg + "0.weight"], db=Gr[pg + "0.bias"])
        be.wgrad(dwp, be._ones_row(G), Gr[pg + "norm.weight"].view(F, 1))
        be.wgrad(r["dYp"], ZT, Gr[m2 + "2.weight"], db=Gr[m2 + "2.bias"], act_in=True)
        be.wgrad_cat(r["dZ"], hT, Gr[m2 + "0.weight"], db=Gr[m2 + "0.bias"])
        self._gu_add(r["gu_t"], G, g_u_in)
        be.wgrad(r["g_agg"], stt["hsum"], Gr[pt + "node_mlp_1.2.weight"],
                 db=Gr[pt + "node_mlp_1.2.bias"], dbscale=float(d.NF))
        return r["g_hsum"]

    def target_node_bwd(self, P, Gr, d, pre, st, g_xt_new, g_xt, g_u):
        be, F, G = self.be, self.F, d.G
        g_agg = be.empty(2 * F, d.NT)
        gu = be.empty(F, d.NT)
        self.mlp_bwd(P, Gr, pre + "node_mlp_2.", g_xt_new, st["sT"],
                     outs=[(g_xt, F, True), (g_agg, 2 * F, False), (gu, F, False)])
        self._gu_add(gu, G, g_u)
        Wt2 = P[pre + "node_mlp_1.2.weight"]
        if d.sp is None:
            be.wgrad(g_agg, st["hsum"], Gr[pre + "node_mlp_1.2.weight"],
                     db=Gr[pre + "node_mlp_1.2.bias"], dbscale=float(d.NF))
        else:
            be.wgrad(g_agg, st["hsum"], Gr[pre + "node_mlp_1.2.weight"])
            be.wgrad(g_agg, d.sp.deg_t, Gr[pre + "node_mlp_1.2.bias"].view(-1, 1))
        return be.lin_t(Wt2, 0, 2 * F, g_agg)

    def target_edge_bwd(self, P, Gr, d, pre, st, g_hsum, want_gxe, g_xs, bn_sums=None):
        """-> gxe; with ``bn_sums`` (_fiber_bn_sums) -> (gxe, BatchNorm sum partials)."""
        be, F = self.be, self.F
        Wt1 = P[pre + "node_mlp_1.0.weight"]
        y, sc, sh = st["xe3"]
        kw = {"tmask": st["tmask"]} if st.get("tmask") is not None else {}
        if bn_sums is not None:
            kw["bn_sums"] = bn_sums
        out = be.target_bwd(d, y, sc, sh, st["Rs"], Wt1, g_hsum,
                            Gr[pre + "node_mlp_1.0.weight"], want_gxe=want_gxe,
                            g_xs=g_xs, **kw)          # + g_xs += Wt1s^T GzT
        GzT, gxe = out[0], out[1]
        be.wgrad(GzT, st["xs"], Gr[pre + "node_mlp_1.0.weight"], col0=0,
                 db=Gr[pre + "node_mlp_1.0.bias"])
        return (gxe, out[2]) if bn_sums is not None else gxe

    # --- GlobalModel (gnn.py:208-223; its RMSNorm also runs twice)
    def global_fwd(self, P, d, pre, xs, xt, u):
        be, F, G = self.be, self.F, d.G
        W1 = P[pre + "0.weight"]
        if 3 * F <= 192 and W1.shape[0] <= 192:
            # the whole model of each graph in one op (means, MLP, RMSNorm x2)
            w = P[pre + "norm.weight"] if self.normed else None
            u_new, means, Z, v, rms = be.global_fwd(
                xs, xt, u, W1, P[pre + "0.bias"], P[pre + "2.weight"], P[pre + "2.bias"], w,
                self._rms_eps(u) if w is not None else 0.0, G)
            sU = ([(u, 0, False), (means, F, False)], Z, None)
            return dict(sU=sU, v=v, rms=rms, u_new=u_new, fused=True)
        # [u, mean x_s, mean x_t] (gnn.py:218-220), in place
        hU = [(u, 0, False), (be.graph_mean2(xs, xt, G), F, False)]
        v, sU = self.mlp_fwd(P, pre, hU)
        if self.normed:
            u_new, rms = be.rms2_fwd(v, P[pre + "norm.weight"], self._rms_eps(v))
        else:
            u_new, rms = v, None
        return dict(sU=sU, v=v, rms=rms, u_new=u_new)

    def global_bwd(self, P, Gr, d, pre, st, g_u_new, g_xs, g_xt, g_u):
        be, F = self.be, self.F
        if st.get("fused"):
            pre_w = pre + "norm.weight"
            segs, Z, _ = st["sU"]
            W1, W2 = P[pre + "0.weight"], P[pre + "2.weight"]
            g_v, dZ = be.global_bwd(g_u_new, st["v"], P[pre_w] if self.normed else None, st["rms"],
                                    self._rms_eps(st["v"]), Gr[pre_w] if self.normed else None,
                                    Z, W1, W2, g_u, g_xs, 1.0 / d.NF, g_xt, 1.0 / d.NC)
            be.wgrad(g_v, Z, Gr[pre + "2.weight"], db=Gr[pre + "2.bias"], act_in=True)
            be.wgrad_cat(dZ, segs, Gr[pre + "0.weight"], db=Gr[pre + "0.bias"])
            return
        if self.normed:
            g_v = be.rms2_bwd(g_u_new, st["v"], P[pre + "norm.weight"], st["rms"],
                              self._rms_eps(st["v"]), Gr[pre + "norm.weight"])
        else:
            g_v = g_u_new
        g_m = be.empty(2 * F, d.G)          # d loss / d [mean x_s; mean x_t]
        self.mlp_bwd(P, Gr, pre, g_v, st["sU"], outs=[(g_u, F, True), (g_m, 2 * F, False)])
        be.graph_bcast_add2(g_xs, 1.0 / d.NF, g_xt, 1.0 / d.NC, g_m)

    # ============================================================ GNN path
    def forward(self, P, BN, d, xs_in, xt_in, xe_in, u_in, training=True, want_grad=False):
        """GNN.forward (gnn.py:280-305).  xs_in [Fs, NS], xt_in [Ft, NT], xe_in [F, E],
        u_in [F, G] (channel-major).  Returns a context with the outputs
        (xs, xt, xe3, u) and everything backward needs."""
        # eval (training=False): BatchNorm on running statistics, nothing updated;
        # with want_grad the context also serves a backward (gnn.eval() under
        # autograd: the norms are affine maps then, gnn.py:101/154/192)
        self.training = training
        self.want_grad = want_grad
        xs, s_enc = self.mlp_fwd(P, "encoder_s.", xs_in)
        xt, t_enc = self.mlp_fwd(P, "encoder_t.", xt_in)
        ctx = {"d": d, "enc": (s_enc, t_enc), "blocks": [], "training": training,
               "want_grad": want_grad}
        xe3 = (xe_in, None, None)
        u = u_in
        parts = None
        for b in range(self.B):
            p = f"mpb.{b}."
            pn = f"mpb.{b + 1}." if b + 1 < self.B else None
            if parts is None:
                parts = self.node_parts(P, d, p + "edge_model.", p + "s_model.", xs, xt, u)
            se = self.edge_fwd(P, BN, d, p + "edge_model.", xs, xt, xe3, u,
                               parts=None if parts is None else parts[:2])
            xe3n = (se["y"], se["sc"], se["sh"])
            # fused block tail: x_s' is mapped to TModel's Rs (and the next block's
            # EdgeModel Ps) where it is normalised; TModel's node MLP, the
            # GlobalModel and the next block's class parts run as one op
            fused = self._fused_tail_ok(P, d, p + "s_model.", p + "t_model.", p + "global_model.")
            epi = None
            if fused:
                F = self.F
                pt1 = p + "t_model.node_mlp_1.0."
                epi = {"Rs": (P[pt1 + "weight"], 0, 2 * F, P[pt1 + "bias"])}
                if pn is not None:
                    epi["Ps_next"] = (P[pn + "edge_model.0.weight"], 0, 4 * F, None)
            ss = self.source_fwd(P, BN, d, p + "s_model.", xs, xt, xe3n, u,
                                 Qt=None if parts is None else parts[2], epi=epi)
            stt = self.target_fwd(P, BN, d, p + "t_model.", ss["xs_new"], xt, xe3n, u,
                                  Rs=ss.get("Rs"),
                                  glob=(p + "global_model.", pn) if fused else None)
            if fused:
                su = stt.pop("su")
                pt = stt.pop("parts_t")
                parts = (ss["Ps_next"],) + tuple(pt) if pn is not None else None
            else:
                su = self.global_fwd(P, d, p + "global_model.", ss["xs_new"], stt["xt_new"], u)
                parts = None
            ctx["blocks"].append((se, ss, stt, su))
            xs, xt, xe3, u = ss["xs_new"], stt["xt_new"], xe3n, su["u_new"]
        ctx["out"] = (xs, xt, xe3, u)
        return ctx

    def backward(self, P, Gr, ctx, g_xe_out=None, g_xs_out=None, g_xt_out=None, g_u_out=None):
        """Accumulates parameter gradients into ``Gr`` (same keys as ``P``).
        g_xe_out is [F, E] canonical, w.r.t. the final edge features."""
        d, be, F = ctx["d"], self.be, self.F
        if not ctx.get("training", True) and not ctx.get("want_grad", False):
            raise NotImplementedError("this eval-mode forward ran for inference only (forward "
                                      "with want_grad=True to differentiate through it)")
        # node weight-gradient reductions are batched over the pass (flushed below)
        be.defer_begin()
        # the final edge BatchNorm's backward sums, made by the loss backward
        # when it alone produced g_xe (train._LossFn; any other consumer drops them)
        g_bn_part = ctx.pop("g_xe_bn_part", None)
        try:
            self._backward(P, Gr, ctx, d, g_xs_out, g_xt_out, g_xe_out, g_u_out, g_bn_part)
        finally:
            self._gu_pend = None
            be.defer_flush()

    def _backward(self, P, Gr, ctx, d, g_xs_out, g_xt_out, g_xe_out, g_u_out, g_bn_part=None):
        be, F = self.be, self.F
        g_xs, g_xt, g_xe, g_u = g_xs_out, g_xt_out, g_xe_out, g_u_out
        self._gu_pend = []
        prev_pend = []     # the block above's pending u[batch] gradients
        stride = (F * (d.NS + d.NT + d.G) + 63) // 64 * 64     # 256-byte aligned slices
        acc_all = be.zeros(self.B * stride)
        for b in reversed(range(self.B)):
            se, ss, stt, su = ctx["blocks"][b]
            p = f"mpb.{b}."
            # the three input-gradient accumulators of every block share one
            # buffer zeroed once per backward pass (one fill, not one per block)
            acc = acc_all[b * stride:b * stride + F * (d.NS + d.NT + d.G)]
            g_xs_in = acc[:F * d.NS].view(F, d.NS)
            g_xt_in = acc[F * d.NS:F * (d.NS + d.NT)].view(F, d.NT)
            g_u_in = acc[F * (d.NS + d.NT):].view(F, d.G)
            # gradients that are None are exactly zero: the models whose outputs
            # feed nothing downstream (the last block's S/T/Global under the
            # train.py objective) contribute nothing and are skipped
            live_t = g_u is not None or g_xt is not None
            live_s = live_t or g_xs is not None
            bnstat = self.edge_bnstat(P, p + "edge_model.", se) if self.normed else None
            ev = "rm" in se     # eval-mode forward: BatchNorm on running statistics
            if live_s:
                # below the last block g_xs / g_xt are this loop's own accumulators
                # and are updated in place; the caller's gradients are copied
                own = b < self.B - 1
                g_xs_new = be.zeros(F, d.NS) if g_xs is None else (g_xs if own else g_xs.clone())
                g_xt_new = be.zeros(F, d.NT) if g_xt is None else (g_xt if own else g_xt.clone())
                tpart = None
                if (g_u is not None and live_t and len(prev_pend) <= 4
                        and all(tg is g_u for _, tg in prev_pend)
                        and self._class_bwd_ok(d, su, stt)):
                    # the block's whole class side in one launch; it also sums the
                    # block above's pending u[batch] gradients into g_u
                    g_hsum = self._class_bwd(P, Gr, d, p, su, stt, [X for X, _ in prev_pend],
                                             g_u, g_xs_new, g_xt_new, g_xt_in, g_u_in)
                    prev_pend = []
                else:
                    self._gu_flush_list(prev_pend, d.G)
                    prev_pend = []
                    if g_u is not None:
                        self.global_bwd(P, Gr, d, p + "global_model.", su, g_u, g_xs_new,
                                        g_xt_new, g_u_in)
                    if live_t:
                        g_hsum = self.target_node_bwd(P, Gr, d, p + "t_model.", stt, g_xt_new,
                                                      g_xt_in, g_u_in)
                bn_part = None
                if live_t:
                    # (g_xs_new is final after TModel's edge backward: its epilogue
                    # also makes SModel's BatchNorm backward sums)
                    bn_sums = self._fiber_bn_sums(d, ss)
                    r = self.target_edge_bwd(P, Gr, d, p + "t_model.", stt, g_hsum, False,
                                             g_xs_new, bn_sums=bn_sums)
                    if bn_sums is not None:
                        bn_part = r[1]
                    tpart = (stt["Rs"], P[p + "t_model.node_mlp_1.0.weight"], g_hsum)
                coef = self.source_node_bwd(P, Gr, d, p + "s_model.", ss, g_xs_new, g_xs_in, g_u_in,
                                            bn_part=bn_part)
                g_tot, *bnc = self.source_edge_bwd(P, Gr, d, p + "s_model.", ss, coef, tpart,
                                                   g_xe, bnstat, g_xt_in,
                                                   se=None if ev else se,
                                                   epre=p + "edge_model.",
                                                   tmask=stt.get("tmask") if live_t else None)
                if not self.normed:
                    bnc = None
                elif ev:
                    bnc = self.edge_bn_coef(P, Gr, d, p + "edge_model.", se, *bnc)
                else:
                    bnc = bnc[0]
            else:
                g_tot = be.zeros(F, d.EP) if g_xe is None else g_xe
                bnc = None
                if self.normed and b == self.B - 1 and g_xe is not None and g_bn_part is not None:
                    # the loss backward, the only consumer of the final edge
                    # state, made this BatchNorm's backward sums as it wrote g_xe
                    key = p + "edge_model.norm."
                    bnc = be.bn2_bwd_coef_part(g_bn_part, se["mu1"], se["var1"], P[key + "weight"],
                                               d.E, self.bn_eps, Gr[key + "weight"],
                                               Gr[key + "bias"])
                elif self.normed:
                    Sg, Sgx = be.edge_bn_grad_sums(d, g_tot, se["y"], *bnstat)
                    bnc = self.edge_bn_coef(P, Gr, d, p + "edge_model.", se, Sg, Sgx)
            g_xe = self.edge_bwd(P, Gr, d, p + "edge_model.", se, g_tot, bnc, b > 0,
                                 g_xs_in, g_xt_in, g_u_in)
            # the block's u[batch] gradients: summed per graph by the next block's
            # class backward, or in one launch before its GlobalModel reads them
            self._gu_flush_list(prev_pend, d.G)
            prev_pend, self._gu_pend = self._gu_pend, []
            g_xs, g_xt, g_u = g_xs_in, g_xt_in, g_u_in
        self._gu_flush_list(prev_pend, d.G)
        s_enc, t_enc = ctx["enc"]
        self.mlp_bwd(P, Gr, "encoder_s.", g_xs, s_enc)
        self.mlp_bwd(P, Gr, "encoder_t.", g_xt, t_enc)

    # ================================================================ loss
    def loss_forward(self, P, d, xe3, ci, sharpness, seed, pclass=0.1, pfiber=0.1, total_time=42.0,
                     nfields=10, wutils=2000.0, wvar=1.0, noiselevel=0.3, want_time=False):
        """train.py:29-80 on the final edge state ``xe3``.  ``ci`` = class_info
        channel-major [>=2, NT] (row 0 = T_i hours per visit, row 1 = N_i)."""
        be = self.be
        y, sc, sh = xe3
        scale = total_time / d.NC                     # TOTAL_TIME/NCLASSES, train.py:42
        dec = [P["decoder_e.0.weight"], P["decoder_e.0.bias"], P["decoder_e.2.weight"], P["decoder_e.2.bias"]]
        n_prime, fiber_time, tmean, tvar, tt = be.loss_fwd(d, y, sc, sh, *dec, ci, scale, sharpness,
                                                          noiselevel, seed, want_time)
        loss, utils, variance, Gn, Gf, Gv = be.loss_finalize(d, n_prime, fiber_time, tvar, ci, pclass,
                                                             pfiber, total_time, nfields, wutils, wvar)
        lctx = dict(d=d, xe3=xe3, ci=ci, scale=scale, sharpness=sharpness, noiselevel=noiselevel,
                    seed=seed, tmean=tmean, Gn=Gn, Gf=Gf, Gv=Gv)
        diag = dict(loss=loss, utils=utils, variance=variance, n_prime=n_prime,
                    fiber_time=fiber_time, time=tt)
        return loss.sum(), diag, lctx

    def loss_bnstat(self, ectx):
        """(mu1, inv1) of the final block's edge BatchNorm when the loss
        backward can make its backward sums (training statistics, complete
        batch, a backend with loss_bwd(bn=...)); else None."""
        blocks = ectx.get("blocks") if ectx is not None else None
        if (not blocks or not self.normed or not ectx.get("training", True)
                or not getattr(self.be, "loss_bn_part", False)
                or os.environ.get("PFSGNN_LOSS_BN_SUMS", "1") == "0"):
            return None
        se = blocks[-1][0]
        if "rm" in se or se.get("inv1") is None:
            return None
        return se["mu1"], se["inv1"]

    def loss_backward(self, P, Gr, lctx, gscale=1.0, bnstat=None):
        """-> gxe (canonical [F, E]); with ``bnstat`` (loss_bnstat) -> (gxe,
        the final edge BatchNorm's backward-sum partials)."""
        be, d = self.be, lctx["d"]
        y, sc, sh = lctx["xe3"]
        dec = [P["decoder_e.0.weight"], P["decoder_e.0.bias"], P["decoder_e.2.weight"], P["decoder_e.2.bias"]]
        kw = {"bn": bnstat} if bnstat is not None else {}
        return be.loss_bwd(d, y, sc, sh, *dec, lctx["ci"], lctx["scale"], lctx["sharpness"],
                           lctx["noiselevel"], lctx["seed"], lctx["Gn"], lctx["Gf"], lctx["Gv"],
                           lctx["tmean"], gscale,
                           Gr["decoder_e.0.weight"], Gr["decoder_e.0.bias"],
                           Gr["decoder_e.2.weight"], Gr["decoder_e.2.bias"], **kw)
