"""Torch-CPU emulation of the pfsgnn op set (TEST INFRASTRUCTURE ONLY).

The product engine (``pfsgnn/engine.py``) orchestrates a small set of ops that
the HIP library (``libpfsgnn.so``) implements as kernels.  This module
implements the *same* ops, with the same arguments and layouts, in plain
torch so that the orchestration (and every hand-derived backward formula in
it) can be checked against the autograd oracle on the CPU, in float64, with
no GPU.  It is never imported by product code and is not a fallback: the
product backend is chosen explicitly and only ``HipBackend`` exists there.

Layouts (see DESIGN.md §Data layout):
* node tensors are channel-major ``[C, N]``;
* edge tensors are channel-major ``[C, E]`` in the canonical class-major
  order ``e = (g*NC + c)*NF + f`` (train.py's own edge order -- fiber-major
  ``(g*NF + f)*NC + c`` -- is only seen at the boundary: the softfloor noise
  is drawn per fiber-major position and ``tt`` is returned in it);
* weights are torch ``Linear`` matrices ``[out, in]``; an op that uses a
  column block of a weight takes ``(W, col0, ncol)``.
"""
import math

import torch

SLOPE = 0.1


def lrelu(x, s=SLOPE):
    return torch.where(x > 0, x, x * s)


def dlrelu(z, s=SLOPE):
    return torch.where(z > 0, torch.ones_like(z), torch.full_like(z, s))


from pfsgnn.engine import Dims  # noqa: E402,F401  (re-exported for the tests)
from pfsgnn.sparse import SparseEdgeOps, SparseGeo  # noqa: E402


def _edge_index(d, device):
    e = torch.arange(d.E, device=device)
    cls = e // d.NF
    fib = (cls // d.NC) * d.NF + e % d.NF
    return fib, cls


def _user_index(d, device):
    """train.py's fiber-major position of each canonical edge."""
    fib, cls = _edge_index(d, device)
    return fib * d.NC + cls % d.NC


def _seg(x, idx, n):
    """Segment sum of [C, E] (or [E]) over edge -> node index."""
    if x.dim() == 1:
        return torch.zeros(n, dtype=x.dtype, device=x.device).index_add_(0, idx, x)
    return torch.zeros(x.shape[0], n, dtype=x.dtype, device=x.device).index_add_(1, idx, x)


def _aff(x, sc, sh):
    if sc is None:
        return x
    return x * sc[:, None] + sh[:, None]


class EmuBackend:
    name = "emu"
    fiber_bn_sums = True   # target_bwd(bn_sums=...) / mlp_bwd(bn_part=...), as HipBackend
    loss_bn_part = True    # loss_bwd(bn=...) / bn2_bwd_coef_part, as HipBackend

    def __init__(self, dtype=torch.float64):
        self.dtype = dtype
        self.device = torch.device("cpu")
        self._sp = SparseEdgeOps(self)

    def empty(self, *shape):
        return torch.empty(*shape, dtype=self.dtype)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=self.dtype)

    def ones(self, *shape):
        return torch.ones(*shape, dtype=self.dtype)

    # ------------------------------------------------------------ node ops
    def lin(self, W, col0, ncol, X, b=None, act_in=False, out=None, add=False, bscale=1.0):
        Xa = lrelu(X) if act_in else X
        Y = W[:, col0:col0 + ncol] @ Xa
        if b is not None:
            Y = Y + bscale * b[:, None]
        if out is None:
            return Y
        if add:
            out += Y
        else:
            out.copy_(Y)
        return out

    def lin_gather(self, W, col0, ncol, X, gathers, b=None):
        Y = self.lin(W, col0, ncol, X, b=b)
        for G, idx in gathers:
            Y = Y + G[:, idx.long()]
        return Y

    def lin_t(self, W, col0, ncol, dY, z=None, out=None, add=False):
        R = W[:, col0:col0 + ncol].t() @ dY
        if z is not None:
            R = R * dlrelu(z)
        if out is None:
            return R
        if add:
            out += R
        else:
            out.copy_(R)
        return out

    def wgrad(self, dY, X, dW, col0=0, db=None, act_in=False, dbscale=1.0):
        Xa = lrelu(X) if act_in else X
        dW[:, col0:col0 + X.shape[0]] += dY @ Xa.t()
        if db is not None:
            db += dbscale * dY.sum(1)

    def linear_batch(self, ops):
        outs = []
        for op in ops:
            if op[0] == "cat":
                _, W, segs, N, b = op
                outs.append(self.lin_cat(W, segs, N, b=b))
            else:
                _, W, col0, ncol, dY, Y, add = op
                outs.append(self.lin_t(W, col0, ncol, dY, out=Y, add=add))
        return outs

    def defer_begin(self):  # weight-gradient batching is a no-op here
        pass

    def defer_flush(self):
        pass

    @staticmethod
    def _expand(X, bc, N):
        return X.repeat_interleave(N // X.shape[1], dim=1) if bc else X

    def lin_cat(self, W, segs, N, b=None, act_in=False, out=None, add=False, bscale=1.0):
        Y = 0
        for X, col, bc in segs:
            Xa = self._expand(lrelu(X) if act_in else X, bc, N)
            Y = Y + W[:, col:col + X.shape[0]] @ Xa
        if b is not None:
            Y = Y + bscale * b[:, None]
        if out is None:
            return Y
        if add:
            out += Y
        else:
            out.copy_(Y)
        return out

    def wgrad_cat(self, dY, segs, dW, db=None, act_in=False, dbscale=1.0):
        N = dY.shape[1]
        for X, col, bc in segs:
            Xa = self._expand(lrelu(X) if act_in else X, bc, N)
            dW[:, col:col + X.shape[0]] += dY @ Xa.t()
        if db is not None:
            db += dbscale * dY.sum(1)

    def mlp_fwd(self, segs, N, W1, b1, W2, b2, bn=None, save_z=True):
        Z = b1[:, None] + 0
        for X, col, bc in segs:
            Z = Z + W1[:, col:col + X.shape[0]] @ self._expand(X, bc, N)
        Yp = W2 @ lrelu(Z) + b2[:, None]
        if bn is None:
            return Yp, Z, Yp, None, None
        g, bt, rm, rv, mom, eps = bn
        Y, mu, var = self.bn_fwd(Yp, g, bt, rm, rv, mom, eps)
        return Y, Z, Yp, mu, var

    def mlp_fwd_epi(self, segs, N, W1, b1, W2, b2, bn, epi):
        Y, Z, Yp, mu, var = self.mlp_fwd(segs, N, W1, b1, W2, b2, bn=bn)
        O = W2.shape[0]
        outs = [W[:nk, col0:col0 + O] @ Y + (0 if b is None else b[:nk, None])
                for W, col0, nk, b in epi]
        return Y, Z, Yp, mu, var, outs

    def target_global_fwd(self, segs, G, NC, W1, b1, W2, b2, bn, xs, NF, u, gW1, gb1, gW2, gb2,
                          gw, reps, nxt=None):
        xt, Z, Yp, mu, var = self.mlp_fwd(segs, G * NC, W1, b1, W2, b2, bn=bn)
        un, means, gZ, gV, rms = self.global_fwd(xs, xt, u, gW1, gb1, gW2, gb2, gw, reps, G)
        r = dict(Z=Z, Yp=Yp, xt=xt, mu=mu, var=var, means=means, gZ=gZ, gV=gV, u=un, rms=rms,
                 Pt=None, Qt=None)
        if nxt is not None:
            We, be, Ws, bs = nxt
            F = xt.shape[0]
            r["Pt"] = self.lin_cat(We, [(xt, F, False), (un, 3 * F, True)], G * NC, b=be)
            r["Qt"] = self.lin(Ws, 0, F, xt, b=bs)
        return r

    def mlp_bwd(self, dY, Z, W1, W2, K, bn=None, outs=(), bn_part=None, mom_coef=None):
        dYp = dY
        if bn is not None:
            Yp, mu, var, g, eps, dg, db = bn
            sums = None
            if bn_part is not None:   # pfsgnn_mlp_bwd_pre: the producer's per-block partials
                O = dY.shape[0]
                sums = (bn_part[:, :O].sum(0), bn_part[:, 16:16 + O].sum(0))
            dYp = self.bn_bwd(dY, Yp, mu, var, g, eps, dg, db, sums=sums)
        dZ = (W2.t() @ dYp) * dlrelu(Z)
        if outs:
            dX = W1[:, :K].t() @ dZ
            r = 0
            for t, rows, add in outs:
                if t is not None:
                    if add:
                        t += dX[r:r + rows]
                    else:
                        t.copy_(dX[r:r + rows])
                r += rows
            if mom_coef is not None:   # pfsgnn_mlp_bwd_pre's moment epilogue
                mom, coef, k0, n = mom_coef
                C = mom.shape[1]
                coef.copy_(self.moment_coef(mom, dX[k0:k0 + 4 * C], n))
        return dYp, dZ

    def bn_fwd(self, X, gamma, beta, rm, rv, momentum, eps):
        n = X.shape[1]
        mu = X.mean(1)
        var = ((X - mu[:, None]) ** 2).mean(1)
        Y = (X - mu[:, None]) / torch.sqrt(var[:, None] + eps) * gamma[:, None] + beta[:, None]
        if rm is not None:
            rm.mul_(1 - momentum).add_(momentum * mu.to(rm.dtype))
            rv.mul_(1 - momentum).add_(momentum * (var * n / max(n - 1, 1)).to(rv.dtype))
        return Y, mu, var

    def bn_bwd(self, dY, X, mu, var, gamma, eps, dgamma, dbeta, sums=None):
        inv = 1.0 / torch.sqrt(var + eps)
        xh = (X - mu[:, None]) * inv[:, None]
        Sg, Sgx = sums if sums is not None else (dY.sum(1), (dY * xh).sum(1))
        n = X.shape[1]
        dgamma += Sgx
        dbeta += Sg
        return (gamma * inv)[:, None] * (dY - Sg[:, None] / n - xh * (Sgx / n)[:, None])

    def graph_reduce(self, X, G, mean=False, out=None):
        C, N = X.shape
        R = X.reshape(C, G, N // G).sum(2)
        R = R / (N // G) if mean else R
        if out is not None:
            out += R
            return out
        return R

    def graph_reduce_multi(self, Xs, G, out):
        for X in Xs:
            self.graph_reduce(X, G, out=out)
        return out

    def graph_bcast_add(self, out, src, scale=1.0):
        C, N = out.shape
        G = src.shape[1]
        out += (src * scale).repeat_interleave(N // G, dim=1)
        return out

    def graph_mean2(self, X1, X2, G):
        return torch.cat([self.graph_reduce(X1, G, mean=True), self.graph_reduce(X2, G, mean=True)])

    def graph_bcast_add2(self, out1, s1, out2, s2, src):
        C = src.shape[0] // 2
        self.graph_bcast_add(out1, src[:C], s1)
        self.graph_bcast_add(out2, src[C:], s2)

    def global_fwd(self, xs, xt, u, W1, b1, W2, b2, w, eps, G):
        F = u.shape[0]
        means = self.graph_mean2(xs, xt, G)
        V, Z, _, _, _ = self.mlp_fwd([(u, 0, False), (means, F, False)], G, W1, b1, W2, b2)
        if w is None:
            return V, means, Z, V, None
        Y, rms = self.rms2_fwd(V, w, eps)
        return Y, means, Z, V, rms

    def global_bwd(self, dY, V, w, rms, eps, dw, Z, W1, W2, g_u, g_xs, s1, g_xt, s2):
        F, G = V.shape
        gV = dY if w is None else self.rms2_bwd(dY, V, w, rms, eps, dw)
        g_m = self.empty(2 * F, G)
        _, dZ = self.mlp_bwd(gV, Z, W1, W2, 3 * F, outs=[(g_u, F, True), (g_m, 2 * F, False)])
        self.graph_bcast_add2(g_xs, s1, g_xt, s2, g_m)
        return gV, dZ

    def rms2_fwd(self, X, w, eps):
        def one(x):
            r = torch.rsqrt((x * x).mean(0, keepdim=True) + eps)
            return x * r * w[:, None], r
        Y1, r1 = one(X)
        Y2, r2 = one(Y1)
        return Y2, (Y1, r1, r2)

    def rms2_bwd(self, dY, X, w, saved, eps, dw):
        Y1, r1, r2 = saved

        def back(dy, x, r):
            # y = x * r * w,  r = (mean(x^2)+eps)^-1/2
            dw.add_((dy * x * r).sum(1))
            dxn = dy * w[:, None]
            C = x.shape[0]
            return r * dxn - x * (r ** 3) * (dxn * x).sum(0, keepdim=True) / C

        d1 = back(dY, Y1, r2)
        return back(d1, X, r1)

    def bn_eval_coef(self, gamma, beta, rm, rv, eps, times):
        a = gamma / torch.sqrt(rv.to(gamma.dtype) + eps)
        b = beta - rm.to(gamma.dtype) * a
        sc, sh = torch.ones_like(a), torch.zeros_like(a)
        for _ in range(times):
            sc, sh = a * sc, a * sh + b
        return sc, sh

    def affine_rows(self, X, sc, sh):
        return X * sc[:, None] + sh[:, None]

    def bn_eval_bwd_coef(self, gamma, beta, rm, rv, eps, times, Sg=None, Sgx=None, dgamma=None,
                         dbeta=None):
        """pfsgnn_bn_eval_bwd_coef: eval BatchNorm1d (applied ``times`` times)
        backward: -> (inv, scale = a^times); dgamma / dbeta += its parameter
        gradients from Sg = sum g, Sgx = sum g (y - rm) inv."""
        sd = torch.sqrt(rv.to(gamma.dtype) + eps)
        inv, a = 1.0 / sd, gamma / sd
        if Sg is not None:
            if times == 2:
                dgamma += 2 * a * Sgx + inv * (beta - rm.to(gamma.dtype)) * Sg
                dbeta += (a + 1) * Sg
            else:
                dgamma += Sgx
                dbeta += Sg
        return inv, (a * a if times == 2 else a)

    def bn2_finalize(self, mu1, var1, gamma, beta, rm, rv, n, momentum, eps):
        """EdgeModel's BatchNorm applied twice (gnn.py:101 -- ``super().forward``
        already runs ``self.norm`` as the Sequential's last child).  The second
        application sees mean == beta and var == gamma^2 var1/(var1+eps), so
        xe_new = sc*y + sh.  Updates the running stats twice, as the reference's
        two calls do (checkpoint: num_batches_tracked == 2 x epochs)."""
        inv1 = 1.0 / torch.sqrt(var1 + eps)
        rho = var1 * inv1 * inv1
        var2 = gamma * gamma * rho
        inv2 = 1.0 / torch.sqrt(var2 + eps)
        sc = gamma * gamma * inv1 * inv2
        sh = beta - mu1 * sc
        if rm is not None:
            f = n / max(n - 1, 1)
            rm.mul_(1 - momentum).add_(momentum * mu1.to(rm.dtype))
            rv.mul_(1 - momentum).add_(momentum * (var1 * f).to(rv.dtype))
            rm.mul_(1 - momentum).add_(momentum * beta.to(rm.dtype))
            rv.mul_(1 - momentum).add_(momentum * (var2 * f).to(rv.dtype))
        return sc, sh, inv1, inv2

    def bn2_bwd_coef_part(self, part, mu1, var1, gamma, n, eps, dgamma, dbeta):
        C = mu1.shape[0]
        S = part.sum(0)
        return self.bn2_bwd_coef(S[:C], S[C:], mu1, var1, gamma, n, eps, dgamma, dbeta)

    def bn2_bwd_coef(self, Sg, Sgx, mu1, var1, gamma, n, eps, dgamma, dbeta):
        """Backward of the double BatchNorm as g_y = alpha*g + gam0 + gam1*y."""
        inv1 = 1.0 / torch.sqrt(var1 + eps)
        rho = var1 * inv1 * inv1
        inv2 = 1.0 / torch.sqrt(gamma * gamma * rho + eps)
        k = gamma * inv2
        M = Sgx / n
        alpha = gamma * inv1 * k
        gam1 = -alpha * M * (k * k + 1 - k * k * rho) * inv1
        gam0 = -alpha * Sg / n - gam1 * mu1
        dgamma += k * Sgx * (2 - k * k * rho)
        dbeta += Sg
        return alpha, gam0, gam1

    def moment_coef(self, mom, gst, n):
        if isinstance(n, torch.Tensor):          # general graph: fiber CSR pointer
            n = (n[1:] - n[:-1]).clamp(min=1).to(mom.dtype)
        """SModel moment backward (gnn.py:140-153) as per-fiber coefficients of
        g_m = C0 + d*(C1 + d*(C2 + d*C3)), d = m - mean.  gst = d(loss)/d
        [mean; std; skew; kurt] ([8F, NS])."""
        mean, c2, c3, c4 = mom
        C = mean.shape[0]
        gmean, gstd, gskew, gkurt = gst[0:C], gst[C:2 * C], gst[2 * C:3 * C], gst[3 * C:4 * C]
        var = torch.where(c2 > 0, c2, 0.01 * c2)
        std = torch.sqrt(var + 1e-6)
        A3 = gskew / std ** 3
        A4 = gkurt / std ** 4
        gstd_tot = gstd - 3 * gskew * c3 / std ** 4 - 4 * gkurt * c4 / std ** 5
        gvr = gstd_tot / (2 * std) * torch.where(c2 > 0, torch.ones_like(c2), torch.full_like(c2, 0.01))
        return torch.stack([(gmean - 3 * c2 * A3 - 4 * c3 * A4) / n, 2 * gvr / n, 3 * A3 / n, 4 * A4 / n])

    # ------------------------------------------------------------ edge ops
    def edge_mlp_fwd(self, d, xe, xsc, xsh, Ps, Pt, W1, W2, b2):
        if d.sp is not None:
            return self._sp.edge_mlp_fwd(d, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
        fib, cls = _edge_index(d, xe.device)
        F = d.F
        x = _aff(xe, xsc, xsh)
        z1 = Ps[:, fib] + Pt[:, cls] + W1[:, 2 * F:3 * F] @ x
        y = W2 @ lrelu(z1) + b2[:, None]
        mu = y.mean(1)
        var = ((y - mu[:, None]) ** 2).mean(1)
        return y, mu, var

    def edge_mlp_fwd_bn(self, d, xe, xsc, xsh, Ps, Pt, W1, W2, b2, bn):
        gamma, beta, rm, rv, momentum, eps = bn
        y, mu, var = self.edge_mlp_fwd(d, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
        sc, sh, inv1, _ = self.bn2_finalize(mu, var, gamma, beta, rm, rv, d.E, momentum, eps)
        return y, mu, var, sc, sh, inv1

    def source_fwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_out):
        """Per-fiber centred moments of the SModel message (gnn.py:136-151).
        Returns mom [4, 2F, NS] = (mean, c2, c3, c4); writes the MLP inputs
        (mean, std, skew, kurt) into hs_out [8F, NS]."""
        if d.sp is not None:
            return self._sp.source_fwd(d, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_out)
        fib, cls = _edge_index(d, y.device)
        F = d.F
        x = _aff(y, sc, sh)
        zs = Qt[:, cls] + Ws1[:, F:2 * F] @ x
        m = Ws2 @ lrelu(zs) + bs2[:, None]
        C = 2 * F
        mean = _seg(m, fib, d.NS) / d.NC
        dd = m - mean[:, fib]
        c2 = _seg(dd ** 2, fib, d.NS) / d.NC
        c3 = _seg(dd ** 3, fib, d.NS) / d.NC
        c4 = _seg(dd ** 4, fib, d.NS) / d.NC
        var = torch.where(c2 > 0, c2, 0.01 * c2)
        std = torch.sqrt(var + 1e-6)
        hs_out[0:C] = mean
        hs_out[C:2 * C] = std
        hs_out[2 * C:3 * C] = c3 / std ** 3
        hs_out[3 * C:4 * C] = c4 / std ** 4
        return torch.stack([mean, c2, c3, c4])

    def target_fwd(self, d, y, sc, sh, Rs, Wt1, agg=None):
        hsum = self._target_fwd(d, y, sc, sh, Rs, Wt1)
        if agg is None:
            return hsum
        Wt2, bt2, bscale = agg
        return hsum, self.lin(Wt2, 0, Wt2.shape[1], hsum, b=bt2, bscale=bscale)

    def _target_fwd(self, d, y, sc, sh, Rs, Wt1):
        if d.sp is not None:
            return self._sp.target_fwd(d, y, sc, sh, Rs, Wt1)
        fib, cls = _edge_index(d, y.device)
        F = d.F
        x = _aff(y, sc, sh)
        zt = Rs[:, fib] + Wt1[:, F:2 * F] @ x
        at = lrelu(zt)
        return _seg(at, cls, d.NT)

    def target_bwd(self, d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=False, g_xs=None,
                   bn_sums=None):
        out = self._target_bwd(d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=want_gxe)
        if g_xs is not None:
            self.lin_t(Wt1, 0, d.F, out[0], out=g_xs, add=True)
        if bn_sums is not None:   # pfsgnn_target_bwd_bn: per-64-fiber partials [nb][32]
            Yp, mu, var, eps = bn_sums
            O, NS = g_xs.shape
            xh = (Yp - mu[:, None]) / torch.sqrt(var[:, None] + eps)
            nb = (NS + 63) // 64
            part = torch.zeros(nb, 32, dtype=g_xs.dtype, device=g_xs.device)
            pad = nb * 64 - NS
            gp = torch.nn.functional.pad(g_xs, (0, pad)).reshape(O, nb, 64)
            xp = torch.nn.functional.pad(g_xs * xh, (0, pad)).reshape(O, nb, 64)
            part[:, :O] = gp.sum(2).t()
            part[:, 16:16 + O] = xp.sum(2).t()
            return out[0], out[1], part
        return out

    def _target_bwd(self, d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=False):
        if d.sp is not None:
            return self._sp.target_bwd(d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=want_gxe)
        fib, cls = _edge_index(d, y.device)
        F = d.F
        x = _aff(y, sc, sh)
        zt = Rs[:, fib] + Wt1[:, F:2 * F] @ x
        gz = g_hsum[:, cls] * dlrelu(zt)
        GzT = _seg(gz, fib, d.NS)
        dWt1[:, F:2 * F] += gz @ x.t()
        gxe = Wt1[:, F:2 * F].t() @ gz if want_gxe else None
        return GzT, gxe

    def source_bwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next,
                   bnstat, dWs1, dWs2, dbs2, bn2=None, g_xt=None):
        out = self._source_bwd(d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next,
                               bnstat, dWs1, dWs2, dbs2)
        if g_xt is not None:
            self.lin_t(Ws1, 0, d.F, out[1], out=g_xt, add=True)
        if bn2 is None:
            return out
        gamma, var1, n, eps, dg, db = bn2
        cf = self.bn2_bwd_coef(out[2], out[3], bnstat[0], var1, gamma, n, eps, dg, db)
        return out[0], out[1], None, None, cf

    def _source_bwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next,
                    bnstat, dWs1, dWs2, dbs2):
        """Returns (g_tot [F,E], GzS [2F, NT], Sg, Sgx).  ``coef`` = [4, 2F, NS]
        (C0..C3 of g_m = C0 + d*(C1 + d*(C2 + d*C3)), d = m - mean)."""
        if d.sp is not None:
            return self._sp.source_bwd(d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next, bnstat, dWs1, dWs2, dbs2)
        fib, cls = _edge_index(d, y.device)
        F = d.F
        x = _aff(y, sc, sh)
        zs = Qt[:, cls] + Ws1[:, F:2 * F] @ x
        a = lrelu(zs)
        m = Ws2 @ a + bs2[:, None]
        dd = m - mean[:, fib]
        gm = coef[0][:, fib] + dd * (coef[1][:, fib] + dd * (coef[2][:, fib] + dd * coef[3][:, fib]))
        dWs2 += gm @ a.t()
        dbs2 += gm.sum(1)
        gz = (Ws2.t() @ gm) * dlrelu(zs)
        dWs1[:, F:2 * F] += gz @ x.t()
        g = Ws1[:, F:2 * F].t() @ gz
        GzS = _seg(gz, cls, d.NT)
        if tpart is not None:
            Rs, Wt1, g_hsum = tpart
            zt = Rs[:, fib] + Wt1[:, F:2 * F] @ x
            gzt = g_hsum[:, cls] * dlrelu(zt)
            g = g + Wt1[:, F:2 * F].t() @ gzt
        if g_next is not None:
            g = g + g_next
        Sg = Sgx = None
        if bnstat is not None:
            mu1, inv1 = bnstat
            xh = (y - mu1[:, None]) * inv1[:, None]
            Sg = g.sum(1)
            Sgx = (g * xh).sum(1)
        return g, GzS, Sg, Sgx

    def edge_bn_grad_sums(self, d, g, y, mu1, inv1):
        if d.sp is not None:
            return self._sp.edge_bn_grad_sums(d, g, y, mu1, inv1)
        xh = (y - mu1[:, None]) * inv1[:, None]
        return g.sum(1), (g * xh).sum(1)

    def edge_mlp_bwd(self, d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2,
                     dW1, dW2, db2, want_gxe=True, nodes=None):
        out = self._edge_mlp_bwd(d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2,
                                 dW1, dW2, db2, want_gxe=want_gxe)
        if nodes is None:
            return out
        F = d.F
        self.lin_t(W1, 0, F, out[1], out=nodes[0], add=True)
        self.lin_t(W1, F, F, out[2], out=nodes[1], add=True)
        return out + (self.lin_t(W1, 3 * F, F, out[2]),)

    def _edge_mlp_bwd(self, d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2,
                      dW1, dW2, db2, want_gxe=True):
        if d.sp is not None:
            return self._sp.edge_mlp_bwd(d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2, dW1, dW2, db2, want_gxe=want_gxe)
        fib, cls = _edge_index(d, y.device)
        F = d.F
        gy = alpha[:, None] * g_tot + gam0[:, None] + gam1[:, None] * y
        x = _aff(xe, xsc, xsh)
        z1 = Ps[:, fib] + Pt[:, cls] + W1[:, 2 * F:3 * F] @ x
        a1 = lrelu(z1)
        dW2 += gy @ a1.t()
        db2 += gy.sum(1)
        gz = (W2.t() @ gy) * dlrelu(z1)
        dW1[:, 2 * F:3 * F] += gz @ x.t()
        GzEs = _seg(gz, fib, d.NS)
        GzEt = _seg(gz, cls, d.NT)
        gxe = W1[:, 2 * F:3 * F].t() @ gz if want_gxe else None
        return gxe, GzEs, GzEt

    def edge_apply(self, d, y, sc, sh):
        if d.sp is not None:
            return self._sp.edge_apply(d, y, sc, sh)
        return _aff(y, sc, sh).clone()

    # ------------------------------------------------------------ loss ops
    def loss_fwd(self, d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel, seed,
                 want_time=False):
        """train.py:42-49 per edge, reduced per class / fiber.  ``uni`` [E] are the
        uniforms of softfloor's noise.  Returns n_prime [NT], fiber_time [NS],
        tt_mean [NT], tt_var [NT] (unbiased over fibers), tt [E]."""
        fib, cls = _edge_index(d, y.device)
        eu = _user_index(d, y.device)
        uni = self.noise_uniform(seed, d.E)[eu]
        x = _aff(y, sc, sh)
        zd = Wd1 @ x + bd1[:, None]
        pred = (Wd2 @ lrelu(zd) + bd2[:, None])[0]
        time = torch.nn.functional.softplus(pred) * scale
        Ti = ci[0][cls]
        v = time / Ti + noiselevel * (uni - 0.5)
        r = 0.0 if sharpness == 0 else math.exp(-1.0 / sharpness)
        th = 2 * math.pi * v
        gal = v + (torch.atan(r * torch.sin(th) / (1 - r * torch.cos(th))) - math.atan(r / (1 - r))) / math.pi
        gal = torch.clamp(gal, min=0.0)
        tt = gal * Ti
        n_prime = _seg(gal, cls, d.NT)
        fiber_time = _seg(tt, fib, d.NS)
        tmean = _seg(tt, cls, d.NT) / d.NF
        tvar = _seg((tt - tmean[cls]) ** 2, cls, d.NT) / (d.NF - 1)
        tt_user = None
        if want_time:
            tt_user = torch.empty_like(tt)
            tt_user[eu] = tt
        return n_prime, fiber_time, tmean, tvar, tt_user

    def loss_bwd(self, d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel, seed,
                 Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2, dbd2, bn=None):
        gxe = self._loss_bwd(d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel,
                             seed, Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2, dbd2)
        if bn is None:
            return gxe
        # the HIP kernel's per-block partials, here as two halves of the edges
        h = d.E // 2
        parts = [self.edge_bn_grad_sums(d, gxe[:, a:b], y[:, a:b], *bn)
                 for a, b in ((0, h), (h, d.E))]
        return gxe, torch.stack([torch.cat(p) for p in parts])

    def _loss_bwd(self, d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel, seed,
                  Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2, dbd2):
        fib, cls = _edge_index(d, y.device)
        uni = self.noise_uniform(seed, d.E)[_user_index(d, y.device)]
        Gn, Gf, Gv = Gn * gscale, Gf * gscale, Gv * gscale
        x = _aff(y, sc, sh)
        zd = Wd1 @ x + bd1[:, None]
        ad = lrelu(zd)
        pred = (Wd2 @ ad + bd2[:, None])[0]
        time = torch.nn.functional.softplus(pred) * scale
        Ti = ci[0][cls]
        v = time / Ti + noiselevel * (uni - 0.5)
        r = 0.0 if sharpness == 0 else math.exp(-1.0 / sharpness)
        th = 2 * math.pi * v
        graw = v + (torch.atan(r * torch.sin(th) / (1 - r * torch.cos(th))) - math.atan(r / (1 - r))) / math.pi
        gal = torch.clamp(graw, min=0.0)
        tt = gal * Ti
        g_tt = Gf[fib] + Gv[cls] * (tt - tmean[cls])
        g_gal = Gn[cls] + Ti * g_tt
        mask = torch.where(graw > 0, torch.ones_like(graw),
                           torch.where(graw == 0, torch.full_like(graw, 0.5), torch.zeros_like(graw)))
        dsf = 1 + 2 * (r * torch.cos(th) - r * r) / (1 - 2 * r * torch.cos(th) + r * r)
        g_time = g_gal * mask * dsf / Ti
        sig = torch.where(pred > 20, torch.ones_like(pred), torch.sigmoid(pred))
        g_pred = g_time * scale * sig
        dWd2 += (g_pred[None, :] @ ad.t())
        dbd2 += g_pred.sum().reshape(1)
        gz = (Wd2.t() @ g_pred[None, :]) * dlrelu(zd)
        dWd1 += gz @ x.t()
        dbd1 += gz.sum(1)
        return Wd1.t() @ gz

    def loss_finalize(self, d, n_prime, fiber_time, tvar, ci, pclass, pfiber, total_time,
                      nfields, wutils, wvar, gscale=1.0):
        """train.py:53-71 per graph.  Returns loss [G], utils [G], variance [G] and
        the per-node gradient coefficients Gn [NT], Gf [NS], Gv [NT] of the loss
        (scaled by ``gscale``)."""
        G, NC, NF = d.G, d.NC, d.NF
        Ni = (ci[1] / nfields).reshape(G, NC)
        npr = n_prime.reshape(G, NC)
        comp = npr / Ni
        utils = comp.min(1).values
        ties = (comp == utils[:, None]).to(comp.dtype)
        share = ties / ties.sum(1, keepdim=True)
        over = torch.relu(npr - Ni)
        cpen = pclass * (over ** 2).sum(1)
        ot = fiber_time.reshape(G, NF) - total_time
        lk = lrelu(ot)
        fpen = pfiber * (lk ** 2).sum(1)
        variance = tvar.reshape(G, NC).sum(1)
        loss = -wutils * utils + fpen + cpen - wvar * variance
        Gn = gscale * (-wutils * share / Ni + 2 * pclass * over)
        Gf = gscale * pfiber * 2 * lk * dlrelu(ot)
        Gv = torch.full_like(tvar, gscale * (-wvar) * 2.0 / (NF - 1))
        return loss, utils, variance, Gn.reshape(-1), Gf.reshape(-1), Gv

    # ------------------------------------------------------------ layout
    # (emulation of pfsgnn_layout_analyze / pfsgnn_edges_{to,from}_canonical:
    # perm[i] = canonical index of the caller's edge i)
    def layout_analyze(self, edge_index, G, NF, NC):
        src, tgt = edge_index[0].long().cpu(), edge_index[1].long().cpu()
        g = src // NF
        ok = bool(((tgt // NC) == g).all()) and bool((src < G * NF).all())
        perm = (g * NC + tgt % NC) * NF + src % NF
        E = G * NF * NC
        complete = ok and perm.numel() == E and torch.equal(torch.sort(perm).values, torch.arange(E))
        fm = torch.equal(perm, self._fm_perm(G, NF, NC)) if complete else False
        ident = torch.equal(perm, torch.arange(E)) if complete else False
        return perm, complete, fm, ident

    @staticmethod
    def _fm_perm(G, NF, NC):
        i = torch.arange(G * NF * NC)
        g, f, c = i // (NF * NC), (i // NC) % NF, i % NC
        return (g * NC + c) * NF + f

    def _perm_of(self, lay):
        sp = getattr(lay, "sp", None)
        if sp is not None:                     # general graph: caller edge -> position
            inv = torch.empty_like(sp.user_of)
            inv[sp.user_of] = torch.arange(sp.E)
            return inv
        if lay.mode == 2:                      # Layout.CANONICAL
            return torch.arange(lay.G * lay.NF * lay.NC)
        if lay.mode == 1:                      # Layout.FIBER_MAJOR
            return self._fm_perm(lay.G, lay.NF, lay.NC)
        return lay.perm

    def edges_to_canonical(self, x, lay):
        out = torch.zeros(x.shape[1], x.shape[0], dtype=self.dtype)
        out[:, self._perm_of(lay)] = x.to(self.dtype).t()
        return out

    def edges_from_canonical(self, y, sc, sh, lay, rowmajor=True):
        u = _aff(y, sc, sh)[:, self._perm_of(lay)]
        return u.t().contiguous() if rowmajor else u.contiguous()

    # ------------------------------------------------------------ general graphs
    # (emulation of pfsgnn_sparse_layout and the primitives of pfsgnn.sparse)
    def sparse_layout(self, edge_index, G, NF, NC):
        src, tgt = edge_index[0].long().cpu(), edge_index[1].long().cpu()
        E = src.numel()
        if not (bool((src >= 0).all()) and bool((src < G * NF).all()) and bool((tgt >= 0).all())
                and bool((tgt < G * NC).all()) and bool(((src // NF) == (tgt // NC)).all())):
            raise ValueError("edge_index has an edge out of range or joining nodes of different graphs")
        user_of = torch.sort(src, stable=True).indices
        src_p, tgt_p = src[user_of], tgt[user_of]
        cls_ord = torch.sort(tgt_p, stable=True).indices
        fib_ptr = torch.searchsorted(src_p, torch.arange(G * NF + 1))
        cls_ptr = torch.searchsorted(tgt_p[cls_ord], torch.arange(G * NC + 1))
        deg_t = (cls_ptr[1:] - cls_ptr[:-1]).to(self.dtype).reshape(1, -1)
        return SparseGeo(E, src_p, tgt_p, user_of, fib_ptr, cls_ord, cls_ptr, deg_t)

    def gather_cols(self, X, idx, mode=0, out=None, Z=None):
        v = X[:, idx.long()]
        if mode == 2:
            v = v * dlrelu(Z)
        if out is None:
            return v
        if mode == 1:
            out += v
        else:
            out.copy_(v)
        return out

    def segment_sum(self, X, ord, ptr, nseg, act=False, out=None, add=False):
        C, E = X.shape
        cnt = (ptr[1:] - ptr[:-1]).long()
        seg = torch.repeat_interleave(torch.arange(nseg), cnt)
        pos = torch.arange(E) if ord is None else ord.long()
        r = _seg((lrelu(X) if act else X)[:, pos], seg, nseg)
        if out is None:
            return r
        if add:
            out += r
        else:
            out.copy_(r)
        return out

    def segment_moments(self, M, ptr, nseg, hs_out):
        C, E = M.shape
        cnt = (ptr[1:] - ptr[:-1]).long()
        seg = torch.repeat_interleave(torch.arange(nseg), cnt)
        n = cnt.clamp(min=1).to(M.dtype)
        mean = _seg(M, seg, nseg) / n
        dd = M - mean[:, seg]
        c2 = _seg(dd ** 2, seg, nseg) / n
        c3 = _seg(dd ** 3, seg, nseg) / n
        c4 = _seg(dd ** 4, seg, nseg) / n
        var = torch.where(c2 > 0, c2, 0.01 * c2)
        std = torch.sqrt(var + 1e-6)
        hs_out[0:C] = mean
        hs_out[C:2 * C] = std
        hs_out[2 * C:3 * C] = c3 / std ** 3
        hs_out[3 * C:4 * C] = c4 / std ** 4
        return torch.stack([mean, c2, c3, c4])

    def segment_moment_grad(self, M, seg, mean, coef):
        seg = seg.long()
        dd = M - mean[:, seg]
        return coef[0][:, seg] + dd * (coef[1][:, seg] + dd * (coef[2][:, seg] + dd * coef[3][:, seg]))

    def rows_stats(self, X):
        mu = X.mean(1)
        return mu, ((X - mu[:, None]) ** 2).mean(1)

    def rows_bn_sums(self, g, y, mu, inv):
        xh = (y - mu[:, None]) * inv[:, None]
        return g.sum(1), (g * xh).sum(1)

    def rows_axpby(self, g, y, alpha, gam1, gam0, out=None):
        r = alpha[:, None] * g + gam1[:, None] * y + gam0[:, None]
        if out is None:
            return r
        out.copy_(r)
        return out

    # ------------------------------------------------------------ optimizer
    def adam(self, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, live=None):
        """pfsgnn_adam (pfsgnn_node.hip k_adam) restated: torch.optim.Adam's
        device update in the tensors' dtype (its fused multiply-adds as one
        rounding each), bias corrections in double
        (from the host int ``step``, or the already incremented count in a
        0-d tensor: the capturable form), elements with live == 0 untouched."""
        st = float(step) if isinstance(step, torch.Tensor) else float(int(step))
        bc1 = 1.0 - beta1 ** st
        bc2 = 1.0 - beta2 ** st
        dt = p.dtype

        def sc(x):   # a double scalar rounded once to the tensors' dtype
            return torch.tensor(x, dtype=torch.float64).to(dt)

        def fma(a, b, c):   # a*b + c rounded once (exact product in float64)
            return (a.double() * b.double() + c.double()).to(dt)

        gi = g if weight_decay == 0.0 else fma(sc(weight_decay), p, g)
        mi = fma(sc(1.0 - beta1), gi - m, m)
        vi = fma(sc(1.0 - beta2), gi * gi, v * sc(beta2))
        pi = fma(sc(-(lr / bc1)), mi / (torch.sqrt(vi) / sc(math.sqrt(bc2)) + sc(eps)), p)
        if live is not None:
            keep = live.reshape(p.shape) != 0
            mi, vi, pi = (torch.where(keep, a, b) for a, b in ((mi, m), (vi, v), (pi, p)))
        m.copy_(mi)
        v.copy_(vi)
        p.copy_(pi)

    # ------------------------------------------------------------ misc
    def noise_uniform(self, seed, E):
        from noise_ref import uniform_numpy
        return torch.as_tensor(uniform_numpy(seed, E), dtype=self.dtype)
