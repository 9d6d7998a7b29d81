"""FusedAdam: ``torch.optim.Adam`` (train.py:111) as one HIP kernel launch.

Same hyper-parameters, update rule (torch/optim/adam.py, amsgrad=False,
maximize=False: exp_avg.lerp_, exp_avg_sq.mul_.addcmul_, bias-corrected
denominator, addcdiv_) and state_dict format as ``torch.optim.Adam``, so a
reference checkpoint's ``optim_state`` loads into it.  When the parameters
are views of one flat buffer (``pfsgnn.GNN`` keeps them so) the whole step is
a single ``pfsgnn_adam`` launch over that buffer.
"""
import torch

from .gnn import backend


def _flat_base(tensors):
    """If `tensors` are views laid out in one storage (possibly with gaps),
    return (base_1d_tensor, [offsets]) covering them; else None."""
    if not tensors:
        return None
    st = tensors[0].untyped_storage()
    if any(t.untyped_storage().data_ptr() != st.data_ptr() or not t.is_contiguous() for t in tensors):
        return None
    offs = [t.storage_offset() for t in tensors]
    lo = min(offs)
    hi = max(o + t.numel() for o, t in zip(offs, tensors))
    base = torch.empty(0, dtype=tensors[0].dtype, device=tensors[0].device)
    base.set_(st, lo, (hi - lo,), (1,))
    return base, [o - lo for o in offs]


def _is_live(p):
    """Whether this step's backward gave p a gradient, as torch.optim.Adam sees
    it (``p.grad is not None``).  pfsgnn's fused backward keeps every
    ``p.grad`` attached to the flat gradient buffer (graph capture) and marks
    the parameters it wrote with ``p._pf_live`` instead (gnn._GradRecorder);
    a gradient accumulated by plain torch autograd (a torch-side term of the
    loss on the weights) sets it too (gnn._mark_live_hook)."""
    live = getattr(p, "_pf_live", None)
    return (p.grad is not None) if live is None else bool(live)


class FusedAdam(torch.optim.Optimizer):
    """``capturable=True`` keeps the step count on the device (as torch's
    capturable Adam does), so ``step()`` issues no host sync and can be
    captured in a HIP graph: each replay increments the count and the kernel
    derives the bias corrections from it.  That count is one per group, so a
    capturable optimizer requires the set of parameters with gradients to stay
    the one of its first step (it raises otherwise).  Without ``capturable``
    every parameter keeps its own step count, as torch.optim.Adam does: a
    parameter without a gradient is skipped (no moment decay, no weight decay,
    no step), and the flat one-launch update runs whenever the live parameters
    share one count (per-parameter launches otherwise)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 capturable=False):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, capturable=capturable)
        super().__init__(params, defaults)
        self._flat = {}
        self._masks = {}
        self._live0 = {}

    def zero_grad(self, set_to_none=True):
        """torch's zero_grad, and every pfsgnn parameter back to 'no gradient
        this step' until a backward writes it (``_pf_live``)."""
        for group in self.param_groups:
            for p in group["params"]:
                if hasattr(p, "_pf_live"):
                    p._pf_live = False
        super().zero_grad(set_to_none=set_to_none)

    def _live_mask(self, gi, group, n, live):
        """Device uint8 mask over the flat buffer, 1 on the parameters in `live`."""
        key = (gi, live)
        m = self._masks.get(key)
        if m is None:
            host = torch.zeros(n, dtype=torch.uint8)
            _, offs = _flat_base([p.detach() for p in group["params"]])
            for p, off, on in zip(group["params"], offs, live):
                if on:
                    host[off:off + p.numel()] = 1
            m = host.to(group["params"][0].device)
            self._masks[key] = m
        return m

    def _group_flat(self, gi, group):
        ps = group["params"]
        pb = _flat_base([p.detach() for p in ps])
        gb = _flat_base([p.grad for p in ps]) if all(p.grad is not None for p in ps) else None
        if pb is None or gb is None or pb[1] != gb[1] or pb[0].numel() != gb[0].numel():
            return None
        cache = self._flat.get(gi)
        if cache is None or cache[0].numel() != pb[0].numel():
            m = torch.zeros_like(pb[0])
            v = torch.zeros_like(pb[0])
            for p, off in zip(ps, pb[1]):
                st = self.state.get(p)
                if st and "exp_avg" in st:
                    m[off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    v[off:off + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
            step = 0
            for p in ps:
                st = self.state.get(p)
                if st and "step" in st:
                    step = int(st["step"])
            if group.get("capturable", False):
                step_t = torch.full((), float(step), dtype=torch.float32, device=pb[0].device)
            else:
                step_t = None
            for p, off in zip(ps, pb[1]):
                st = self.state.get(p)
                own = float(st["step"]) if st and "step" in st else 0.0
                self.state[p] = {"step": step_t if step_t is not None else torch.tensor(own),
                                 "exp_avg": m[off:off + p.numel()].view(p.shape),
                                 "exp_avg_sq": v[off:off + p.numel()].view(p.shape)}
            cache = (m, v)
            self._flat[gi] = cache
        return pb[0], gb[0], cache[0], cache[1]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        be = backend()
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            ps = group["params"]
            flat = self._group_flat(gi, group)
            live = tuple(_is_live(q) for q in ps)
            if flat is not None and group.get("capturable", False):
                p, g, m, v = flat
                first = self._live0.setdefault(gi, live)
                if live != first:
                    raise RuntimeError("FusedAdam(capturable=True) keeps one device step count per "
                                       "group: the set of parameters with gradients must stay the "
                                       "one of the first step")
                # the dead parameters of a fixed live set never had a gradient:
                # zero moments, so a zero-gradient update leaves them unchanged
                # unless weight decay applies
                mask = (None if all(live) or group["weight_decay"] == 0.0
                        else self._live_mask(gi, group, p.numel(), live))
                step_t = self.state[ps[0]]["step"]          # one device tensor shared by the group
                step_t.add_(1.0)
                be.adam(p, g, m, v, step_t, group["lr"], beta1, beta2, group["eps"],
                        group["weight_decay"], live=mask)
                continue
            if flat is not None:
                p, g, m, v = flat
                steps = [int(self.state[q]["step"]) for q in ps]     # host tensors: no sync
                counts = {c for c, on in zip(steps, live) if on}
                if len(counts) <= 1:
                    step = (counts.pop() if counts else 0) + 1
                    # a dead parameter is left exactly as it is (torch skips it)
                    # unless its moments are zero and no weight decay applies
                    need = any(not on and (group["weight_decay"] != 0.0 or c > 0)
                               for c, on in zip(steps, live))
                    mask = self._live_mask(gi, group, p.numel(), live) if need else None
                    be.adam(p, g, m, v, step, group["lr"], beta1, beta2, group["eps"],
                            group["weight_decay"], live=mask)
                    for q, on in zip(ps, live):
                        if on:
                            self.state[q]["step"] = torch.tensor(float(step))
                    continue
            for q in ps:
                if q.grad is None or not _is_live(q):
                    continue
                st = self.state[q]
                if "exp_avg" not in st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(q)
                    st["exp_avg_sq"] = torch.zeros_like(q)
                step = int(st["step"]) + 1
                st["step"].fill_(float(step))
                be.adam(q.detach(), q.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], step,
                        group["lr"], beta1, beta2, group["eps"], group["weight_decay"])
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat = {}   # re-flattened (copying the loaded moments) at the next step
