"""Drop-in operator surface of the reference ``src/gnn.py`` on the HIP engine.

Same classes, constructor signatures, forward signatures and state_dict keys
as the reference (``BipartiteData`` gnn.py:7, ``Loader`` :49, ``MLP`` :65,
``EdgeModel`` :73, ``SModel`` :104, ``TModel`` :157, ``GlobalModel`` :195,
``Block`` :226, ``GNN`` :261), so a reference checkpoint loads with
``load_state_dict`` and a reference training script runs unchanged apart from
the import.  Every forward and backward is computed by ``libpfsgnn.so``
through ``pfsgnn.engine``; PyTorch only allocates, streams and runs autograd's
bookkeeping.

Edge layout: the kernels run on the canonical class-major order
``(g*NC + c)*NF + f`` of a batch of complete bipartite graphs (one wavefront
lane per fiber, one class per wave iteration; DESIGN.md §Data layout).
``edge_index`` may list the edges in any order; it is validated on the device
once (cached per tensor).  train.py's fiber-major order ((g*NF + f)*NC + c,
train.py:94) is mapped arithmetically; any other order (``graphs/graph-0.pt``:
each fiber's classes come out of an unstable argsort) through a permutation.
Results are always reported in the caller's edge order.
Any other edge_index (ragged degrees, missing or repeated pairs) runs on the
general-graph path (pfsgnn.sparse: CSR by fiber / class, DESIGN.md §General
graphs); edges that leave their graph are rejected loudly.

Batching: G graphs collated PyG-style (``Batch.from_data_list``, increments
from ``BipartiteData.__inc__``) with ``x_u`` of shape [G, F]; ``u[g]`` is
broadcast to the edges / nodes of graph g and the GlobalModel means are
per graph.  With G == 1 this is exactly the reference.
"""
import os
import weakref

import torch

from . import config
from .engine import Dims, Engine
from .native import HipBackend

_BACKEND = None


def backend():
    global _BACKEND
    if _BACKEND is None:
        _BACKEND = HipBackend()
    return _BACKEND


# ====================================================================== data
class BipartiteData:
    """gnn.py:7-47 without torch_geometric: same attributes and __inc__."""

    def __init__(self, edge_index=None, x_s=None, x_t=None, x_e=None, x_u=None):
        dev = config.device
        self.edge_index = edge_index.to(dev) if edge_index is not None else None
        self.x_s = x_s.to(dev) if x_s is not None else None
        self.x_t = x_t.to(dev) if x_t is not None else None
        if x_t is not None:
            self.num_nodes = len(self.x_t)
        self.x_e = x_e.to(dev) if x_e is not None else None
        self.x_u = x_u.to(dev) if x_u is not None else None

    def __inc__(self, key, value, *args):
        if key == "edge_index":
            return torch.tensor([[self.x_s.size(0)], [self.x_t.size(0)]], device=self.edge_index.device)
        return 0

    @property
    def num_graphs(self):
        return 1 if self.x_u is None else int(self.x_u.size(0))

    def to(self, device):
        out = BipartiteData.__new__(BipartiteData)
        for k, v in self.__dict__.items():
            setattr(out, k, v.to(device) if isinstance(v, torch.Tensor) else v)
        return out

    def keys(self):
        return [k for k in ("edge_index", "x_s", "x_t", "x_e", "x_u") if getattr(self, k) is not None]


class Batch:
    @staticmethod
    def from_data_list(graphs):
        """PyG-style collation (torch_geometric.data.Batch) using __inc__."""
        ei, xs, xt, xe, xu = [], [], [], [], []
        inc = None
        for g in graphs:
            e = g.edge_index if inc is None else g.edge_index + inc
            ei.append(e)
            step = g.__inc__("edge_index", g.edge_index)
            inc = step if inc is None else inc + step
            xs.append(g.x_s)
            xt.append(g.x_t)
            xe.append(g.x_e)
            xu.append(g.x_u)
        return BipartiteData(torch.cat(ei, 1), torch.cat(xs), torch.cat(xt), torch.cat(xe), torch.cat(xu))


class Loader(torch.utils.data.Dataset):
    """gnn.py:49-63."""

    def __init__(self, graphs_list=None):
        self.graphs_list = graphs_list

    def __len__(self):
        return len(self.graphs_list)

    def __getitem__(self, idx):
        return self.graphs_list[idx]


# ==================================================================== layout
class _TensorCache:
    """Results cached per live tensor OBJECT and its in-place version counter.

    Keys are ``id(tensor)`` plus a weak reference that must still resolve to
    that same object: a freed tensor whose address (or id) the allocator hands
    to a new tensor never hits a stale entry, and an in-place write bumps
    ``_version`` and misses.  (Keying on ``data_ptr`` would silently reuse
    the previous batch's layout or features whenever the caching allocator
    recycles a block of the same size.)"""

    def __init__(self, cap):
        self.cap = cap
        self.d = {}

    def get(self, t, extra):
        e = self.d.get(id(t))
        if e is None:
            return None
        ref, ver, ex, val = e
        if ref() is not t or ver != t._version or ex != extra:
            return None
        return val

    def put(self, t, extra, val):
        if len(self.d) >= self.cap:
            self.d = {k: e for k, e in self.d.items() if e[0]() is not None}
            if len(self.d) >= self.cap:
                self.d.clear()
        self.d[id(t)] = (weakref.ref(t), t._version, extra, val)

    def clear(self):
        self.d.clear()


_LAYOUT_CACHE = _TensorCache(32)
_EDGE_CACHE = _TensorCache(4)


class Layout:
    """How the caller's edge order maps onto the kernels' edge order (the
    ``mode`` argument of pfsgnn_edges_{to,from}_canonical).  A general batch
    (``sp`` set) is a PERM layout over its E positions (G=1, NF=E, NC=1 in the
    ABI's terms) whose permutation is the position -> caller-edge map."""
    PERM, FIBER_MAJOR, CANONICAL = 0, 1, 2
    SLOTS = 3   # a sliced general batch: positions of native.SlicedLayout (pos_user)

    def __init__(self, G, NF, NC, mode, perm=None, fiber_major=False, sp=None):
        self.G, self.NF, self.NC, self.mode = G, NF, NC, mode
        self.perm = perm if mode == Layout.PERM else None
        self.fiber_major = fiber_major    # caller order == train.py's positional order
        self.sp = sp


def sliced_on():
    return os.environ.get("PFSGNN_SLICED", "1") != "0"


def sliced_ok(NC, F):
    """General batches run on the fused sliced kernels (pfsgnn_sliced.hip) when
    the current edge path has them at this Fdim and their class tables fit the
    LDS (``pfsgnn_sliced_max_nc``: at most 128 classes per graph, 124 at Fdim
    16; none on the bf16 edge-state paths), unless PFSGNN_SLICED=0 (the
    composed ops of pfsgnn.sparse)."""
    be = backend()
    if not (sliced_on() and F in (8, 10, 16) and hasattr(be, "sliced_layout")):
        return False
    return NC <= be.sliced_max_nc(F)


def geometry(x_s, x_t, x_u, edge_index, F):
    """(Dims, Layout) for a batch: complete bipartite graphs run on the fused
    edge kernels; any other edge_index (gnn.py:7-47 takes one) on the general
    path (pfsgnn.sparse), laid out once per edge_index tensor."""
    G = 1 if x_u is None else int(x_u.size(0))
    S, T = int(x_s.size(0)), int(x_t.size(0))
    if S % G or T % G:
        raise ValueError(f"x_s ({S}) / x_t ({T}) rows are not a multiple of the {G} graphs in x_u")
    NF, NC = S // G, T // G
    E = int(edge_index.size(1))
    if E == 0:
        raise ValueError("edge_index has no edges")
    key = (E, G, NF, NC)
    hit = _LAYOUT_CACHE.get(edge_index, key)
    if hit is not None and hit.sp is not None and (hit.sp.sl is not None) != sliced_ok(NC, F):
        # a general batch's sliced / composed choice follows Fdim and the edge
        # path (sliced_ok): a layout made under another choice is remade
        hit = None
    if hit is None:
        complete = False
        if E == G * NF * NC:
            perm, complete, fm, identity = backend().layout_analyze(edge_index, G, NF, NC)
        if complete:
            mode = Layout.CANONICAL if identity else (Layout.FIBER_MAJOR if fm else Layout.PERM)
            hit = Layout(G, NF, NC, mode, perm, fiber_major=fm)
        else:
            sp = backend().sparse_layout(edge_index, G, NF, NC)
            if sliced_ok(NC, F):
                # the fused general-graph kernels (pfsgnn_sliced.hip)
                sp.sl = backend().sliced_layout(sp, G, NF, NC)
                hit = Layout(1, E, 1, Layout.SLOTS, sp.sl.pos_user, sp=sp)
            else:
                hit = Layout(1, E, 1, Layout.PERM, sp.user_of, sp=sp)
        _LAYOUT_CACHE.put(edge_index, key, hit)
    return Dims(G, NF, NC, F, sp=hit.sp), hit


def edges_in(x_e, lay, cache=False):
    """User edge features [E, F] -> canonical channel-major [F, E]."""
    if (lay.mode == Layout.CANONICAL and x_e.dtype == torch.float32 and x_e.is_cuda
            and x_e.t().is_contiguous()):
        return x_e.t()
    key = (tuple(x_e.shape), lay)      # the Layout object itself (identity compare)
    if cache:
        hit = _EDGE_CACHE.get(x_e, key)
        if hit is not None:
            return hit
    out = backend().edges_to_canonical(x_e, lay)
    if cache:
        _EDGE_CACHE.put(x_e, key, out)
    return out


def edges_out(xe3, lay, d):
    """Canonical (y, sc, sh) -> user edge tensor [E, F] in the caller's order."""
    be = backend()
    y, sc, sh = xe3
    if lay.mode == Layout.CANONICAL:
        return be.edge_apply(d, y, sc, sh).t()
    return be.edges_from_canonical(y, sc, sh, lay, rowmajor=True)


def is_zero_grad(g):
    """The placeholder gradient of a fused consumer that handed its canonical
    gradient over directly (``train._LossFn``): an expanded zero scalar."""
    return g is not None and g.dim() == 2 and g.stride() == (0, 0)


def grad_edges_in(g, lay):
    """Gradient w.r.t. a user edge tensor [E, F] -> canonical [F, E]."""
    if g is None or is_zero_grad(g):
        return None
    if lay.mode == Layout.CANONICAL and g.t().is_contiguous():
        return g.t()
    return backend().edges_to_canonical(g.contiguous(), lay)


def grad_edges_out(gc, lay):
    if gc is None:
        return None
    if lay.mode == Layout.CANONICAL:
        return gc.t()
    return backend().edges_from_canonical(gc, None, None, lay, rowmajor=True)


def _cm(x):
    """[N, C] user node tensor -> channel-major [C, N] fp32 on the device."""
    return x.detach().to(device=config.device, dtype=torch.float32).t().contiguous()


# ========================================================= parameter store
class _ParamMixin:
    """Hands the engine a module's parameters and gradient tensors by name."""

    def _check_device(self):
        for n, p in self.named_parameters():
            if not (p.is_cuda and p.dtype == torch.float32):
                raise RuntimeError(f"parameter {n} must be float32 on the HIP device "
                                   f"(call .to('cuda')); got {p.dtype} on {p.device}")

    def _flat_sync(self):
        self._check_device()

    def _flat_params(self):
        return {n: p.detach() for n, p in self.named_parameters()}

    def _flat_grads(self):
        out = {}
        for n, p in self.named_parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            out[n] = p.grad
        return out

    def _bn_buffers(self):
        return {n: b for n, b in self.named_buffers() if "running" in n}

    def _recording_grads(self):
        """The gradient dict a backward writes through, recording which
        parameters it wrote (``_mark_live`` after the backward)."""
        return _GradRecorder(self._flat_grads())

    def _mark_live(self, names):
        """Parameters a backward wrote (the ones the reference's autograd would
        give a .grad); FusedAdam skips the others (weight decay, step counts)."""
        params = dict(self.named_parameters())
        for n in names:
            p = params.get(n)
            if p is not None:
                p._pf_live = True

    def _bump_batches(self, edge_keys=(), node_keys=()):
        bufs = dict(self.named_buffers())
        for k in edge_keys:
            bufs[k + "num_batches_tracked"].add_(2)
        for k in node_keys:
            bufs[k + "num_batches_tracked"].add_(1)


def _mark_live_hook(p):
    p._pf_live = True


class _FlatMixin(_ParamMixin):
    """Top-level modules keep all parameters (and grads) as views of one flat
    fp32 buffer in the reference's state_dict order: the optimiser (FusedAdam)
    and the data-parallel gradient all-reduce then see a single buffer."""

    def _flat_sync(self):
        params = list(self.named_parameters())
        flat = getattr(self, "_pf_flat", None)
        if flat is not None and len(params) == len(self._pf_off):
            ok = True
            for (name, p), (off, n) in zip(params, self._pf_off):
                if p.data_ptr() != flat.data_ptr() + 4 * off or p.device != flat.device:
                    ok = False
                    break
            if ok:
                return
        dev = config.device
        offs, total = [], 0
        for _, p in params:
            offs.append((total, p.numel()))
            total += (p.numel() + 3) // 4 * 4
        flat = torch.zeros(total, dtype=torch.float32, device=dev)
        gflat = torch.zeros(total, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for (name, p), (off, n) in zip(params, offs):
                flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + n].view(p.shape)
                p.grad = None
        for mod in self.modules():                     # move BN buffers along
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.to(dev)
        self._pf_flat, self._pf_gflat, self._pf_off = flat, gflat, offs
        # a gradient that reaches a parameter through plain torch autograd (a
        # regulariser on the weights, ...) marks it live too, as p.grad is not
        # None would for torch.optim.Adam (FusedAdam reads _pf_live)
        for _, p in params:
            if not getattr(p, "_pf_hooked", False):
                p.register_post_accumulate_grad_hook(_mark_live_hook)
                p._pf_hooked = True

    def _flat_grads(self):
        """Attach every p.grad as a view of the flat grad buffer (zeroing the
        slices of grads that were None, keeping the values of existing ones)."""
        params = [p for _, p in self.named_parameters()]
        gflat = self._pf_gflat
        need = [(p, off, n) for p, (off, n) in zip(params, self._pf_off)
                if p.grad is None or p.grad.data_ptr() != gflat.data_ptr() + 4 * off]
        if need:
            if len(need) == len(params) and all(p.grad is None for p, _, _ in need):
                gflat.zero_()
                for p, off, n in need:
                    p.grad = gflat[off:off + n].view(p.shape)
            else:
                for p, off, n in need:
                    sl = gflat[off:off + n]
                    if p.grad is None:
                        sl.zero_()
                    else:
                        sl.copy_(p.grad.reshape(-1))
                    p.grad = sl.view(p.shape)
        return {n: p.grad for n, p in self.named_parameters()}

    def _bump_batches(self, edge_keys=(), node_keys=()):
        """num_batches_tracked += 2 (edge BatchNorms, applied twice) / += 1 for
        every BatchNorm of a forward, as ONE device add: the counters are
        views of one int64 buffer (re-made if a buffer was replaced, e.g. by
        ``.to()`` or ``load_state_dict`` assigning new tensors)."""
        key = (tuple(edge_keys), tuple(node_keys))
        names = [k + "num_batches_tracked" for k in key[0] + key[1]]
        cache = self.__dict__.get("_pf_nbt")
        bufs = None
        if cache is not None and cache[0] == key:
            flat = cache[1]
            bufs = dict(self.named_buffers())
            if any(bufs[n].data_ptr() != flat.data_ptr() + 8 * i or bufs[n].device != flat.device
                   for i, n in enumerate(names)):
                cache = None
        else:
            cache = None
        if cache is None:
            bufs = bufs or dict(self.named_buffers())
            flat = torch.stack([bufs[n].detach().reshape(()) for n in names]).contiguous()
            for i, n in enumerate(names):
                mod = self.get_submodule(n.rsplit(".", 1)[0])
                mod._buffers["num_batches_tracked"] = flat[i]
            inc = torch.tensor([2] * len(key[0]) + [1] * len(key[1]), dtype=flat.dtype,
                               device=flat.device)
            cache = (key, flat, inc)
            self.__dict__["_pf_nbt"] = cache
        cache[1].add_(cache[2])

    def zero_grad(self, set_to_none=True):
        """Zero the flat gradient buffer in one kernel and keep every ``p.grad``
        attached to it (the buffer the fused backward accumulates into, the
        all-reduce and FusedAdam read).  Dead parameters thus carry zero rather
        than None gradients; with Adam's moments starting at zero that leaves
        them exactly unchanged, as the reference's skipped None grads do.  No
        host sync and no reallocation, so the step can be graph-captured."""
        gflat = getattr(self, "_pf_gflat", None)
        for p in self.parameters():
            p._pf_live = False          # the reference's zero_grad leaves every .grad None
        if gflat is not None:
            params = [p for _, p in self.named_parameters()]
            if len(params) == len(self._pf_off) and all(
                    p.grad is not None and p.grad.data_ptr() == gflat.data_ptr() + 4 * off
                    for p, (off, n) in zip(params, self._pf_off)):
                gflat.zero_()
                return
        super().zero_grad(set_to_none=set_to_none)

    def flat_parameters(self):
        """(flat params, flat grads) -- the buffers FusedAdam / DDP operate on."""
        self._flat_sync()
        self._flat_grads()
        return self._pf_flat, self._pf_gflat


def _norm_or_identity(module, Fdim, normed, kind):
    if normed:
        module.norm = torch.nn.BatchNorm1d(Fdim) if kind == "bn" else torch.nn.RMSNorm(Fdim)
    else:
        module.norm = lambda x: x


def _engine_for(F, normed, B=0):
    return Engine(backend(), F=F, B=B, normed=normed)


# =================================================================== models
class _MLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, module):
        eng = _engine_for(module[0].out_features, True)
        P = module._flat_params()
        X = _cm(x)
        Y, saved = eng.mlp_fwd(P, "", X)
        ctx.module, ctx.saved_pf = module, saved
        return Y.t()

    @staticmethod
    def backward(ctx, gy):
        module = ctx.module
        eng = _engine_for(module[0].out_features, True)
        P = module._flat_params()
        Gr = module._recording_grads()
        be = backend()
        K = module[0].in_features
        dx = be.empty(K, gy.shape[0])
        eng.mlp_bwd(P, Gr, "", gy.t().contiguous(), ctx.saved_pf, outs=[(dx, K, False)])
        module._mark_live(Gr.used)
        return dx.t(), None, None


class MLP(_ParamMixin, torch.nn.Sequential):
    """gnn.py:65-71: Linear(D1, D2) -> LeakyReLU(0.1) -> Linear(D2, D3)."""

    def __init__(self, D1, D2, D3):
        super().__init__(torch.nn.Linear(D1, D2), torch.nn.LeakyReLU(0.1), torch.nn.Linear(D2, D3))

    def forward(self, x):
        self._flat_sync()
        return _MLPFn.apply(x, self[0].weight, self)


def _graph_of(x_s, x_t, u, edge_index, F):
    d, lay = geometry(x_s, x_t, u, edge_index, F)
    return d, lay


class _EdgeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_s, x_t, edge_attr, u, anchor, module, edge_index):
        F = module.Fdim
        d, lay = _graph_of(x_s, x_t, u, edge_index, F)
        eng = _engine_for(F, module.normed)
        eng.training = module.training
        eng.want_grad = not module.training    # (eval() under autograd: running statistics)
        P, BN = module._flat_params(), module._bn_buffers()
        st = eng.edge_fwd(P, BN, d, "", _cm(x_s), _cm(x_t), (edges_in(edge_attr, lay), None, None), _cm(u))
        if module.normed and module.training:
            module._bump_batches(edge_keys=("norm.",))
        ctx.pf = (module, d, lay, st)
        return edges_out((st["y"], st["sc"], st["sh"]), lay, d)

    @staticmethod
    def backward(ctx, g):
        module, d, lay, st = ctx.pf
        be, F = backend(), module.Fdim
        eng = _engine_for(F, module.normed)
        P, Gr = module._flat_params(), module._recording_grads()
        gc = grad_edges_in(g, lay)
        gc = be.zeros(F, d.EP) if gc is None else gc.contiguous()
        bnc = None
        if module.normed:
            Sg, Sgx = be.edge_bn_grad_sums(d, gc, st["y"], *eng.edge_bnstat(P, "", st))
            bnc = eng.edge_bn_coef(P, Gr, d, "", st, Sg, Sgx)
        g_xs, g_xt, g_u = be.zeros(F, d.NS), be.zeros(F, d.NT), be.zeros(F, d.G)
        g_xe = eng.edge_bwd(P, Gr, d, "", st, gc, bnc, True, g_xs, g_xt, g_u)
        module._mark_live(Gr.used)
        return g_xs.t(), g_xt.t(), grad_edges_out(g_xe, lay), g_u.t(), None, None, None


class EdgeModel(MLP):
    """gnn.py:73-101 (its BatchNorm runs twice, as in the reference)."""

    def __init__(self, Fdim=10, normed=True):
        F_message = 4 * Fdim
        super().__init__(F_message, F_message, Fdim)
        self.Fdim, self.normed = Fdim, normed
        _norm_or_identity(self, Fdim, normed, "bn")

    def forward(self, x_s, x_t, edge_index, edge_attr, u):
        self._flat_sync()
        return _EdgeFn.apply(x_s, x_t, edge_attr, u, self[0].weight, self, edge_index)


class _SourceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_s, x_t, edge_attr, u, anchor, module, edge_index):
        F = module.Fdim
        d, lay = _graph_of(x_s, x_t, u, edge_index, F)
        eng = _engine_for(F, module.normed)
        eng.training = module.training
        eng.want_grad = not module.training    # (eval() under autograd: running statistics)
        P, BN = module._flat_params(), module._bn_buffers()
        st = eng.source_fwd(P, BN, d, "", _cm(x_s), _cm(x_t), (edges_in(edge_attr, lay), None, None), _cm(u))
        if module.normed and module.training:
            module._bump_batches(node_keys=("norm.",))
        ctx.pf = (module, d, lay, st)
        return st["xs_new"].t()

    @staticmethod
    def backward(ctx, g):
        module, d, lay, st = ctx.pf
        be, F = backend(), module.Fdim
        eng = _engine_for(F, module.normed)
        P, Gr = module._flat_params(), module._recording_grads()
        g_xs, g_xt, g_u = be.zeros(F, d.NS), be.zeros(F, d.NT), be.zeros(F, d.G)
        coef = eng.source_node_bwd(P, Gr, d, "", st, g.t().contiguous(), g_xs, g_u)
        g_tot = eng.source_edge_bwd(P, Gr, d, "", st, coef, None, None, None, g_xt)[0]
        module._mark_live(Gr.used)
        return g_xs.t(), g_xt.t(), grad_edges_out(g_tot, lay), g_u.t(), None, None, None


class SModel(_ParamMixin, torch.nn.Module):
    """gnn.py:104-154."""

    def __init__(self, Fdim=10, normed=True):
        super().__init__()
        F_message = 2 * Fdim
        self.node_mlp_1 = MLP(F_message, F_message, F_message)
        F_message2 = 4 * F_message + 2 * Fdim
        self.node_mlp_2 = MLP(F_message2, F_message2, Fdim)
        self.Fdim, self.normed = Fdim, normed
        _norm_or_identity(self, Fdim, normed, "bn")

    def forward(self, x_s, x_t, edge_index, edge_attr, u):
        self._flat_sync()
        return _SourceFn.apply(x_s, x_t, edge_attr, u, self.node_mlp_1[0].weight, self, edge_index)


class _TargetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_s, x_t, edge_attr, u, anchor, module, edge_index):
        F = module.Fdim
        d, lay = _graph_of(x_s, x_t, u, edge_index, F)
        eng = _engine_for(F, module.normed)
        eng.training = module.training
        eng.want_grad = not module.training    # (eval() under autograd: running statistics)
        P, BN = module._flat_params(), module._bn_buffers()
        st = eng.target_fwd(P, BN, d, "", _cm(x_s), _cm(x_t), (edges_in(edge_attr, lay), None, None), _cm(u))
        if module.normed and module.training:
            module._bump_batches(node_keys=("norm.",))
        ctx.pf = (module, d, lay, st)
        return st["xt_new"].t()

    @staticmethod
    def backward(ctx, g):
        module, d, lay, st = ctx.pf
        be, F = backend(), module.Fdim
        eng = _engine_for(F, module.normed)
        P, Gr = module._flat_params(), module._recording_grads()
        g_xs, g_xt, g_u = be.zeros(F, d.NS), be.zeros(F, d.NT), be.zeros(F, d.G)
        g_hsum = eng.target_node_bwd(P, Gr, d, "", st, g.t().contiguous(), g_xt, g_u)
        gxe = eng.target_edge_bwd(P, Gr, d, "", st, g_hsum, True, g_xs)
        module._mark_live(Gr.used)
        return g_xs.t(), g_xt.t(), grad_edges_out(gxe, lay), g_u.t(), None, None, None


class TModel(_ParamMixin, torch.nn.Module):
    """gnn.py:157-192."""

    def __init__(self, Fdim=10, normed=True):
        super().__init__()
        F_message = 2 * Fdim
        self.node_mlp_1 = MLP(F_message, F_message, F_message)
        F_message2 = 4 * Fdim
        self.node_mlp_2 = MLP(F_message2, F_message2, Fdim)
        self.Fdim, self.normed = Fdim, normed
        _norm_or_identity(self, Fdim, normed, "bn")

    def forward(self, x_s, x_t, edge_index, edge_attr, u):
        self._flat_sync()
        return _TargetFn.apply(x_s, x_t, edge_attr, u, self.node_mlp_1[0].weight, self, edge_index)


class _GlobalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_s, x_t, u, anchor, module):
        F = module.Fdim
        G = int(u.size(0))
        d = Dims(G, x_s.size(0) // G, x_t.size(0) // G, F)
        eng = _engine_for(F, module.normed)
        P = module._flat_params()
        st = eng.global_fwd(P, d, "", _cm(x_s), _cm(x_t), _cm(u))
        ctx.pf = (module, d, st)
        return st["u_new"].t()

    @staticmethod
    def backward(ctx, g):
        module, d, st = ctx.pf
        be, F = backend(), module.Fdim
        eng = _engine_for(F, module.normed)
        P, Gr = module._flat_params(), module._recording_grads()
        g_xs, g_xt, g_u = be.zeros(F, d.NS), be.zeros(F, d.NT), be.zeros(F, d.G)
        eng.global_bwd(P, Gr, d, "", st, g.t().contiguous(), g_xs, g_xt, g_u)
        module._mark_live(Gr.used)
        return g_xs.t(), g_xt.t(), g_u.t(), None, None


class GlobalModel(MLP):
    """gnn.py:195-223 (its RMSNorm runs twice, as in the reference)."""

    def __init__(self, Fdim=10, normed=True):
        F_message = 3 * Fdim
        super().__init__(F_message, F_message, Fdim)
        self.Fdim, self.normed = Fdim, normed
        _norm_or_identity(self, Fdim, normed, "rms")

    def forward(self, x_s, x_t, edge_index, edge_attr, u):
        self._flat_sync()
        return _GlobalFn.apply(x_s, x_t, u, self[0].weight, self)


class Block(torch.nn.Module):
    """gnn.py:226-259: edge -> source -> target -> global."""

    def __init__(self, Fdim=10, e_model=True, s_model=True, t_model=True, u_model=True, normed=True):
        super().__init__()
        if e_model:
            self.edge_model = EdgeModel(Fdim, normed=normed)
        if s_model:
            self.s_model = SModel(Fdim, normed=normed)
        if t_model:
            self.t_model = TModel(Fdim, normed=normed)
        if u_model:
            self.global_model = GlobalModel(Fdim, normed=normed)

    def forward(self, args):
        edge_index, x_s, x_t, x_e, x_u = args
        if hasattr(self, "edge_model"):
            x_e = self.edge_model(x_s, x_t, edge_index, x_e, x_u)
        if hasattr(self, "s_model"):
            x_s = self.s_model(x_s, x_t, edge_index, x_e, x_u)
        if hasattr(self, "t_model"):
            x_t = self.t_model(x_s, x_t, edge_index, x_e, x_u)
        if hasattr(self, "global_model"):
            x_u = self.global_model(x_s, x_t, edge_index, x_e, x_u)
        return edge_index, x_s, x_t, x_e, x_u


# ====================================================================== GNN
class _GNNFn(torch.autograd.Function):
    """The whole GNN.forward as one fused engine call; its backward is the
    engine's hand-fused block backward (engine.Engine.backward).

    The final edge features are NOT an output: they stay in the engine's lazy
    canonical state (y, sc, sh).  In their place the function returns a 0-dim
    ``token`` that every consumer of the edge state takes as its autograd
    input -- the fused loss (train._LossFn) or the caller-order ``x_e`` view
    (_EdgesOutFn, built only if ``out.x_e`` is read).  Consumers hand their
    canonical [F, E] gradient over through the context, so nothing is ever
    converted to the caller's order unless the caller asks for it."""

    @staticmethod
    def forward(ctx, anchor, model, d, lay, xs_in, xt_in, xe_in, u_in):
        ctx.set_materialize_grads(False)      # unused outputs -> None -> dead work skipped
        P, BN = model._flat_params(), model._bn_buffers()
        # (eval() under autograd: BatchNorm on running statistics, nothing
        # updated, the backward differentiates those affine maps)
        ectx = model._engine().forward(P, BN, d, xs_in, xt_in, xe_in, u_in,
                                       training=model.training, want_grad=not model.training)
        if model.normed and model.training:
            model._bump_batches(
                edge_keys=[f"mpb.{b}.edge_model.norm." for b in range(model.B)],
                node_keys=[f"mpb.{b}.{m}.norm." for b in range(model.B) for m in ("s_model", "t_model")])
        xs, xt, xe3, u = ectx["out"]
        ctx.pf = (model, d, lay, ectx)
        model._pf_last = (xe3, ectx)
        token = xs.new_empty(())            # connectivity only: its value is never read
        return xs.t(), xt.t(), token, u.t()

    @staticmethod
    def backward(ctx, g_xs, g_xt, g_token, g_u):
        model, d, lay, ectx = ctx.pf
        P, Gr = model._flat_params(), model._recording_grads()
        cm = (lambda g: None if g is None else g.t().contiguous())
        # consumers of the edge state hand their gradient over in canonical order
        gc = ectx.pop("g_xe_canonical", None)
        model._engine().backward(P, Gr, ectx, gc, cm(g_xs), cm(g_xt), cm(g_u))
        model._mark_live(Gr.used)
        return (None,) * 8


class _EdgesOutFn(torch.autograd.Function):
    """Caller-order ``x_e`` [E, F] of a GNN output, materialised on first read
    from the lazy canonical state; its gradient goes back to _GNNFn through
    the shared context (canonical order), the token gets a zero."""

    @staticmethod
    def forward(ctx, token, ectx, xe3, lay, d):
        ctx.pf = (ectx, lay)
        return edges_out(xe3, lay, d)

    @staticmethod
    def backward(ctx, g):
        ectx, lay = ctx.pf
        gc = grad_edges_in(g, lay)
        if gc is not None:
            gc = gc.contiguous()
            prev = ectx.get("g_xe_canonical")
            ectx["g_xe_canonical"] = gc if prev is None else prev + gc
            # (a second consumer: the loss's BatchNorm sums no longer cover g_xe)
            ectx.pop("g_xe_bn_part", None)
        return None, None, None, None, None


class _GradRecorder(dict):
    """Parameter-gradient dict that records which entries a backward wrote
    (the parameters autograd would give a .grad in the reference)."""

    def __init__(self, d):
        super().__init__(d)
        self.used = set()

    def __getitem__(self, k):
        self.used.add(k)
        return super().__getitem__(k)


class GNNOutput(BipartiteData):
    """The BipartiteData GNN.forward returns (gnn.py:305).  ``x_e`` is built on
    first read (caller's edge order); the fused loss never reads it."""

    @property
    def x_e(self):
        v = self.__dict__.get("_x_e_val")
        if v is None:
            mk = self.__dict__.get("_x_e_make")
            if mk is None:
                return None
            v = mk()
            self.__dict__["_x_e_val"] = v
        return v

    @x_e.setter
    def x_e(self, v):
        self.__dict__["_x_e_val"] = v
        self.__dict__["_x_e_make"] = None
        if "_pf" in self.__dict__:        # replaced by the caller: the fused loss
            self.__dict__["_pf_replaced"] = True   # must not read the engine state

    def to(self, device):
        return BipartiteData(self.edge_index, self.x_s, self.x_t, self.x_e, self.x_u).to(device)


class GNN(_FlatMixin, torch.nn.Module):
    """gnn.py:261-326."""

    def __init__(self, B=4, Fdim=16, T=12, F_s=1, F_t=1, normed=True):
        super().__init__()
        self.encoder_s = MLP(F_s, Fdim, Fdim)
        self.encoder_t = MLP(F_t, Fdim, Fdim)
        self.mpb = torch.nn.Sequential(*(Block(Fdim, normed=normed) for b in range(B)))
        self.decoder_e = MLP(Fdim, Fdim, 1)
        self.decoder_s = MLP(Fdim, Fdim, T)
        self.B, self.Fdim, self.T, self.F_s, self.F_t, self.normed = B, Fdim, T, F_s, F_t, normed

    def _engine(self):
        return Engine(backend(), F=self.Fdim, B=self.B, Fs=self.F_s, Ft=self.F_t, T=self.T,
                      normed=self.normed)

    def forward(self, graph):
        # eval() with autograd on (gnn.eval() then loss.backward(): BatchNorm on
        # running statistics, round() the identity, gnn.py:321-325) runs the
        # differentiable path as in training, nothing updated
        grad = self.training or (torch.is_grad_enabled() and any(
            p.requires_grad for p in self.parameters()))
        for t in (graph.x_s, graph.x_t, graph.x_e, graph.x_u):
            if t is not None and t.requires_grad:
                raise NotImplementedError("gradients w.r.t. the graph inputs are not computed")
        self._flat_sync()
        d, lay = geometry(graph.x_s, graph.x_t, graph.x_u, graph.edge_index, self.Fdim)
        xe_in = edges_in(graph.x_e, lay, cache=True)
        out = GNNOutput.__new__(GNNOutput)
        if grad:
            anchor = self.encoder_s[0].weight
            xs, xt, token, u = _GNNFn.apply(anchor, self, d, lay, _cm(graph.x_s), _cm(graph.x_t),
                                            xe_in, _cm(graph.x_u))
            xe3, ectx = self.__dict__.pop("_pf_last")
            out._x_e_make = lambda: _EdgesOutFn.apply(token, ectx, xe3, lay, d)
        else:
            xs, xt, u = self._forward_eval(d, lay, _cm(graph.x_s), _cm(graph.x_t), xe_in,
                                           _cm(graph.x_u))
            xe3, ectx = self.__dict__.pop("_pf_last")
            token = None
            out._x_e_make = lambda: edges_out(xe3, lay, d)
        out._x_e_val = None
        out.edge_index, out.x_s, out.x_t, out.x_u = graph.edge_index, xs, xt, u
        out.num_nodes = xt.size(0)
        # lets train.loss_function fuse on the lazy final edge state (y, sc, sh)
        out._pf = (self, d, lay, token, xe3, ectx)
        return out

    def _forward_eval(self, d, lay, xs_in, xt_in, xe_in, u_in):
        """GNN.forward in eval mode (gnn.py:280-305 with every BatchNorm1d on its
        running statistics, none updated, num_batches_tracked unchanged)."""
        P, BN = self._flat_params(), self._bn_buffers()
        ectx = self._engine().forward(P, BN, d, xs_in, xt_in, xe_in, u_in, training=False)
        xs, xt, xe3, u = ectx["out"]
        self._pf_last = (xe3, ectx)
        return xs.t(), xt.t(), u.t()

    def edge_prediction(self, x_e, scale=1):
        """gnn.py:307-312 (``round`` is the identity: ``self.train`` is a bound
        method, always truthy, gnn.py:321)."""
        pred = self.decoder_e(x_e)
        return torch.nn.functional.softplus(pred) * scale

    def node_prediction(self, x_s, scale=1):
        """gnn.py:314-319."""
        pred = self.decoder_s(x_s)
        return torch.softmax(pred, dim=-1) * scale

    def round(self, x):
        return x
