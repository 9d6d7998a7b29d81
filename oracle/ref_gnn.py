"""CPU restatement of the reference GNN (``src/gnn.py``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the checker for the
HIP path, never the thing measured or shipped.

Each class follows the reference line by line (citations are to
``src/gnn.py`` of joshua-lintropic/pfs-neural-net).  Module and parameter
names are kept identical so ``state_dict`` objects interchange with the
reference checkpoint (``params/model_gnn_0.pth``) and with the product
modules.

Batching: the reference builds single graphs (train.py:94, graph.py:14) and
its ``u.expand(E, -1)`` (gnn.py:100) only accepts one graph.  For a batch of
G graphs (PyG-style disjoint union, BipartiteData.__inc__ gnn.py:32) this
oracle broadcasts ``u[g]`` to the edges / nodes of graph g and takes the
GlobalModel means per graph; with G == 1 both reduce exactly to the
reference expressions.  BatchNorm statistics are taken over the whole batch,
as torch.nn.BatchNorm1d does on the concatenated rows.
"""
import torch
import torch.nn.functional as F

from .ref_scatter import scatter


class Graph:
    """Minimal stand-in for ``gnn.BipartiteData`` (gnn.py:7): attribute names
    match the reference (edge_index, x_s, x_t, x_e, x_u).  ``s_batch`` /
    ``t_batch`` give the graph id of every source / target node (PyG's
    ``batch`` vectors); ``None`` means a single graph."""

    def __init__(self, edge_index, x_s, x_t, x_e, x_u, s_batch=None, t_batch=None):
        self.edge_index = edge_index
        self.x_s = x_s
        self.x_t = x_t
        self.x_e = x_e
        self.x_u = x_u
        self.s_batch = s_batch
        self.t_batch = t_batch


def _u_rows(u, batch, n):
    # gnn.py:100 / 153 / 191 use u.expand(n, -1); per-graph broadcast for G > 1
    if batch is None:
        return u.expand(n, -1)
    return u[batch]


class MLP(torch.nn.Sequential):
    """gnn.py:65-71: Linear -> LeakyReLU(0.1) -> Linear."""

    def __init__(self, D1, D2, D3):
        super().__init__(torch.nn.Linear(D1, D2), torch.nn.LeakyReLU(0.1), torch.nn.Linear(D2, D3))


class EdgeModel(MLP):
    """gnn.py:73-101."""

    def __init__(self, Fdim=10, normed=True):
        F_message = 4 * Fdim
        super().__init__(F_message, F_message, Fdim)
        self.norm = torch.nn.BatchNorm1d(Fdim) if normed else (lambda x: x)

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None):
        src, tgt = edge_index
        E = edge_attr.size(0)
        ue = _u_rows(u, None if s_batch is None else s_batch[src], E)
        h = torch.cat([x_s[src], x_t[tgt], edge_attr, ue], dim=-1)       # gnn.py:100
        return self.norm(super().forward(h))                              # gnn.py:101


class SModel(torch.nn.Module):
    """gnn.py:104-154: source (fiber) update from moment statistics."""

    def __init__(self, Fdim=10, normed=True):
        super().__init__()
        F_message = 2 * Fdim
        self.node_mlp_1 = MLP(F_message, F_message, F_message)
        F_message2 = 4 * F_message + 2 * Fdim
        self.node_mlp_2 = MLP(F_message2, F_message2, Fdim)
        self.norm = torch.nn.BatchNorm1d(Fdim) if normed else (lambda x: x)

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None):
        src, tgt = edge_index
        n = x_s.size(0)
        msg = torch.cat([x_t[tgt], edge_attr], dim=1)                     # gnn.py:136
        msg = self.node_mlp_1(msg)
        mean = scatter(msg, src, n, reduce="mean")                        # gnn.py:140
        var = F.leaky_relu(scatter(msg ** 2, src, n, reduce="mean") - mean ** 2)   # gnn.py:141
        std = torch.sqrt(var + 1e-6)
        skew = scatter((msg - mean[src]) ** 3, src, n, reduce="mean") / std ** 3  # gnn.py:143
        kurt = scatter((msg - mean[src]) ** 4, src, n, reduce="mean") / std ** 4  # gnn.py:144
        mean = torch.nan_to_num(mean, nan=0.0)                           # gnn.py:147-151
        var = torch.nan_to_num(var, nan=0.0)
        std = torch.sqrt(var + 1e-6)
        skew = torch.nan_to_num(skew, nan=0.0)
        kurt = torch.nan_to_num(kurt, nan=0.0)
        h_cat = torch.cat([x_s, mean, std, skew, kurt, _u_rows(u, s_batch, n)], dim=-1)  # gnn.py:153
        return self.norm(self.node_mlp_2(h_cat))


class TModel(torch.nn.Module):
    """gnn.py:157-192: target (class) update from summed messages."""

    def __init__(self, Fdim=10, normed=True):
        super().__init__()
        F_message = 2 * Fdim
        self.node_mlp_1 = MLP(F_message, F_message, F_message)
        F_message2 = 4 * Fdim
        self.node_mlp_2 = MLP(F_message2, F_message2, Fdim)
        self.norm = torch.nn.BatchNorm1d(Fdim) if normed else (lambda x: x)

    def forward(self, x_s, x_t, edge_index, edge_attr, u, t_batch=None):
        src, tgt = edge_index
        msg = torch.cat([x_s[src], edge_attr], dim=1)                     # gnn.py:188
        msg = self.node_mlp_1(msg)
        agg = scatter(msg, tgt, x_t.size(0), reduce="sum")                # gnn.py:190
        h_cat = torch.cat([x_t, agg, _u_rows(u, t_batch, len(x_t))], dim=-1)  # gnn.py:191
        return self.norm(self.node_mlp_2(h_cat))


class GlobalModel(MLP):
    """gnn.py:195-223."""

    def __init__(self, Fdim=10, normed=True):
        F_message = 3 * Fdim
        super().__init__(F_message, F_message, Fdim)
        self.norm = torch.nn.RMSNorm(Fdim) if normed else (lambda x: x)

    def forward(self, x_s, x_t, edge_index, edge_attr, u, s_batch=None, t_batch=None):
        if s_batch is None:
            s_mean = x_s.mean(dim=0, keepdim=True)                        # gnn.py:220
            t_mean = x_t.mean(dim=0, keepdim=True)
        else:
            G = u.size(0)
            s_mean = scatter(x_s, s_batch, G, reduce="mean")
            t_mean = scatter(x_t, t_batch, G, reduce="mean")
        h_cat = torch.cat([u, s_mean, t_mean], dim=-1)                    # gnn.py:222
        return self.norm(super().forward(h_cat))


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

    def forward(self, args, s_batch=None, t_batch=None):
        edge_index, x_s, x_t, x_e, x_u = args
        if hasattr(self, "edge_model"):
            x_e = self.edge_model(x_s, x_t, edge_index, x_e, x_u, s_batch)
        if hasattr(self, "s_model"):
            x_s = self.s_model(x_s, x_t, edge_index, x_e, x_u, s_batch)
        if hasattr(self, "t_model"):
            x_t = self.t_model(x_s, x_t, edge_index, x_e, x_u, t_batch)
        if hasattr(self, "global_model"):
            x_u = self.global_model(x_s, x_t, edge_index, x_e, x_u, s_batch, t_batch)
        return edge_index, x_s, x_t, x_e, x_u


class GNN(torch.nn.Module):
    """gnn.py:261-326."""

    def __init__(self, B=4, Fdim=16, T=12, F_s=1, F_t=1, normed=True):
        super().__init__()
        self.encoder_s = MLP(F_s, Fdim, Fdim)
        self.encoder_t = MLP(F_t, Fdim, Fdim)
        self.mpb = torch.nn.Sequential(*(Block(Fdim, normed=normed) for _ in range(B)))
        self.decoder_e = MLP(Fdim, Fdim, 1)
        self.decoder_s = MLP(Fdim, Fdim, T)

    def forward(self, graph):
        x_s = self.encoder_s(graph.x_s)                                   # gnn.py:297
        x_t = self.encoder_t(graph.x_t)
        args = (graph.edge_index, x_s, x_t, graph.x_e, graph.x_u)
        for blk in self.mpb:                                              # gnn.py:302
            args = blk(args, graph.s_batch, graph.t_batch)
        _, x_s, x_t, x_e, x_u = args
        return Graph(graph.edge_index, x_s, x_t, x_e, x_u, graph.s_batch, graph.t_batch)

    def edge_prediction(self, x_e, scale=1):
        # gnn.py:307-312.  ``self.round`` tests ``self.train`` -- a bound method,
        # always truthy -- so the reference's rounding is the identity in every
        # mode (gnn.py:321-325); restated as such.
        pred = self.decoder_e(x_e)
        return F.softplus(pred) * scale

    def node_prediction(self, x_s, scale=1):
        # gnn.py:314-319 (round is the identity, see above)
        pred = self.decoder_s(x_s)
        return torch.softmax(pred, dim=-1) * scale
