"""CPU oracle for the bipartite message-passing training step.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker (or, in ``bench.py``, as the timed
CPU baseline).  The product path (``pfs-neural-net_amd/pfsgnn``) never imports
this package and fails loudly when its HIP library is missing.

What it is: a plain PyTorch-CPU restatement of the reference algorithm
(joshua-lintropic/pfs-neural-net, ``src/gnn.py`` + ``src/train.py`` +
``src/graph.py``), with ``torch_scatter.scatter`` restated as
``index_add_``-based sums (the reference's third-party scatter is absent from
this image; see ``oracle/ref_scatter.py`` for the restated semantics).
Autograd supplies the backward pass, exactly as in the reference's
``loss.backward()`` (train.py:140).

How it is pinned: against the reference's own shipped
fixtures -- the raw tensor storages of ``graphs/graph-0.pt`` (edge order and
node features, ``tests/golden/graph0.npz``) and the trained checkpoint
``params/model_gnn_0.pth`` (state-dict keys/shapes, and the BatchNorm running
statistics its training run recorded, reproduced statistically by this
oracle's forward pass: ``tests/golden/ckpt_pin.npz``).  The reference itself
cannot run here (``torch_geometric`` and ``torch_scatter`` are not installed),
so no output vectors of the reference exist; the BatchNorm running-statistics
pin is the known-answer test for the forward wiring.
"""
