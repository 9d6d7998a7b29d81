"""One training step at a given shape; prints a digest of every output and
gradient (sha1 of the raw fp32 bytes), so two builds / knob settings can be
compared for bitwise equality from separate processes.
    python tools/step_digest.py [G NF NC B]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pfs-neural-net_amd")]
from harness import make_problem  # noqa: E402
from test_gpu_parity import ours_step  # noqa: E402

G, NF, NC, B = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (2, 2394, 128, 8)
model, graph = make_problem(G, NF, NC, B=B, seed=5, dtype=torch.float32)
gnn, out, loss = ours_step(model, graph, G, NF, NC, B, 99, 10.0)
h = hashlib.sha1()
for t in [loss.reshape(1), out.x_e, out.x_s, out.x_t, out.x_u] + [p.grad for p in gnn.parameters()]:
    h.update(t.detach().float().contiguous().cpu().numpy().tobytes())
print("digest", G, NF, NC, B, h.hexdigest(), f"loss {loss.item():.9g}")
