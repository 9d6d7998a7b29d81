"""The SModel message cache (pfsgnn_msg_bytes / pfsgnn_source_fwd_msg /
pfsgnn_source_bwd(_bn)_msg; off unless PFSGNN_MSG=1, read once per process):
a training step with the forward's messages kept and read back by the
backward must equal the recomputing step bit for bit, on both edge paths that
keep it (mfma, mfma32) -- each arm in its own process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

SCRIPT = r"""
import hashlib, os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "tests"), os.path.join({root!r}, "pfs-neural-net_amd")]
import torch
from pfsgnn import native
from harness import make_problem
from test_gpu_parity import ours_step
G, NF, NC, B = 2, 150, 24, 3
model, graph = make_problem(G, NF, NC, B=B, seed=9, dtype=torch.float32)
gnn, out, loss = ours_step(model, graph, G, NF, NC, B, 31, 10.0)
h = hashlib.sha1()
for t in [loss.reshape(1), out.x_e, out.x_s, out.x_t, out.x_u] + [p.grad for p in gnn.parameters()]:
    h.update(t.detach().float().contiguous().cpu().numpy().tobytes())
print("MSGBYTES", native.lib().pfsgnn_msg_bytes(G, NF, NC, 10))
print("DIGEST", h.hexdigest())
"""


def run(path, msg):
    env = dict(os.environ, PFSGNN_EDGE_PATH=path, PFSGNN_MSG=str(msg))
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    vals = dict(l.split(None, 1) for l in r.stdout.splitlines() if l.startswith(("MSG", "DIG")))
    return int(vals["MSGBYTES"]), vals["DIGEST"]


@pytest.mark.parametrize("path", ["mfma", "mfma32"])
def test_message_cache_step_is_bitwise_the_recomputing_step(path):
    on_bytes, on = run(path, 1)
    off_bytes, off = run(path, 0)
    assert on_bytes == 2 * 150 * 24 * 2 * 10 * 4 and off_bytes == 0
    assert on == off
