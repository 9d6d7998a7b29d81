"""Phase clocks of k_class_tail_fwd (diagnostic build with -DPF_TAIL_STAMPS,
PFSGNN_LIB_VARIANT=stamps): runs bench-shape training steps, then prints per
phase the median / max over workgroups of the s_memtime ticks since the
earliest workgroup start, for the last tail launch of the last step (GPU box).

    PFSGNN_LIB_VARIANT=stamps python tools/tail_stamps.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn import config, native  # noqa: E402

G, NF, NC, F, B = 16, 2394, 128, 10, 8
config.device = torch.device("cuda")
e = torch.arange(G * NF * NC)
ei = torch.stack([e // NC, (e // (NF * NC)) * NC + e % NC])
gen = torch.Generator().manual_seed(0)
xs = torch.arange(NF, dtype=torch.float).repeat(G).reshape(-1, 1)
xt = torch.cat([torch.randint(2, 13, (G * NC, 1), generator=gen).float(),
                torch.randint(1000, 100000, (G * NC, 1), generator=gen).float()], 1)
xe = 2.0 + 8.0 * torch.rand(G * NF * NC, F, generator=gen)
data = pfsgnn.BipartiteData(ei, xs, xt, xe, torch.zeros(G, F))
gnn = pfsgnn.GNN(B=B, Fdim=F, T=NC, F_s=1, F_t=2).cuda()
gnn.train()
for _ in range(3):
    out = gnn(data)
    (out.x_e.sum() + out.x_s.sum()).backward()
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (512 * 8))()
assert native.lib().pfsgnn_debug_tail_stamps(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8).astype(np.int64)
st = st[st[:, 0] > 0]
# (s_memtime counts per XCD: only differences within a workgroup are compared)
names = ["weights", "partials(1st unit)", "phase1 rest", "barrier wait", "bn stats", "phase 2"]
print(f"{len(st)} workgroups; shader-clock ticks per phase (min / median / max over workgroups):")
for i, n in enumerate(names):
    v = st[:, i + 1] - st[:, i]
    print(f"  {n:22s} {int(v.min()):8d} {int(np.median(v)):8d} {int(v.max()):8d}")
v = st[:, 6] - st[:, 0]
print(f"  {'total':22s} {int(v.min()):8d} {int(np.median(v)):8d} {int(v.max()):8d}")
# within one XCD (workgroups b with the same b % 8 share a clock): spread of
# the starts, the barrier arrivals and the barrier exits
for x in range(2):
    sub = st[x::8]
    for i, n in ((0, "start"), (3, "arrive"), (4, "exit")):
        v = sub[:, i] - sub[:, 0].min()
        print(f"  xcd {x} {n:7s} min {int(v.min()):7d} median {int(np.median(v)):7d} max {int(v.max()):7d}")
assert native.lib().pfsgnn_debug_cb_stamps(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8).astype(np.int64)
st = st[st[:, 0] > 0]
names = ["weights", "phase 1", "barrier 1", "phase 2", "barrier 2", "phase 3"]
print(f"class backward: {len(st)} workgroups; ticks per phase (min / median / max):")
for i, n in enumerate(names):
    v = st[:, i + 1] - st[:, i]
    print(f"  {n:22s} {int(v.min()):8d} {int(np.median(v)):8d} {int(v.max()):8d}")
print("sync faults:", native.HipBackend().sync_faults())
