"""Per-shape device time of the node GEMM ops (GPU box): 50 back-to-back launches per shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd")]
import torch  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

hb = HipBackend()
dev = "cuda"
SH = [(100, 100, 38304), (10, 100, 38304), (40, 40, 38304), (20, 20, 38304), (10, 40, 38304),
      (40, 40, 2048), (20, 20, 2048), (10, 40, 2048), (30, 30, 16), (10, 30, 16)]


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for M, K, N in SH:
    W = torch.randn(M, K, device=dev)
    X = torch.randn(K, N, device=dev)
    dY = torch.randn(M, N, device=dev)
    Z = torch.randn(K, N, device=dev)
    dW = torch.zeros(M, K, device=dev)
    db = torch.zeros(M, device=dev)
    t1 = timeit(lambda: hb.lin(W, 0, K, X))
    t2 = timeit(lambda: hb.lin_t(W, 0, K, dY, z=Z))
    t3 = timeit(lambda: hb.wgrad(dY, X, dW, db=db))
    gb = (M * N + K * N) * 4 / 1e9
    print(f"M={M:4d} K={K:4d} N={N:6d}  lin {t1:7.1f}us  lin_t {t2:7.1f}us  wgrad {t3:7.1f}us  "
          f"(in+out {gb * 1e3:.1f} MB -> {gb / 8e3 * 1e6:.1f}us at 8TB/s)")
