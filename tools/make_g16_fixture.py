"""Oracle fixture for the bench geometry (tests/test_gpu_bench_geometry.py).

The bench batch -- G=16 complete 2394x128 graphs, B=8 blocks, the full
train.py training step -- on the CPU oracle in float64 and in float32, saved
as tests/golden/g16_oracle.npz.  The oracle needs ~130 GB of host memory at
this size (this container has 64), so the fixture is made on the GPU box's
host, which has the memory:

    gpurun -- 'python tools/make_g16_fixture.py gpurun_out/g16_oracle.npz'

and copied to tests/golden/.  Since round 4 the file also holds a second
float32 run with the edges in reversed order ("f32r:" keys; the test's fp32
error level is the larger of the two, as test_gpu_parity's), added to an
existing fixture without recomputing float64:

    gpurun -- 'python tools/make_g16_fixture.py --add-reverse tests/golden/g16_oracle.npz gpurun_out/g16_oracle.npz'

A heartbeat line every 30 s keeps the long oracle steps visibly alive.
Everything compared by the test is in the file:
the loss, every parameter gradient, the BatchNorm running statistics, x_t and
x_u whole, x_s and x_e on seeded row samples, and x_e's per-channel sums and
sums of squares over all 4.9 M edges (float64 accumulation).
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pfs-neural-net_amd")]

from harness import make_problem  # noqa: E402
from test_gpu_parity import oracle_step  # noqa: E402

G, NF, NC, B, SHARP = 16, 2394, 128, 8, 10.0
MODEL_SEED, NOISE_SEED = 2394 + G, 4242 + G
N_XS, N_XE = 4096, 16384


def samples():
    gen = torch.Generator().manual_seed(77)
    ixs = torch.randperm(G * NF, generator=gen)[:N_XS].sort().values
    ixe = torch.randperm(G * NF * NC, generator=gen)[:N_XE].sort().values
    return ixs, ixe


def heartbeat(t0):
    import threading

    def beat():
        while True:
            time.sleep(30)
            print(f"[g16] ... working ({time.time() - t0:.0f}s)", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def run(dtype, t0, reverse=False):
    model, graph = make_problem(G, NF, NC, B=B, seed=MODEL_SEED)
    print(f"[g16] {dtype} oracle step (reverse={reverse}) ... ({time.time() - t0:.0f}s)", flush=True)
    m, out, loss = oracle_step(model, graph, G, NF, NC, NOISE_SEED, SHARP, dtype, reverse=reverse)
    print(f"[g16] {dtype} done ({time.time() - t0:.0f}s)", flush=True)
    ixs, ixe = samples()
    d = {"loss": np.array([loss.item()])}
    for n, p in m.named_parameters():
        d["grad " + n] = (p.grad if p.grad is not None else torch.zeros_like(p)).double().numpy()
    for k, v in m.state_dict().items():
        if "running" in k or "num_batches" in k:
            d[k] = v.double().numpy()
    xe = out.x_e.detach()
    d["x_t"] = out.x_t.detach().double().numpy()
    d["x_u"] = out.x_u.detach().double().numpy()
    d["x_s_sample"] = out.x_s.detach()[ixs].double().numpy()
    d["x_e_sample"] = xe[ixe].double().numpy()
    d["x_e_sum"] = xe.double().sum(0).numpy()
    d["x_e_sumsq"] = (xe.double() ** 2).sum(0).numpy()
    return d


def add_reverse(src, dst):
    """Add the reversed-order float32 run ("f32r:") to an existing fixture."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.time()
    heartbeat(t0)
    z = np.load(src)
    out = {k: z[k] for k in z.files}
    for k, v in run(torch.float32, t0, reverse=True).items():
        out["f32r:" + k] = v
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    np.savez_compressed(dst, **out)
    print(f"[g16] wrote {dst} ({os.path.getsize(dst) / 1e6:.1f} MB, {time.time() - t0:.0f}s)", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--add-reverse":
        return add_reverse(sys.argv[2], sys.argv[3])
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "g16_oracle.npz")
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.time()
    heartbeat(t0)
    r64 = run(torch.float64, t0)
    r32 = run(torch.float32, t0)
    r32r = run(torch.float32, t0, reverse=True)
    ixs, ixe = samples()
    out = {"G": G, "NF": NF, "NC": NC, "B": B, "sharp": SHARP, "model_seed": MODEL_SEED,
           "noise_seed": NOISE_SEED, "ix_s": ixs.numpy(), "ix_e": ixe.numpy()}
    for k, v in r64.items():
        out["f64:" + k] = v
    for k, v in r32.items():
        out["f32:" + k] = v
    for k, v in r32r.items():
        out["f32r:" + k] = v
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    np.savez_compressed(dst, **out)
    print(f"[g16] wrote {dst} ({os.path.getsize(dst) / 1e6:.1f} MB, {time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
