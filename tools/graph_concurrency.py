"""Does a captured HIP graph run independent tiny kernels concurrently?

Captures 2 x 200 small elementwise kernels (a) on one stream and (b) forked
over two streams, and compares replay times (GPU box)."""
import torch

torch.cuda.set_device(0)
n = 200
a = [torch.zeros(4096, device="cuda") for _ in range(4)]
main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def work(t, k):
    for _ in range(k):
        t.add_(1.0)


def capture(two):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(main)
    with torch.cuda.stream(s):
        work(a[0], 1)
    main.wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        if two:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                work(a[1], n)
            work(a[0], n)
            cur.wait_stream(side)
        else:
            work(a[1], n)
            work(a[0], n)
    return g


for two in (False, True, False, True):
    g = capture(two)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        g.replay()
    e.record()
    e.synchronize()
    print(f"{'two streams' if two else 'one stream '}: {s.elapsed_time(e) / 20 * 1e3:8.1f} us per "
          f"replay of {2 * n} kernels", flush=True)
