"""Which rounding does torch.optim.Adam's device path use?  Runs each foreach
primitive of torch/optim/adam.py _multi_tensor_adam on the GPU and compares it
bit for bit with candidate fp32 formulas evaluated exactly on the host
(diagnostic for pfsgnn_adam / tests/test_gpu_adam_resume.py)."""
import torch

torch.manual_seed(0)
n = 1 << 20
dev = "cuda"
p = torch.randn(n) * 0.3
m = torch.randn(n) * 1e-3
v = torch.rand(n) * 1e-5 + 1e-9
bc2s = (1 - 0.999 ** 40001) ** 0.5
s = -(5e-4 / (1 - 0.9 ** 40001))
eps = 1e-8


def f32(x):
    return x.to(torch.float32)


def fma(a, b, c):
    return f32(a.double() * b.double() + c.double())


# 1. sqrt
sq = torch._foreach_sqrt([v.to(dev)])[0].cpu()
print("sqrt exact:", torch.equal(sq, f32(v.double().sqrt())))
# 2. div by scalar list
dv = [sq.to(dev).clone()]
torch._foreach_div_(dv, [bc2s])
dv = dv[0].cpu()
print("div a/b:", torch.equal(dv, f32(sq.double() / f32(torch.tensor(bc2s, dtype=torch.float64)).double())),
      " a*(1/b):", torch.equal(dv, f32(sq.double() * f32(1.0 / torch.tensor(bc2s, dtype=torch.float64)).double())),
      " double b:", torch.equal(dv, f32(sq.double() / bc2s)))
# 3. add eps
de = [dv.to(dev).clone()]
torch._foreach_add_(de, eps)
de = de[0].cpu()
print("add eps f32:", torch.equal(de, f32(dv.double() + f32(torch.tensor(eps, dtype=torch.float64)).double())),
      " double eps:", torch.equal(de, f32(dv.double() + eps)))
# 4. addcdiv with scalar list
pp = [p.to(dev).clone()]
torch._foreach_addcdiv_(pp, [m.to(dev)], [de.to(dev)], [s])
pp = pp[0].cpu()
sf = f32(torch.tensor(s, dtype=torch.float64))
q = f32(m.double() / de.double())
cands = {
    "fma(s, m/d, p)": fma(sf, q, p),
    "p + round(s*(m/d))": f32(p.double() + f32(sf.double() * q.double()).double()),
    "p + round(round(s*m)/d)": f32(p.double() + f32(f32(sf.double() * m.double()).double() / de.double()).double()),
    "fma(s double, m/d, p)": f32(torch.tensor(s, dtype=torch.float64) * q.double() + p.double()),
}
for k, c in cands.items():
    print(f"addcdiv {k}: equal={torch.equal(pp, c)} mismatches={(pp != c).sum().item()}")
