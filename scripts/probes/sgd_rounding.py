"""Which rounding does torch.optim.SGD's plain step use on this ROCm build? Compares torch's
result bit for bit with p - lr*g as one fma and as a rounded multiply then add, for the
foreach (default), fused and single-tensor implementations."""
import torch

torch.manual_seed(0)
dev = torch.device("cuda:0")
n = 1 << 20
p0 = torch.randn(n, device=dev)
g = torch.randn(n, device=dev) * 3.7
for lr in (1.0, 0.1, 0.0123, 1e-4):
    lr32 = torch.tensor(lr, dtype=torch.float32).item()
    fma = torch.addcmul(p0, g, torch.full_like(g, -lr32))  # reference points, computed on host below
    pd, gd = p0.double().cpu(), g.double().cpu()
    lrf = torch.tensor(lr, dtype=torch.float32)
    fma_ref = (pd - lrf.double() * gd).float()                 # exact product, one rounding
    mul_add = (p0.cpu() + (-lrf) * g.cpu())                     # rounded product, then add (CPU fp32)
    for kw in ({}, {"foreach": True}, {"foreach": False}, {"fused": True}):
        p = p0.clone().requires_grad_(True)
        p.grad = g.clone()
        opt = torch.optim.SGD([p], lr=lr, **kw)
        opt.step()
        got = p.detach().cpu()
        print(f"lr {lr} {kw or 'default'}: equal fma {torch.equal(got, fma_ref)}, equal mul+add "
              f"{torch.equal(got, mul_add)}, diffs vs fma {(got != fma_ref).sum().item()} vs mul+add "
              f"{(got != mul_add).sum().item()}")
