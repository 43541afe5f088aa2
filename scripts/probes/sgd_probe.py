import torch, time
dev = torch.device("cuda:0")
ent = torch.randn(14208, 200, device=dev, requires_grad=True)
rel = torch.randn(235, 200, device=dev, requires_grad=True)
for fused in (False, True):
    try:
        opt = torch.optim.SGD([ent, rel], lr=1.0, fused=fused) if fused else torch.optim.SGD([ent, rel], lr=1.0)
    except Exception as e:
        print("fused", fused, "unsupported", e); continue
    ent.grad = torch.randn_like(ent); rel.grad = torch.randn_like(rel)
    for _ in range(10): opt.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(200): opt.step()
    e.record(); torch.cuda.synchronize()
    print("fused", fused, s.elapsed_time(e) / 200 * 1000, "us per step")
