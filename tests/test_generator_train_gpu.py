"""GPU parity of the generator's training form: forward with the spectral-norm power
iteration and the HIP backward (mmre_generator_backward) against the float64 torch-autograd
restatement of spectral_norm.py:39-89 / model.py:679-686 (oracle/zsl_gan.py). Tolerance
1e-4 relative to each gradient's largest magnitude."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("n,D,train", [(512, 200, True), (20, 200, False), (37, 256, True), (9, 1, True)])
def test_generator_backward_matches_autograd(n, D, train):
    import zsl_gan as og
    from mmre.generator import RelationGenerator
    torch.manual_seed(n + D)
    gen = RelationGenerator(384, 15, D)
    with torch.no_grad():
        gen.ln_a.normal_(1.0, 0.1)
        gen.ln_b.normal_(0.0, 0.1)
    layers = [(L.weight_orig.detach().double().clone().requires_grad_(), L.bias.detach().double().clone()
               .requires_grad_(), L.weight_u.double().clone(), L.weight_v.double().clone())
              for L in (gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2)]
    a = gen.ln_a.detach().double().clone().requires_grad_()
    b = gen.ln_b.detach().double().clone().requires_grad_()
    cls, noise = torch.randn(n, 384), 0.1 * torch.randn(n, 15)
    up = torch.randn(n, D)
    ref, uv = og.generator(noise.double(), cls.double(), layers, a, b, train)
    (ref * up.double()).sum().backward()
    gen = gen.to(DEV).train(train)
    out = gen(cls.to(DEV), noise.to(DEV))
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())
    got = [gen.generate_fc_layer.weight_orig, gen.generate_fc_layer.bias, gen.des_rel_map_layer1.weight_orig,
           gen.des_rel_map_layer1.bias, gen.des_rel_map_layer2.weight_orig, gen.des_rel_map_layer2.bias,
           gen.ln_a, gen.ln_b]
    want = [layers[0][0], layers[0][1], layers[1][0], layers[1][1], layers[2][0], layers[2][1], a, b]
    for i, (g, w) in enumerate(zip(got, want)):
        gg = g.grad.detach().cpu().double()
        ww = w.grad if w.grad is not None else torch.zeros_like(gg)  # D = 1: LN is the identity
        scale = ww.abs().max().item()
        # + 1e-6 absolute: a 1x1 SN weight (D = 1) is scale-invariant, its exact gradient is 0
        assert (gg - ww).abs().max().item() <= 1e-4 * scale + 1e-6, (i, (gg - ww).abs().max().item(), scale)
    for L, (u2, v2) in zip((gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2), uv):
        assert np.allclose(L.weight_u.cpu().numpy(), u2.numpy(), atol=1e-5)
        assert np.allclose(L.weight_v.cpu().numpy(), v2.numpy(), atol=1e-5)
