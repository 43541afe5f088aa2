"""GPU checks of the small split-K GEMM (csrc/gemm.hip) behind the GAN Discriminator's products
and their autograd (mmre/gemm.py): values against float64, strided (transposed) operands, the
K-split path, and first and second derivatives against torch's float64 autograd -- the
gradient penalty differentiates the Discriminator's gradient (module/utils.py:692-707)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _close(got, ref, tol=1e-5):
    got, ref = got.detach().double().cpu(), ref.detach().double().cpu()
    assert (got - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("m,k,n", [(512, 200, 200), (200, 512, 200), (206, 512, 200), (512, 200, 1), (1, 7, 3),
                                   (33, 1000, 65), (5, 0, 4)])
def test_mm_values_and_strides(m, k, n):
    from mmre import _lib
    from mmre.gemm import mm_hip
    g = torch.Generator().manual_seed(m * 7 + k + n)
    a = torch.randn(m, k, generator=g)
    b = torch.randn(k, n, generator=g)
    ref = a.double() @ b.double()
    _close(mm_hip(a.to(DEV), b.to(DEV)), ref)
    # transposed views: a stored (k, m), b stored (n, k)
    at = a.t().contiguous().to(DEV).t()
    bt = b.t().contiguous().to(DEV).t()
    _close(mm_hip(at, bt), ref)
    torch.cuda.synchronize()
    assert _lib.lib().mmre_gemm_splits(m, n, k) >= 1


def test_mm_double_backward_matches_float64():
    """grad of a gradient-penalty-like objective through mm (create_graph=True)."""
    from mmre.gemm import mm
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(64, 48, generator=g)
    w0 = torch.randn(40, 48, generator=g) / 7
    c0 = torch.randn(30, 40, generator=g)

    def objective(x, w, c, matmul):
        h = torch.tanh(matmul(x, w.t()))
        s = matmul(h, c.t())
        gx = torch.autograd.grad(s.sum(), x, create_graph=True)[0]
        return ((gx.norm(2, dim=1) - 1) ** 2).mean()

    xs, ws, cs = (t.double().requires_grad_() for t in (x0, w0, c0))
    ref = objective(xs, ws, cs, torch.matmul)
    ref.backward()
    xd, wd, cd = (t.to(DEV).requires_grad_() for t in (x0, w0, c0))
    out = objective(xd, wd, cd, mm)
    out.backward()
    torch.cuda.synchronize()
    _close(out, ref, 1e-4)
    for a, b in ((xd, xs), (wd, ws), (cd, cs)):
        _close(a.grad, b.grad, 1e-4)


def test_mm_bias_and_splits():
    from mmre.gemm import gemm_splits, mm
    g = torch.Generator().manual_seed(5)
    a, b, bias = torch.randn(512, 200, generator=g), torch.randn(200, 384, generator=g), torch.randn(384, generator=g)
    ref = a.double() @ b.double() + bias.double()
    _close(mm(a.to(DEV), b.to(DEV), bias.to(DEV)), ref)
    assert 1 <= gemm_splits(512, 200, 200) <= 8 and gemm_splits(32, 32, 4096) == 8 and gemm_splits(7, 7, 31) == 1


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("out,inn", [(200, 200), (1, 200), (384, 399)])
def test_sn_weight_matches_spectral_norm(train, out, inn):
    """mmre.gemm.sn_weight == torch.nn.utils.spectral_norm's weight (spectral_norm.py:39-89):
    W / sigma, the in-place u, v update of the power iteration, and dL/dW_orig."""
    from mmre.gemm import sn_weight
    torch.manual_seed(out + inn)
    ref = torch.nn.utils.spectral_norm(torch.nn.Linear(inn, out)).double()
    mod = torch.nn.utils.spectral_norm(torch.nn.Linear(inn, out)).to(DEV)
    with torch.no_grad():
        mod.weight_orig.copy_(ref.weight_orig.float())
        mod.weight_u.copy_(ref.weight_u.float())
        mod.weight_v.copy_(ref.weight_v.float())
    ref.train(train)
    mod.train(train)
    up = torch.randn(out, inn)
    ref(torch.zeros(1, inn, dtype=torch.float64))  # runs the hook: ref.weight = W / sigma
    (ref.weight * up.double()).sum().backward()
    w = sn_weight(mod)
    (w * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    _close(w, ref.weight, 1e-5)
    _close(mod.weight_u, ref.weight_u, 1e-5)
    _close(mod.weight_v, ref.weight_v, 1e-5)
    _close(mod.weight_orig.grad, ref.weight_orig.grad, 1e-4)


def test_layer_norm_first_and_second_order():
    """mmre.gemm.layer_norm == LayerNormalization (module/submodule.py:58-77): values, the
    first-order backward (HIP) and a create_graph double backward (torch ops)."""
    from mmre.gemm import layer_norm
    from module.submodule import LayerNormalization
    torch.manual_seed(11)
    ln = LayerNormalization(200)
    with torch.no_grad():
        ln.a_2.normal_(1.0, 0.2)
        ln.b_2.normal_(0.0, 0.2)
    z0, up = torch.randn(300, 200) * 3 + 1, torch.randn(300, 200)
    import torch.nn as nn
    import zsl_gan

    class _RefLN(nn.Module):  # the reference formula in float64 torch ops (oracle/zsl_gan.py)
        def __init__(self):
            super().__init__()
            self.a_2 = nn.Parameter(ln.a_2.detach().double().clone())
            self.b_2 = nn.Parameter(ln.b_2.detach().double().clone())

        def forward(self, z):
            return zsl_gan.layer_norm_ref(z, self.a_2, self.b_2, ln.eps)

    lref = _RefLN()
    zr = z0.double().requires_grad_()
    out_r = lref(zr)
    (out_r * up.double()).sum().backward()
    lhip = ln.to(DEV)
    zd = z0.to(DEV).requires_grad_()
    out_d = layer_norm(lhip, zd)
    (out_d * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    _close(out_d, out_r, 1e-5)
    for got, want in ((zd.grad, zr.grad), (lhip.a_2.grad, lref.a_2.grad), (lhip.b_2.grad, lref.b_2.grad)):
        _close(got, want, 1e-4)

    def penalty(z, f):
        o = f(z)
        gz = torch.autograd.grad((o * o).sum(), z, create_graph=True)[0]
        return (gz.norm(2, dim=1) - 1).pow(2).mean()

    lref.zero_grad()
    lhip.zero_grad()
    zr = z0.double().requires_grad_()
    pr = penalty(zr, lref)
    pr.backward()
    zd = z0.to(DEV).requires_grad_()
    pd = penalty(zd, lambda z: layer_norm(lhip, z))
    pd.backward()
    torch.cuda.synchronize()
    _close(pd, pr, 1e-4)
    for got, want in ((zd.grad, zr.grad), (lhip.a_2.grad, lref.a_2.grad), (lhip.b_2.grad, lref.b_2.grad)):
        _close(got, want, 1e-4)
