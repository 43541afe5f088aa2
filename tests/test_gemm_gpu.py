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
