"""Rows backward at wide embeddings: mmre_score_rows_backward -- the backward of
the repo scoring path and of every non-MarginLoss / cross-mode model(data) step
(NegativeSampling.forward -> Model.forward -> mmre.ns.score_rows) -- at dim 1,024 and 2,048,
against float64 autograd of the reference op sequences (TransE.py:46-60 with norm_flag,
DistMult.py:34-44, ComplEx.py:20-27). The reference's own example trains TransE at dim 1,024
with SigmoidLoss and cross sampling (OpenKE/examples/train_transe_WN18_adv_sigmoidloss.py)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _score64(model, T, h, t, r):
    import torch.nn.functional as F
    if model == "transe":
        hv, tv, rv = (F.normalize(x, 2, -1) for x in (T["ent"][h], T["ent"][t], T["rel"][r]))
        return torch.norm((hv + rv) - tv, 1, -1)
    if model == "distmult":
        return torch.sum((T["ent"][h] * T["rel"][r]) * T["ent"][t], -1)
    er, ei, rr, ri = T["ent"], T["ent_im"], T["rel"], T["rel_im"]
    return torch.sum(er[h] * er[t] * rr[r] + ei[h] * ei[t] * rr[r] + er[h] * ei[t] * ri[r] - ei[h] * er[t] * ri[r], -1)


@pytest.mark.parametrize("model,dim", [("transe", 1024), ("distmult", 1024), ("complex", 1024), ("transe", 2048)])
def test_score_rows_backward_wide(model, dim):
    from mmre.ns import NSSpec, score_rows
    g = torch.Generator().manual_seed(dim + len(model))
    E, R, n = 3000, 40, 4096
    names = ["ent", "rel"] + (["ent_im", "rel_im"] if model == "complex" else [])
    base = {k: (torch.rand((E if k.startswith("ent") else R, dim), generator=g) - 0.5) * 0.2 for k in names}
    h, t, r = torch.randint(0, E, (n,), generator=g), torch.randint(0, E, (n,), generator=g), \
        torch.randint(0, R, (n,), generator=g)
    g_up = torch.linspace(-1.0, 1.0, n) / n
    spec = NSSpec(model, dim, norm_flag=model == "transe")
    grads = []
    for _ in range(2):   # bit-reproducible (slots + row owner, no float atomics)
        T = {k: v.to(DEV).clone().requires_grad_(True) for k, v in base.items()}
        s = score_rows(spec, T["ent"], T["rel"], h.to(DEV), t.to(DEV), r.to(DEV), T.get("ent_im"), T.get("rel_im"))
        (s * g_up.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        grads.append({k: T[k].grad.clone() for k in names})
    T64 = {k: v.double().requires_grad_(True) for k, v in base.items()}
    s64 = _score64(model, T64, h, t, r)
    assert (s.detach().cpu().double() - s64.detach()).abs().max().item() <= 1e-4 * max(1.0, s64.abs().max().item())
    (s64 * g_up.double()).sum().backward()
    for k in names:
        assert torch.equal(grads[0][k], grads[1][k]), k
        gw, gg = T64[k].grad.numpy(), grads[0][k].cpu().double().numpy()
        # Frobenius: an L1 element within rounding of 0 may take the other subgradient sign
        assert np.linalg.norm(gg - gw) <= 1e-4 * np.linalg.norm(gw), (k, np.linalg.norm(gg - gw), np.linalg.norm(gw))
