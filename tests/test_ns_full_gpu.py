"""The negative-sampling training path at the C2 training shape (B = 2,721
positives, neg_ent 25 and 10, d = 200, TransE p=1 norm_flag) on the GPU: the bit-exact sampler's
batch, the fused margin loss (mmre.ns) and its gradients into the dense tables against the
reference's op sequence evaluated in float64 on the same batch (oracle/ref_trainer.py, pinned to
the reference strategy's golden loss and gradients). Tolerances: scores 1e-4 relative to
max(1, |s|) (north_star), loss 1e-5 relative, gradients 1e-4 of the largest gradient entry
(float32 sums of up to ~10^4 contributions per row, in atomic order) on every table row that
no sign-ambiguous element touches: the L1 norm's subgradient sign(x) flips between float32
and float64 where |x| is within rounding of 0 (~30 of the 14 M elements of a batch), so rows
fed by an element with |x| < 1e-7 are held to the relative Frobenius bound instead (1e-3)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def c2_training():
    from mmre.data import TrainIndex
    from mmre.workloads import zs_workload
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    idx = TrainIndex(w["filter_h"], w["filter_t"], w["filter_r"], w["n_ent"], w["n_rel"])
    return w, idx


@pytest.mark.parametrize("neg,margin,adv,regul", [(25, 5.0, None, 0.0), (10, 3.0, None, 0.5), (25, 5.0, 1.0, 0.0)])
def test_fused_ns_at_c2_shape_matches_reference(c2_training, neg, margin, adv, regul):
    import ref_trainer
    from mmre.ns import NSSpec, fused_ns_loss
    from mmre.sampler import OpenKESampler
    w, idx = c2_training
    B, d = 2721, 200
    smp = OpenKESampler(idx, DEV, bern=True)
    smp.sample(B, neg)                       # advance past the first batch: a mid-epoch batch
    b = smp.sample(B, neg)
    ent = w["ent"].to(DEV).requires_grad_(True)
    rel = w["rel"].to(DEV).requires_grad_(True)
    loss, score = fused_ns_loss(NSSpec("transe", d, norm_flag=True), ent, rel, b["batch_h"], b["batch_t"],
                                b["batch_r"], B, neg, margin, adv, regul)
    loss.backward()
    torch.cuda.synchronize()
    h, t, r = (b[k].cpu() for k in ("batch_h", "batch_t", "batch_r"))
    # a sampler batch in the reference's layout: negative j of positive i at row i + (j + 1) B
    assert torch.equal(r[:B].repeat(neg), r[B:])
    assert bool(((h[B:] == h[:B].repeat(neg)) | (t[B:] == t[:B].repeat(neg))).all())
    e64 = w["ent"].double().requires_grad_(True)
    r64 = w["rel"].double().requires_grad_(True)
    ref_loss, ref_score = ref_trainer.transe_ns_loss(e64, r64, h, t, r, B, margin, norm_flag=True,
                                                     adv_temperature=adv, regul_rate=regul)
    ref_loss.backward()
    rs = ref_score.detach().numpy()
    assert np.abs(score.cpu().numpy() - rs).max() <= 1e-4 * max(1.0, np.abs(rs).max())
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    # rows fed by a sign-ambiguous element (|x| < 1e-7, x = (h^ + r^) - t^ of some batch row)
    with torch.no_grad():
        nz = lambda v: v / v.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        x = (nz(e64[h]) + nz(r64[r])) - nz(e64[t])
        amb = (x.abs() < 1e-7).any(1).numpy()
    skip_ent = np.zeros(w["n_ent"], bool)
    skip_ent[h.numpy()[amb]] = True
    skip_ent[t.numpy()[amb]] = True
    skip_rel = np.zeros(w["n_rel"], bool)
    skip_rel[r.numpy()[amb]] = True
    assert skip_ent.sum() <= 400
    for got, want, skip in ((ent.grad, e64.grad, skip_ent), (rel.grad, r64.grad, skip_rel)):
        gw, gg = want.numpy(), got.cpu().double().numpy()
        err = np.abs(gg - gw)[~skip].max()
        assert err <= 1e-4 * np.abs(gw).max(), (err, np.abs(gw).max())
        assert np.linalg.norm(gg - gw) <= 1e-3 * np.linalg.norm(gw)
    # rows never touched by the batch get exactly zero gradient
    touched = np.zeros(w["n_ent"], bool)
    touched[h.numpy()] = True
    touched[t.numpy()] = True
    assert not ent.grad.cpu().numpy()[~touched].any()
