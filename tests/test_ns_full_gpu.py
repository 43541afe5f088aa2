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


def _c2_batch(c2_training, neg, skip=1):
    from mmre.sampler import OpenKESampler
    w, idx = c2_training
    smp = OpenKESampler(idx, DEV, bern=True)
    for _ in range(skip):
        smp.sample(2721, neg)
    return smp.sample(2721, neg)


@pytest.mark.parametrize("regul", [0.0, 0.5])
def test_fused_ns_gradients_are_bit_reproducible(c2_training, regul):
    """The TransE gradient has no float atomics (slots sorted by table row, one wave per row
    summing them in batch order): the same batch gives bit-identical gradient tables, run to
    run, and an upstream gradient G scales them exactly (the row-owner pass multiplies once)."""
    from mmre.ns import NSSpec, fused_ns_loss
    w, _ = c2_training
    b = _c2_batch(c2_training, 25)
    spec = NSSpec("transe", 200, norm_flag=True)
    grads = []
    for scale in (1.0, 1.0, 2.5):
        ent = w["ent"].to(DEV).requires_grad_(True)
        rel = w["rel"].to(DEV).requires_grad_(True)
        loss, _ = fused_ns_loss(spec, ent, rel, b["batch_h"], b["batch_t"], b["batch_r"], 2721, 25, 5.0, None, regul)
        (loss * scale).backward()
        grads.append((ent.grad.clone(), rel.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    assert torch.equal(grads[2][0], grads[0][0] * 2.5) and torch.equal(grads[2][1], grads[0][1] * 2.5)


def test_one_shot_abi_equals_autograd_pair(c2_training):
    """mmre_ns_forward_backward (forward + gradient, upstream 1, tables written without a fill)
    gives the autograd pair's loss, scores and gradients bit for bit."""
    from mmre._lib import call, lib, ptr, stream_ptr
    from mmre.ns import NSSpec, fused_ns_loss
    w, _ = c2_training
    b = _c2_batch(c2_training, 10, skip=2)
    B, k, d = 2721, 10, 200
    E, R = int(w["n_ent"]), int(w["n_rel"])
    ent = w["ent"].to(DEV).requires_grad_(True)
    rel = w["rel"].to(DEV).requires_grad_(True)
    loss, score = fused_ns_loss(NSSpec("transe", d, norm_flag=True), ent, rel, b["batch_h"], b["batch_t"],
                                b["batch_r"], B, k, 3.0, None, 0.5)
    loss.backward()
    e0, r0 = ent.detach(), rel.detach()
    work = torch.empty(int(lib().mmre_ns_fused_workspace(0, 1, B, k, E, R, d)), dtype=torch.float32, device=DEV)
    s1 = torch.empty(B * (1 + k), dtype=torch.float32, device=DEV)
    l1 = torch.empty(1, dtype=torch.float32, device=DEV)
    ge = torch.full_like(e0, float("nan"))  # poisoned: every row must be written
    gr = torch.full_like(r0, float("nan"))
    call("mmre_ns_forward_backward", 0, 1, 0.0, 0, ptr(e0), None, ptr(r0), None, E, R, d, 0.0, ptr(b["batch_h"]),
         ptr(b["batch_t"]), ptr(b["batch_r"]), B, k, 3.0, 0.0, 0.5, ptr(s1), ptr(l1), ptr(ge), None, ptr(gr), None,
         ptr(work), stream_ptr(DEV))
    torch.cuda.synchronize()
    assert torch.equal(l1[0], loss.detach()) and torch.equal(s1, score)
    assert torch.equal(ge, ent.grad) and torch.equal(gr, rel.grad)


@pytest.mark.parametrize("frac,p_norm,adv", [(0.05, 1, None), (0.05, 2, 1.0), (1.0, 1, None)])
def test_fused_ns_deferred_generic_rows(c2_training, frac, p_norm, adv):
    """Batches that are not OpenKE-shaped: negatives replaced by random (h, r, t) rows (sharing
    fewer than two rows with their positive), by a relation corruption, or by the positive
    itself. The fused kernel handles such rows in line (a row sharing fewer than two rows with
    its positive builds its x as its rows arrive; each of its rows that is not the positive's
    gets a slot); frac = 1.0 puts one in every positive. Loss, scores and gradients vs the
    float64 reference op sequence; the gradient tables stay bit-reproducible."""
    import ref_trainer
    from mmre.ns import NSSpec, fused_ns_loss
    w, _ = c2_training
    B, k, d = 2721, 25, 200
    E, R = int(w["n_ent"]), int(w["n_rel"])
    b = _c2_batch(c2_training, k)
    h, t, r = (b[x].clone() for x in ("batch_h", "batch_t", "batch_r"))
    g = torch.Generator().manual_seed(7)
    pos = torch.nonzero(torch.rand(B, generator=g) < frac).flatten()
    for i, j in enumerate(torch.randint(0, k, (len(pos),), generator=g).tolist()):
        row = int(pos[i]) + (j + 1) * B
        kind = i % 3
        if kind == 0:    # random row: the generic path
            h[row] = int(torch.randint(0, E, (1,), generator=g))
            t[row] = int(torch.randint(0, E, (1,), generator=g))
            r[row] = int(torch.randint(0, R, (1,), generator=g))
        elif kind == 1:  # relation corruption (shares h and t)
            h[row], t[row] = h[int(pos[i])], t[int(pos[i])]
            r[row] = (r[int(pos[i])] + 1) % R
        else:            # a copy of the positive
            h[row], t[row], r[row] = h[int(pos[i])], t[int(pos[i])], r[int(pos[i])]
    grads = []
    for _ in range(2):
        ent = w["ent"].to(DEV).requires_grad_(True)
        rel = w["rel"].to(DEV).requires_grad_(True)
        loss, score = fused_ns_loss(NSSpec("transe" if p_norm == 1 else "transe_l2", d, norm_flag=True), ent, rel, h, t, r, B, k,
                                    5.0, adv, 0.0)
        loss.backward()
        grads.append((ent.grad.clone(), rel.grad.clone()))
    torch.cuda.synchronize()
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    hc, tc, rc = h.cpu(), t.cpu(), r.cpu()
    e64 = w["ent"].double().requires_grad_(True)
    r64 = w["rel"].double().requires_grad_(True)
    ref_loss, ref_score = ref_trainer.transe_ns_loss(e64, r64, hc, tc, rc, B, 5.0, norm_flag=True, p_norm=p_norm,
                                                     adv_temperature=adv)
    ref_loss.backward()
    rs = ref_score.detach().numpy()
    assert np.abs(score.detach().cpu().numpy() - rs).max() <= 1e-4 * max(1.0, np.abs(rs).max())
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    for got, want in ((grads[0][0], e64.grad), (grads[0][1], r64.grad)):
        gw, gg = want.numpy(), got.cpu().double().numpy()
        assert np.linalg.norm(gg - gw) <= 1e-3 * np.linalg.norm(gw)


def _tables(model, w, seed=0):
    """Float32 tables of the C2 id space for another model (OpenKE-like init, seed fixed)."""
    g = torch.Generator().manual_seed(seed)
    E, R, d = int(w["n_ent"]), int(w["n_rel"]), 200
    u = lambda n, c, s: (torch.rand((n, c), generator=g) * 2 - 1) * s
    if model == "distmult":
        return {"ent": u(E, d, 0.5), "rel": u(R, d, 0.5)}
    if model == "complex":
        return {"ent": u(E, d, 0.3), "ent_im": u(E, d, 0.3), "rel": u(R, d, 0.3), "rel_im": u(R, d, 0.3)}
    return {"ent": u(E, 2 * d, 8.0 / (2 * d)), "rel": u(R, d, 8.0 / d)}   # RotatE: (margin + eps) / (2) d


@pytest.mark.parametrize("model,neg,margin,adv,regul", [
    ("distmult", 25, 5.0, None, 0.0), ("distmult", 10, 3.0, 1.0, 0.5),
    ("complex", 25, 5.0, None, 0.5), ("complex", 10, 3.0, 1.0, 0.0),
    ("rotate", 25, 5.0, None, 0.0), ("rotate", 10, 6.0, 1.0, 0.5)])
def test_other_models_row_owner_gradients_at_c2_shape(c2_training, model, neg, margin, adv, regul):
    """DistMult / ComplEx / RotatE at the C2 training shape (B 2,721, d 200): the row-owner
    gradient (no float atomics): loss, scores and gradients vs the float64 reference op sequence
    (oracle/ref_trainer.model_ns_loss) -- gradients within 1e-4 of the table's largest entry --
    and bit-identical gradient tables run to run."""
    import ref_trainer
    from mmre.link import rotate_phase_denom
    from mmre.ns import NSSpec, fused_ns_loss
    w, _ = c2_training
    B, d = 2721, 200
    b = _c2_batch(c2_training, neg)
    tabs = _tables(model, w)
    spec = NSSpec(model, d, model_margin=6.0 if model == "rotate" else None,
                  phase_denom=rotate_phase_denom(6.0, 2.0, d) if model == "rotate" else 0.0)
    runs = []
    for _ in range(2):
        T = {k: v.to(DEV).requires_grad_(True) for k, v in tabs.items()}
        loss, score = fused_ns_loss(spec, T["ent"], T["rel"], b["batch_h"], b["batch_t"], b["batch_r"], B, neg, margin,
                                    adv, regul, ent_im=T.get("ent_im"), rel_im=T.get("rel_im"))
        loss.backward()
        runs.append((loss.detach().clone(), score.clone(), {k: v.grad.clone() for k, v in T.items()}))
    torch.cuda.synchronize()
    for k in tabs:
        assert torch.equal(runs[0][2][k], runs[1][2][k]), k
    T64 = {k: v.double().requires_grad_(True) for k, v in tabs.items()}
    h, t, r = (b[x].cpu() for x in ("batch_h", "batch_t", "batch_r"))
    ref_loss, ref_score = ref_trainer.model_ns_loss(model, T64, h, t, r, B, margin, adv, regul, model_margin=6.0)
    ref_loss.backward()
    rs = ref_score.detach().numpy()
    assert np.abs(runs[0][1].cpu().numpy() - rs).max() <= 1e-4 * max(1.0, np.abs(rs).max())
    assert abs(float(runs[0][0]) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    for k in tabs:
        gw, gg = T64[k].grad.numpy(), runs[0][2][k].cpu().double().numpy()
        assert np.abs(gg - gw).max() <= 1e-4 * np.abs(gw).max(), (k, np.abs(gg - gw).max(), np.abs(gw).max())


@pytest.mark.parametrize("model", ["transe", "distmult", "complex", "rotate"])
def test_fused_sgd_step_equals_backward_then_step(c2_training, model):
    """fused_ns_loss(..., optimizer=mmre.optim.SGD): the backward applies the SGD step in its
    row-owner pass and step() skips the tables -- parameters and gradients bit-identical to the
    unfused backward() + step(), over three training steps."""
    from mmre.link import rotate_phase_denom
    from mmre.ns import NSSpec, fused_ns_loss
    from mmre.optim import SGD
    w, _ = c2_training
    B, k, d = 2721, 10, 200
    tabs = _tables(model, w) if model != "transe" else {"ent": w["ent"], "rel": w["rel"]}
    spec = NSSpec(model, d, norm_flag=model == "transe", model_margin=6.0 if model == "rotate" else None,
                  phase_denom=rotate_phase_denom(6.0, 2.0, d) if model == "rotate" else 0.0)
    batches = [_c2_batch(c2_training, k, skip=s) for s in (1, 2, 3)]
    out = []
    for fuse in (False, True):
        T = {n: v.to(DEV).clone().requires_grad_(True) for n, v in tabs.items()}
        opt = SGD(list(T.values()), lr=0.7)
        for b in batches:
            opt.zero_grad(set_to_none=True)
            loss, _ = fused_ns_loss(spec, T["ent"], T["rel"], b["batch_h"], b["batch_t"], b["batch_r"], B, k, 4.0,
                                    None, 0.25, ent_im=T.get("ent_im"), rel_im=T.get("rel_im"),
                                    optimizer=opt if fuse else None)
            loss.backward()
            if fuse:
                assert len(opt._fused_done) == len(T)
            opt.step()
        torch.cuda.synchronize()
        out.append({n: (v.detach().clone(), v.grad.clone()) for n, v in T.items()})
    for n in tabs:
        assert torch.equal(out[0][n][0], out[1][n][0]), n
        assert torch.equal(out[0][n][1], out[1][n][1]), n
        assert not torch.equal(out[0][n][0], tabs[n].to(DEV))


@pytest.mark.parametrize("model,n_pos", [("transe", 700), ("transe", 3000), ("distmult", 700), ("rotate", 3000)])
def test_hub_rows_ordered_deterministically(c2_training, model, n_pos):
    """Hub rows: every positive of a batch shares one relation, so that relation's bucket holds
    n_pos slots -- past the 64-slot bucket into the overflow list, ordered in LDS (700) or by
    the repeated-minimum fallback (3,000). Gradients vs the float64 reference, bit-reproducible."""
    import ref_trainer
    from mmre.link import rotate_phase_denom
    from mmre.ns import NSSpec, fused_ns_loss
    w, _ = c2_training
    k, d = 5, 200
    b = _c2_batch(c2_training, k)
    B0 = 2721
    sel = torch.arange(n_pos) % B0
    rows = torch.cat([sel + j * B0 for j in range(1 + k)]).to(DEV)
    h, t, r = (b[x][rows].clone() for x in ("batch_h", "batch_t", "batch_r"))
    r[:] = 17                                           # one hub relation
    tabs = _tables(model, w) if model != "transe" else {"ent": w["ent"], "rel": w["rel"]}
    spec = NSSpec(model, d, norm_flag=model == "transe", model_margin=6.0 if model == "rotate" else None,
                  phase_denom=rotate_phase_denom(6.0, 2.0, d) if model == "rotate" else 0.0)
    grads = []
    for _ in range(2):
        T = {n: v.to(DEV).clone().requires_grad_(True) for n, v in tabs.items()}
        loss, _ = fused_ns_loss(spec, T["ent"], T["rel"], h, t, r, n_pos, k, 5.0, None, 0.5, ent_im=T.get("ent_im"),
                                rel_im=T.get("rel_im"))
        loss.backward()
        grads.append({n: v.grad.clone() for n, v in T.items()})
    torch.cuda.synchronize()
    for n in tabs:
        assert torch.equal(grads[0][n], grads[1][n]), n
    T64 = {n: v.double().requires_grad_(True) for n, v in tabs.items()}
    hc, tc, rc = h.cpu(), t.cpu(), r.cpu()
    if model == "transe":
        ref_loss, _ = ref_trainer.transe_ns_loss(T64["ent"], T64["rel"], hc, tc, rc, n_pos, 5.0, norm_flag=True,
                                                 regul_rate=0.5)
    else:
        ref_loss, _ = ref_trainer.model_ns_loss(model, T64, hc, tc, rc, n_pos, 5.0, None, 0.5, model_margin=6.0)
    ref_loss.backward()
    for n in tabs:
        gw, gg = T64[n].grad.numpy(), grads[0][n].cpu().double().numpy()
        assert np.linalg.norm(gg - gw) <= 1e-4 * np.linalg.norm(gw), (n, np.linalg.norm(gg - gw), np.linalg.norm(gw))


@pytest.mark.parametrize("regul,adv,pipeline", [(0.0, None, False), (0.5, None, False), (0.0, 1.0, False),
                                                 (0.0, None, True), (0.5, None, True), (0.0, 1.0, True)])
def test_train_step_equals_the_autograd_path(c2_training, regul, adv, pipeline):
    """mmre_ns_step_openke (mmre.ns.OpenKETrainStep: sampler + pre-pass in one launch, the fused
    loss kernel, the row owner with SGD and the loss reduction) and its pipelined form
    (mmre_ns_step_openke_pipe: the row owner also draws the next batch and writes the norms of
    the rows it updates; two launches a step) against the drop-in path (OpenKESampler.sample +
    fused_ns_loss + backward + mmre.optim.SGD.step) over four steps at the C2 training shape:
    batches, losses, scores, gradients, parameters and LCG states bit-identical."""
    from mmre.ns import NSSpec, OpenKETrainStep, fused_ns_loss
    from mmre.optim import SGD
    from mmre.sampler import OpenKESampler
    w, idx = c2_training
    B, k, margin, lr = 2721, 25, 5.0, 1.0
    spec = NSSpec("transe", 200, norm_flag=True)
    ea = w["ent"].to(DEV).clone().requires_grad_(True)
    ra = w["rel"].to(DEV).clone().requires_grad_(True)
    eb = w["ent"].to(DEV).clone().requires_grad_(True)
    rb = w["rel"].to(DEV).clone().requires_grad_(True)
    sa = OpenKESampler(idx, DEV, bern=True)
    sb = OpenKESampler(idx, DEV, bern=True)
    opt = SGD([ea, ra], lr=lr)
    step = OpenKETrainStep(sb, spec, eb, rb, B, k, margin, lr, adv_temperature=adv, regul_rate=regul,
                           pipeline=pipeline)
    for i in range(4):
        ba = sa.sample(B, k)
        opt.zero_grad(set_to_none=True)
        la, sc_a = fused_ns_loss(spec, ea, ra, ba["batch_h"], ba["batch_t"], ba["batch_r"], B, k, margin, adv, regul,
                                 optimizer=opt)
        la.backward()
        opt.step()
        lb = step()
        torch.cuda.synchronize()
        for key in ("batch_h", "batch_t", "batch_r", "batch_y"):
            assert torch.equal(ba[key], step.batch[key]), (i, key)
        assert torch.equal(la.detach().reshape(1), lb.reshape(1)), (i, float(la), float(lb))
        assert torch.equal(sc_a, step.score), i
        assert torch.equal(ea.grad, eb.grad) and torch.equal(ra.grad, rb.grad), i
        assert torch.equal(ea.detach(), eb.detach()) and torch.equal(ra.detach(), rb.detach()), i
    if pipeline:  # the prefetch drew batch 5 already, into the other buffer
        b5 = sa.sample(B, k)
        assert step.batch is step._bufs[1]  # four steps: the last trained on parity 1's buffer
        torch.cuda.synchronize()
        for key in ("batch_h", "batch_t", "batch_r", "batch_y"):
            assert torch.equal(b5[key], step._bufs[0][key]), key
    assert np.array_equal(sa.seeds, sb.seeds)
    assert torch.equal(sa._seeds_dev, sb._seeds_dev)


def test_pipelined_train_step_falls_back_when_its_prefetch_is_stale(c2_training):
    """OpenKETrainStep(pipeline=True) uses the previous call's prefetched batch and pre-pass only
    while they are current: parameters changed in place between steps re-run the pre-pass (the
    prefetched batch is kept), a batch drawn from the sampler elsewhere (or a reseed) discards
    the prefetch and draws again; over a sequence with both, every step equals the unpipelined
    step on the same sampler history, and a pipelined two-graph replay equals eager steps."""
    from mmre.ns import NSSpec, OpenKETrainStep
    from mmre.sampler import OpenKESampler
    w, idx = c2_training
    B, k, margin, lr = 2721, 25, 5.0, 1.0
    spec = NSSpec("transe", 200, norm_flag=True)
    tabs = [w[x].to(DEV).clone().requires_grad_(True) for x in ("ent", "rel", "ent", "rel")]
    ea, ra, eb, rb = tabs
    sa, sb = OpenKESampler(idx, DEV, bern=True), OpenKESampler(idx, DEV, bern=True)
    plain = OpenKETrainStep(sa, spec, ea, ra, B, k, margin, lr, pipeline=False)
    pipe = OpenKETrainStep(sb, spec, eb, rb, B, k, margin, lr, pipeline=True)

    def both(tag):
        la, lb = plain(), pipe()
        torch.cuda.synchronize()
        for key in ("batch_h", "batch_t", "batch_r", "batch_y"):
            assert torch.equal(plain.batch[key], pipe.batch[key]), (tag, key)
        assert torch.equal(la.reshape(1), lb.reshape(1)), tag
        assert torch.equal(ea.grad, eb.grad) and torch.equal(ra.grad, rb.grad), tag
        assert torch.equal(ea.detach(), eb.detach()) and torch.equal(ra.detach(), rb.detach()), tag

    both("first")
    both("prefetched")
    with torch.no_grad():  # in-place parameter edits: the pre-pass runs again, the batch is kept
        for t in (ea, eb):
            t[:7].mul_(0.5)
    both("params edited")
    both("prefetched again")
    # a C-ABI writer between steps (mmre.optim.SGD: mmre_sgd_step through raw pointers) bumps the
    # tables' version counters like torch's in-place ops, so the pre-pass runs again
    from mmre.optim import SGD
    fb = SGD.fallback_steps
    for e_, r_ in ((ea, ra), (eb, rb)):
        v = e_._version
        SGD([e_, r_], lr=0.25).step()
        assert e_._version > v
    assert SGD.fallback_steps == fb  # the HIP step ran, not torch's
    both("mmre SGD between steps")
    both("prefetched after SGD")
    # another consumer draws from the samplers: the pipelined step's prefetched batch is stale
    # (it drew batch i + 1 before the other consumer drew) and is discarded -- both steps then
    # train on the next batch each sampler yields from its current state
    sb.seeds = sa.seeds  # the pipelined step's sampler reset to the plain one's state
    both("reseeded")
    # pipelined replays of two captured graphs (one per parity) equal eager pipelined steps
    both("before capture")
    graphs = []
    for _ in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            pipe()
        graphs.append(g)
    # the captures advanced the pipelined object's host state by two steps: replay both graphs
    # and run the plain step twice
    for g in graphs:
        g.replay()
        plain()
    torch.cuda.synchronize()
    assert torch.equal(ea.detach(), eb.detach()) and torch.equal(ra.detach(), rb.detach())
    assert torch.equal(plain.loss, pipe.loss)
    sa.sample(B, k)  # the pipelined sampler is one batch ahead (its prefetch)
    assert torch.equal(sa._seeds_dev, sb._seeds_dev) and np.array_equal(sa.seeds, sb.seeds)


@pytest.mark.parametrize("model,pipeline", [("distmult", True), ("complex", True), ("rotate", True),
                                            ("distmult", False)])
def test_generic_train_step_equals_the_autograd_path(c2_training, model, pipeline):
    """mmre_ns_step_openke_gen_pipe (OpenKETrainStep for DistMult / ComplEx / RotatE: the forward,
    the slot records, the row owner with SGD + the loss reduction + (pipelined) the next batch's
    sampler) against the drop-in path (OpenKESampler.sample + fused_ns_loss + backward +
    mmre.optim.SGD.step, the bench's --ns-autograd) over four steps at the C2 training shape:
    batches, losses, scores, gradients and parameters bit-identical."""
    from mmre.link import rotate_phase_denom
    from mmre.ns import NSSpec, OpenKETrainStep, fused_ns_loss
    from mmre.optim import SGD
    from mmre.sampler import OpenKESampler
    from mmre.workloads import zs_workload
    w0, idx = c2_training
    w = zs_workload("FB15K-237-ZS", model, 200)
    B, k, margin, lr, d = 2721, 25, 5.0, 1.0, 200
    if model == "rotate":
        spec = NSSpec("rotate", d, model_margin=6.0, phase_denom=rotate_phase_denom(6.0, 2.0, d))
    else:
        spec = NSSpec(model, d)
    names = [n for n in ("ent", "rel", "ent_im", "rel_im") if n in w]
    ta = {n: w[n].to(DEV).clone().requires_grad_(True) for n in names}
    tb = {n: w[n].to(DEV).clone().requires_grad_(True) for n in names}
    sa, sb = OpenKESampler(idx, DEV, bern=True), OpenKESampler(idx, DEV, bern=True)
    opt = SGD(list(ta.values()), lr=lr)
    step = OpenKETrainStep(sb, spec, tb["ent"], tb["rel"], B, k, margin, lr, pipeline=pipeline,
                           ent_im=tb.get("ent_im"), rel_im=tb.get("rel_im"))
    for i in range(4):
        ba = sa.sample(B, k)
        opt.zero_grad(set_to_none=True)
        la, sc_a = fused_ns_loss(spec, ta["ent"], ta["rel"], ba["batch_h"], ba["batch_t"], ba["batch_r"], B, k, margin,
                                 optimizer=opt, ent_im=ta.get("ent_im"), rel_im=ta.get("rel_im"))
        la.backward()
        opt.step()
        lb = step()
        torch.cuda.synchronize()
        for key in ("batch_h", "batch_t", "batch_r", "batch_y"):
            assert torch.equal(ba[key], step.batch[key]), (i, key)
        assert torch.equal(la.detach().reshape(1), lb.reshape(1)), (i, float(la), float(lb))
        assert torch.equal(sc_a, step.score), i
        for n in names:
            assert torch.equal(ta[n].grad, tb[n].grad), (i, n)
            assert torch.equal(ta[n].detach(), tb[n].detach()), (i, n)
    if pipeline:
        sa.sample(B, k)  # the prefetch drew batch 5
    assert torch.equal(sa._seeds_dev, sb._seeds_dev) and np.array_equal(sa.seeds, sb.seeds)
