"""The drop-in surfaces on the GPU: OpenKE's model/strategy/loss/Trainer/Tester/data API and
the repo's NegativeSampling / generator / main.evaluate, driven exactly like the reference's
example scripts (OpenKE/examples/train_transe_FB15K237.py) on the golden dataset."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SMALL = os.path.join(GOLDEN, "data", "small")


def _load_golden_weights(model, g, name):
    sd = {k[len(name) + 1:]: torch.from_numpy(v) for k, v in g.items() if k.startswith(name + ".")}
    model.load_state_dict(sd, strict=False)


@pytest.mark.parametrize("name,cls,kw", [
    ("transe", "TransE", dict(dim=32, p_norm=1, norm_flag=True)),
    ("transe_nonorm_margin", "TransE", dict(dim=32, p_norm=1, norm_flag=False, margin=5.0)),
    ("transe_l2", "TransE", dict(dim=32, p_norm=2, norm_flag=True)),
    ("distmult", "DistMult", dict(dim=32)),
    ("complex", "ComplEx", dict(dim=24)),
    ("rotate", "RotatE", dict(dim=16, margin=6.0, epsilon=2.0)),
])
@pytest.mark.parametrize("tc", [False, True])
def test_tester_matches_reference_metrics(golden, name, cls, kw, tc):
    """Tester.run_link_prediction on the reference's weights returns the reference Base.so's
    hit@{10,3,1} exactly (and MRR/MR when no near-tie, checked in test_link_gpu)."""
    import openke.module.model as M
    from openke.config import Tester
    from openke.data import TestDataLoader
    g = golden("link_small")
    dl = TestDataLoader(SMALL, "link")
    model = getattr(M, cls)(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), **kw)
    _load_golden_weights(model, g, name)
    tester = Tester(model=model, data_loader=dl, use_gpu=True)
    mrr, mr, hit10, hit3, hit1 = tester.run_link_prediction(type_constrain=tc)
    ref = g[f"{name}_tc{int(tc)}_metrics"]
    assert np.array_equal(np.array([hit10, hit3, hit1], np.float32), ref[2:])
    assert abs(mrr - ref[0]) < 1e-6 and abs(mr - ref[1]) < 1e-3


def test_predict_matches_reference_scores(golden):
    import openke.module.model as M
    from openke.config import Tester
    from openke.data import TestDataLoader
    g = golden("link_small")
    dl = TestDataLoader(SMALL, "link")
    for name, cls, kw in [("transe", "TransE", dict(dim=32)), ("rotate", "RotatE", dict(dim=16)),
                          ("complex", "ComplEx", dict(dim=24))]:
        model = getattr(M, cls)(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), **kw)
        _load_golden_weights(model, g, name)
        tester = Tester(model=model, data_loader=dl, use_gpu=True)
        for i, (dh, dt) in enumerate(dl):
            if i >= 5:
                break
            for data, side in ((dh, "head"), (dt, "tail")):
                got = tester.test_one_step(data)
                ref = g[f"{name}_pred_{side}"][i]
                assert np.all(np.abs(got - ref) <= 1e-4 * np.maximum(1, np.abs(ref))), (name, side, i)


def test_openke_training_example_runs():
    """train_transe_FB15K237.py flow on the small dataset: GPU sampler -> fused loss -> SGD,
    loss decreases; then link prediction."""
    from openke.config import Tester, Trainer
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    tdl = TrainDataLoader(in_path=SMALL, nbatches=10, threads=8, sampling_mode="normal", bern_flag=1,
                          filter_flag=1, neg_ent=25, neg_rel=0)
    transe = TransE(ent_tot=tdl.get_ent_tot(), rel_tot=tdl.get_rel_tot(), dim=32, p_norm=1, norm_flag=True)
    model = NegativeSampling(model=transe, loss=MarginLoss(margin=5.0), batch_size=tdl.get_batch_size())
    trainer = Trainer(model=model, data_loader=tdl, train_times=30, alpha=1.0, use_gpu=True)
    trainer.run()
    assert trainer.log[-1] < trainer.log[0]
    tester = Tester(model=transe, data_loader=TestDataLoader(SMALL, "link"), use_gpu=True)
    mrr, mr, hit10, hit3, hit1 = tester.run_link_prediction(type_constrain=False)
    assert 0.0 <= hit1 <= hit3 <= hit10 <= 1.0 and mr >= 1.0


@pytest.mark.parametrize("model_name,regul", [("transe", 0.0), ("transe", 0.25), ("distmult", 0.0),
                                              ("complex", 0.25), ("rotate", 0.0)])
def test_trainer_one_call_step_equals_per_batch_path(model_name, regul):
    """Trainer.run() on TransE / DistMult / ComplEx / RotatE + MarginLoss + SGD takes the one-call
    step (mmre_ns_step_openke_pipe / _gen_pipe): over 3 epochs of 10 batches its epoch losses,
    embedding tables and sampler states equal the per-batch path's (train_one_step: loader
    sampling, fused loss, backward, SGD) bit for bit."""
    import torch
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import ComplEx, DistMult, RotatE, TransE
    from openke.module.strategy import NegativeSampling
    runs = []
    for one_call in (True, False):
        torch.manual_seed(0)
        tdl = TrainDataLoader(in_path=SMALL, nbatches=10, threads=8, sampling_mode="normal", bern_flag=1,
                              filter_flag=1, neg_ent=25, neg_rel=0)
        E, R = tdl.get_ent_tot(), tdl.get_rel_tot()
        kg = {"transe": lambda: TransE(ent_tot=E, rel_tot=R, dim=32, p_norm=1, norm_flag=True),
              "distmult": lambda: DistMult(ent_tot=E, rel_tot=R, dim=32),
              "complex": lambda: ComplEx(ent_tot=E, rel_tot=R, dim=32),
              "rotate": lambda: RotatE(ent_tot=E, rel_tot=R, dim=32, margin=6.0, epsilon=2.0)}[model_name]()
        model = NegativeSampling(model=kg, loss=MarginLoss(margin=5.0), batch_size=tdl.get_batch_size(),
                                 regul_rate=regul)
        trainer = Trainer(model=model, data_loader=tdl, train_times=3, alpha=0.5, use_gpu=True)
        trainer.one_call_step = one_call
        trainer.run()
        assert trainer.used_one_call_step == one_call
        runs.append((list(trainer.log), [t.detach().clone() for t in kg._tables() if t is not None],
                     tdl.sampler.seeds.copy()))
    (la, ta, sa), (lb, tb, sb) = runs
    assert la == lb
    assert all(torch.equal(x, y) for x, y in zip(ta, tb))
    assert np.array_equal(sa, sb)


def test_cross_sampling_mode_trains():
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import SigmoidLoss
    from openke.module.model import RotatE
    from openke.module.strategy import NegativeSampling
    tdl = TrainDataLoader(in_path=SMALL, batch_size=128, threads=8, sampling_mode="cross", bern_flag=0,
                          filter_flag=1, neg_ent=8, neg_rel=0)
    rotate = RotatE(ent_tot=tdl.get_ent_tot(), rel_tot=tdl.get_rel_tot(), dim=16, margin=6.0, epsilon=2.0)
    model = NegativeSampling(model=rotate, loss=SigmoidLoss(adv_temperature=2), batch_size=tdl.get_batch_size(),
                             regul_rate=0.0)
    trainer = Trainer(model=model, data_loader=tdl, train_times=5, alpha=2e-5, use_gpu=True, opt_method="adam")
    trainer.run()
    assert np.isfinite(trainer.log).all()


def test_model_forward_backward_matches_reference(golden):
    """model(data) in 'normal' mode + autograd (OpenKE strategy graph) vs reference gradients."""
    import openke.module.model as M
    from openke.module.loss import MarginLoss
    from openke.module.strategy import NegativeSampling
    g = golden("strategy")
    B, k = int(g["B"]), int(g["k"])
    model = M.TransE(int(g["E"]), int(g["R"]), dim=32, p_norm=1, norm_flag=True).cuda()
    with torch.no_grad():
        model.ent_embeddings.weight.copy_(torch.from_numpy(g["transe.ent_embeddings.weight"]))
        model.rel_embeddings.weight.copy_(torch.from_numpy(g["transe.rel_embeddings.weight"]))
    data = {"batch_h": torch.from_numpy(g["transe_h"]).cuda(), "batch_t": torch.from_numpy(g["transe_t"]).cuda(),
            "batch_r": torch.from_numpy(g["transe_r"]).cuda(), "mode": "normal"}
    score = model(data)
    loss = MarginLoss(margin=5.0)(score[:B].view(-1, B).permute(1, 0), score[B:].view(-1, B).permute(1, 0))
    loss.backward()
    assert abs(loss.item() - float(g["transe_loss"])) < 1e-4
    ref = g["transe.grad.ent_embeddings.weight"]
    assert np.abs(model.ent_embeddings.weight.grad.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max()
    # and the fused strategy path gives the same loss
    model.zero_grad()
    strat = NegativeSampling(model=model, loss=MarginLoss(margin=5.0), batch_size=B)
    l2 = strat(data)
    assert abs(l2.item() - float(g["transe_loss"])) < 1e-4


def test_repo_negative_sampling_forward(golden):
    """module.NegativeSampling.forward with a stand-in upstream encoder returning the golden
    x_gcn / rel_emb; sampler -> fused loss -> total loss assembly (P9)."""
    import types
    from module.NegativeSampling import NegativeSampling
    from module.loss import MarginLoss
    g = golden("repo")
    dev = torch.device("cuda:0")
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    rel = torch.from_numpy(g["rel"]).to(dev).requires_grad_(True)
    B = rel.shape[0]

    class Enc(torch.nn.Module):
        num_relations, dim = 23, 48

        def forward(self, edge_index, edge_type, batch, deterministic=False):
            return x, rel, {"contrastive_loss": 0.0}

    args = types.SimpleNamespace(image_loss_weight=0.7, text_loss_weight=0.5, gcn_loss_weight=0.7,
                                 contrastive_loss_weight=0.5)
    rng = np.random.default_rng(11)
    N = 60
    glob = rng.permutation(1000)[:N]
    ns = NegativeSampling(args, [list(range(1000)), [0] * 1000, list(range(1000))], model=Enc(),
                          loss_fn=MarginLoss(margin=3.0), regul_rate=0.5, neg_ent=10)
    edge_index = torch.from_numpy(np.stack([g["eh"][:B], g["et"][:B]]).astype(np.int64)).to(dev)
    edge_type = torch.zeros(B, dtype=torch.int64, device=dev)
    loss, info = ns({i: int(glob[i]) for i in range(N)}, edge_index, edge_type, {})
    loss.backward()
    assert info["gcn_loss"] is info["struct_loss"]
    assert torch.isfinite(loss).item() and x.grad is not None and rel.grad is not None
    # evaluate(): TransE L1 of explicit rows equals the reference's NegativeSampling.evaluate
    ev = ns.evaluate(torch.from_numpy(g["ev_ent"][g["ev_qh"][:1]]).to(dev).repeat(5, 1),
                     torch.from_numpy(g["ev_rel"][g["ev_qr"][:1]]).to(dev).repeat(5, 1),
                     torch.from_numpy(g["ev_ent"][g["ev_cids"][:5]]).to(dev))
    assert np.allclose(ev.detach().cpu().numpy(), g["ev_scores"][:5], rtol=1e-4, atol=1e-4)


def test_main_evaluate_surface(golden, tmp_path, monkeypatch):
    """main.evaluate(args, ent_embs, rel_embs, e2id, r2id, model) reading
    origin_data/<dataset>/test/test_candidates.json, reproducing the reference's ranks."""
    import types

    import main
    g = golden("repo")
    off, cids = g["ev_off"], g["ev_cids"]
    e2id = {f"e{i}": i for i in range(g["ev_ent"].shape[0])}
    r2id = {f"r{i}": i for i in range(g["ev_rel"].shape[0])}
    cand = {}
    for q in range(len(g["ev_qh"])):
        rname = f"r{g['ev_qr'][q]}"
        key = f"e{g['ev_qh'][q]}\t{rname}\tq{q}"
        cand.setdefault(rname, {})[key] = [f"e{c}" for c in cids[off[q]:off[q + 1]]]
    d = tmp_path / "origin_data" / "TOY" / "test"
    d.mkdir(parents=True)
    (d / "test_candidates.json").write_text(json.dumps(cand))
    monkeypatch.chdir(tmp_path)
    res = main.evaluate(types.SimpleNamespace(dataset="TOY"), torch.from_numpy(g["ev_ent"]),
                        torch.from_numpy(g["ev_rel"]), e2id, r2id, None)
    # queries are grouped by relation in the json; compare as multisets per query key
    order = []
    for rname in cand:
        for key in cand[rname]:
            order.append(int(key.split("\tq")[1]))
    assert np.array_equal(res["ranks"], g["ev_ranks"][order])
