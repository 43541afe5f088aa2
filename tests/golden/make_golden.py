"""make_golden.py -- generate the golden fixtures from the REFERENCE itself.

Runs only in the build container (needs /root/reference). It never runs on the
GPU box and nothing from the reference travels: only the numbers it writes
under tests/golden/*.npz and the synthetic datasets under tests/golden/data/.

What is executed from the reference (read-only, bytecode writing disabled):
* OpenKE Python models/strategy/loss, imported from /root/reference/OpenKE
  (TransE.py, DistMult.py, ComplEx.py, RotatE.py, strategy/NegativeSampling.py,
  loss/MarginLoss.py) -- no stubs needed;
* OpenKE's C++ core compiled from /root/reference/OpenKE/openke/base/Base.cpp by
  oracle/Makefile into oracle/_ref/Base.so (flags of OpenKE/openke/make.sh:2);
* repo-level module/NegativeSampling.py, module/loss.py, module/model.py
  (UnifiedModel.generate), module/submodule.py, module/spectral_norm.py, imported
  with sys.modules stubs for third-party packages absent from the image and not on
  the hot path (skimage, torch_geometric, ml_collections, wandb, torchvision) and
  for the absent module/vqgan.py. The frozen M3AE text
  encoder (out of scope) is replaced by a module returning a fixed CLS input;
* sklearn.metrics.pairwise.cosine_similarity for the ZSL ranking rule.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes
import importlib.machinery
import json
import os
import subprocess
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
DATA = os.path.join(HERE, "data")


# ------------------------------------------------------------ datasets ------
def write_openke_dataset(path, n_ent, n_rel, n_train, n_valid, n_test, seed):
    """Synthetic dataset in OpenKE's file format (OpenKE/README.md:126-141, Reader.h:53-317):
    first line = count, then `h t r` per line. Relations get head/tail type pools so the
    filter sets and type constraints are non-trivial."""
    rng = np.random.default_rng(seed)
    os.makedirs(path, exist_ok=True)
    pools_h = [rng.choice(n_ent, size=int(rng.integers(5, n_ent // 3)), replace=False) for _ in range(n_rel)]
    pools_t = [rng.choice(n_ent, size=int(rng.integers(5, n_ent // 3)), replace=False) for _ in range(n_rel)]
    total = n_train + n_valid + n_test
    trip = set()
    out = []
    while len(out) < total:
        r = int(rng.integers(n_rel))
        h = int(rng.choice(pools_h[r]))
        t = int(rng.choice(pools_t[r]))
        if (h, r, t) in trip:
            continue
        trip.add((h, r, t))
        out.append((h, t, r))
    out = np.array(out, np.int64)
    rng.shuffle(out)
    splits = {"train2id.txt": out[:n_train], "valid2id.txt": out[n_train:n_train + n_valid],
              "test2id.txt": out[n_train + n_valid:]}
    for name, arr in splits.items():
        with open(os.path.join(path, name), "w") as f:
            f.write(f"{len(arr)}\n")
            for h, t, r in arr:
                f.write(f"{h} {t} {r}\n")
    with open(os.path.join(path, "entity2id.txt"), "w") as f:
        f.write(f"{n_ent}\n")
        for i in range(n_ent):
            f.write(f"e{i}\t{i}\n")
    with open(os.path.join(path, "relation2id.txt"), "w") as f:
        f.write(f"{n_rel}\n")
        for i in range(n_rel):
            f.write(f"r{i}\t{i}\n")
    # type_constrain.txt (format read by Reader.h:266-317): line 1 = #rel; then per relation
    # "rel n ids..." for allowed heads and the same for allowed tails.
    allt = out
    with open(os.path.join(path, "type_constrain.txt"), "w") as f:
        f.write(f"{n_rel}\n")
        for r in range(n_rel):
            hs = sorted(set(allt[allt[:, 2] == r][:, 0].tolist()))
            ts = sorted(set(allt[allt[:, 2] == r][:, 1].tolist()))
            f.write(f"{r}\t{len(hs)}\t" + "\t".join(map(str, hs)) + "\n")
            f.write(f"{r}\t{len(ts)}\t" + "\t".join(map(str, ts)) + "\n")


# ------------------------------------------------------------ Base.so -------
def load_base():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "Base.so"))
    P = ctypes.c_void_p
    I = ctypes.c_int64
    lib.setInPath.argtypes = [ctypes.c_char_p]
    lib.setWorkThreads.argtypes = [I]
    lib.setBern.argtypes = [I]
    lib.getHeadBatch.argtypes = [P, P, P]
    lib.getTailBatch.argtypes = [P, P, P]
    lib.testHead.argtypes = [P, I, I]
    lib.testTail.argtypes = [P, I, I]
    lib.test_link_prediction.argtypes = [I]
    for n in ["getTestLinkMRR", "getTestLinkMR", "getTestLinkHit10", "getTestLinkHit3", "getTestLinkHit1"]:
        getattr(lib, n).argtypes = [I]
        getattr(lib, n).restype = ctypes.c_float
    for n in ["getEntityTotal", "getRelationTotal", "getTestTotal", "getTrainTotal"]:
        getattr(lib, n).restype = I
    lib.sampling.argtypes = [P, P, P, P, I, I, I, I, ctypes.c_bool, ctypes.c_bool, ctypes.c_bool]
    return lib


def fglob(lib, name):
    return ctypes.c_float.in_dll(lib, name).value


def base_setup(lib, path, threads=1, bern=0):
    lib.setInPath((path.rstrip("/") + "/").encode())
    lib.setWorkThreads(threads)
    lib.setBern(bern)
    lib.randReset()
    lib.importTrainFiles()
    lib.importTestFiles()
    lib.importTypeFiles()


def seeds_now(lib, threads):
    p = ctypes.c_void_p.in_dll(lib, "next_random").value
    return np.ctypeslib.as_array((ctypes.c_uint64 * threads).from_address(p)).copy()


# ------------------------------------------------------------ reference -----
def import_openke():
    sys.path.insert(0, os.path.join(REF, "OpenKE"))
    from openke.module.model import TransE, DistMult, ComplEx, RotatE  # noqa: E402
    from openke.module.loss import MarginLoss  # noqa: E402
    from openke.module.strategy import NegativeSampling  # noqa: E402
    return dict(TransE=TransE, DistMult=DistMult, ComplEx=ComplEx, RotatE=RotatE, MarginLoss=MarginLoss,
                NegativeSampling=NegativeSampling)


def install_stubs():
    import torch.nn as nn

    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    class ConfigDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError:
                raise AttributeError(k)

        def __setattr__(self, k, v):
            self[k] = v

        def copy_and_resolve_references(self):
            return ConfigDict(self)

    class _RGCN(nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

    mc = stub("ml_collections", ConfigDict=ConfigDict)
    cd = stub("ml_collections.config_dict", placeholder=lambda *a, **k: None)
    cd.config_dict = cd
    mc.config_dict = cd
    cf = stub("ml_collections.config_flags")
    cf.config_flags = cf
    mc.config_flags = cf
    sk = stub("skimage")
    sk.io = stub("skimage.io")
    sk.color = stub("skimage.color", gray2rgb=None, rgba2rgb=None)
    tg = stub("torch_geometric")
    tg.nn = stub("torch_geometric.nn", RGCNConv=_RGCN)
    tg.loader = stub("torch_geometric.loader", NeighborSampler=object)
    tg.data = stub("torch_geometric.data", Data=object, Dataset=object)
    stub("wandb")
    tv = stub("torchvision")
    tv.transforms = stub("torchvision.transforms")
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import module  # noqa: F401  (namespace package of the reference)
    stub("module.vqgan", get_image_tokenizer=None)


# ------------------------------------------------------------ fixtures ------
def link_fixture(lib, ok, path, tag):
    """Reference Tester loop (Tester.py:70-91) with getHeadBatch/predict/testHead per query."""
    base_setup(lib, path)
    E = lib.getEntityTotal()
    R = lib.getRelationTotal()
    T = lib.getTestTotal()
    ph = np.zeros(E, np.int64)
    pt = np.zeros(E, np.int64)
    pr = np.zeros(E, np.int64)
    cfgs = [
        ("transe", dict(cls="TransE", kw=dict(dim=32, p_norm=1, norm_flag=True))),
        ("transe_nonorm_margin", dict(cls="TransE", kw=dict(dim=32, p_norm=1, norm_flag=False, margin=5.0))),
        ("transe_l2", dict(cls="TransE", kw=dict(dim=32, p_norm=2, norm_flag=True))),
        ("distmult", dict(cls="DistMult", kw=dict(dim=32))),
        ("complex", dict(cls="ComplEx", kw=dict(dim=24))),
        ("rotate", dict(cls="RotatE", kw=dict(dim=16, margin=6.0, epsilon=2.0))),
    ]
    res = {"E": E, "R": R, "T": T}
    for i, (name, cfg) in enumerate(cfgs):
        torch.manual_seed(100 + i)
        model = ok[cfg["cls"]](ent_tot=E, rel_tot=R, **cfg["kw"])
        sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
        for tc in (0, 1):
            lib.initTest()
            heads, tails = [], []
            preds_h, preds_t = [], []
            qh, qr, qt = [], [], []
            for idx in range(T):
                lib.getHeadBatch(ph.ctypes.data, pt.ctypes.data, pr.ctypes.data)
                qt.append(int(pt[0]))
                qr.append(int(pr[0]))
                data = {"batch_h": torch.from_numpy(ph.copy()), "batch_t": torch.from_numpy(pt.copy()),
                        "batch_r": torch.from_numpy(pr.copy()), "mode": "head_batch"}
                s = np.ascontiguousarray(model.predict(data), dtype=np.float32)
                before = [fglob(lib, n) for n in ["l_rank", "l_filter_rank", "l_rank_constrain",
                                                  "l_filter_rank_constrain"]]
                lib.testHead(s.ctypes.data, idx, tc)
                after = [fglob(lib, n) for n in ["l_rank", "l_filter_rank", "l_rank_constrain",
                                                 "l_filter_rank_constrain"]]
                heads.append([int(round(a - b)) - 1 for a, b in zip(after, before)])
                preds_h.append(s)
                lib.getTailBatch(ph.ctypes.data, pt.ctypes.data, pr.ctypes.data)
                qh.append(int(ph[0]))
                data = {"batch_h": torch.from_numpy(ph.copy()), "batch_t": torch.from_numpy(pt.copy()),
                        "batch_r": torch.from_numpy(pr.copy()), "mode": "tail_batch"}
                s = np.ascontiguousarray(model.predict(data), dtype=np.float32)
                before = [fglob(lib, n) for n in ["r_rank", "r_filter_rank", "r_rank_constrain",
                                                  "r_filter_rank_constrain"]]
                lib.testTail(s.ctypes.data, idx, tc)
                after = [fglob(lib, n) for n in ["r_rank", "r_filter_rank", "r_rank_constrain",
                                                 "r_filter_rank_constrain"]]
                tails.append([int(round(a - b)) - 1 for a, b in zip(after, before)])
                preds_t.append(s)
            lib.test_link_prediction(tc)
            metrics = np.array([lib.getTestLinkMRR(tc), lib.getTestLinkMR(tc), lib.getTestLinkHit10(tc),
                                lib.getTestLinkHit3(tc), lib.getTestLinkHit1(tc)], np.float32)
            key = f"{name}_tc{tc}"
            res[f"{key}_head_counts"] = np.array(heads, np.int64)
            res[f"{key}_tail_counts"] = np.array(tails, np.int64)
            res[f"{key}_metrics"] = metrics
            if tc == 0:
                res[f"{name}_pred_head"] = np.stack(preds_h)
                res[f"{name}_pred_tail"] = np.stack(preds_t)
        res["qh"] = np.array(qh, np.int64)
        res["qr"] = np.array(qr, np.int64)
        res["qt"] = np.array(qt, np.int64)
        for k, v in sd.items():
            res[f"{name}.{k}"] = v
    np.savez_compressed(os.path.join(HERE, f"link_{tag}.npz"), **res)
    print("link fixture", tag, "E", E, "R", R, "T", T)


def sampler_fixture(lib, path, tag):
    res = {}
    cases = [
        ("t4_b64_k3_bern0", dict(threads=4, B=64, neg=3, negrel=0, mode=0, bern=0)),
        ("t3_b70_k2_bern1", dict(threads=3, B=70, neg=2, negrel=1, mode=0, bern=1)),
        ("t8_b97_k5_m-1", dict(threads=8, B=97, neg=5, negrel=0, mode=-1, bern=0)),
        ("t2_b33_k4_m1", dict(threads=2, B=33, neg=4, negrel=0, mode=1, bern=0)),
    ]
    for name, c in cases:
        base_setup(lib, path, threads=c["threads"], bern=c["bern"])
        res[f"{name}_seeds0"] = seeds_now(lib, c["threads"])
        n = c["B"] * (1 + c["neg"] + c["negrel"])
        for step in range(3):
            bh = np.zeros(n, np.int64)
            bt = np.zeros(n, np.int64)
            br = np.zeros(n, np.int64)
            by = np.zeros(n, np.float32)
            lib.sampling(bh.ctypes.data, bt.ctypes.data, br.ctypes.data, by.ctypes.data, c["B"], c["neg"],
                         c["negrel"], c["mode"], True, False, False)
            res[f"{name}_step{step}"] = np.stack([bh, bt, br]).astype(np.int64)
            res[f"{name}_y{step}"] = by
        res[f"{name}_seeds_end"] = seeds_now(lib, c["threads"])
        res[f"{name}_cfg"] = np.array([c["threads"], c["B"], c["neg"], c["negrel"], c["mode"], c["bern"]],
                                      np.int64)
        res[f"{name}_train_total"] = np.array(lib.getTrainTotal(), np.int64)
    np.savez_compressed(os.path.join(HERE, f"sampler_{tag}.npz"), **res)
    print("sampler fixture", tag)


def strategy_fixture(ok):
    """OpenKE NegativeSampling(TransE/DistMult, MarginLoss) forward + gradients (Trainer.py:43-54)."""
    res = {}
    E, R, B, k = 300, 17, 40, 5
    rng = np.random.default_rng(7)
    for i, (name, cls, kw, loss_kw, regul) in enumerate([
        ("transe", "TransE", dict(dim=32, p_norm=1, norm_flag=True), dict(margin=5.0), 0.0),
        ("transe_nonorm", "TransE", dict(dim=32, p_norm=1, norm_flag=False), dict(margin=3.0), 0.5),
        ("transe_adv", "TransE", dict(dim=32, p_norm=1, norm_flag=True), dict(margin=5.0, adv_temperature=1.0), 0.0),
        ("distmult", "DistMult", dict(dim=32), dict(margin=5.0), 0.25),
        ("complex", "ComplEx", dict(dim=16), dict(margin=4.0), 0.1),
        ("rotate", "RotatE", dict(dim=16, margin=6.0, epsilon=2.0), dict(margin=6.0, adv_temperature=2.0), 0.0),
    ]):
        torch.manual_seed(300 + i)
        model = ok[cls](ent_tot=E, rel_tot=R, **kw)
        strat = ok["NegativeSampling"](model=model, loss=ok["MarginLoss"](**loss_kw), batch_size=B,
                                       regul_rate=regul)
        h = rng.integers(0, E, B * (1 + k))
        t = rng.integers(0, E, B * (1 + k))
        r = np.tile(rng.integers(0, R, B), 1 + k)
        data = {"batch_h": torch.from_numpy(h), "batch_t": torch.from_numpy(t), "batch_r": torch.from_numpy(r),
                "batch_y": torch.zeros(len(h)), "mode": "normal"}
        for p in model.parameters():
            p.grad = None
        loss = strat(data)
        loss.backward()
        score = model(data).detach().numpy()
        res[f"{name}_h"] = h
        res[f"{name}_t"] = t
        res[f"{name}_r"] = r
        res[f"{name}_loss"] = np.array(loss.item(), np.float64)
        res[f"{name}_score"] = score
        for pn, p in model.named_parameters():
            if p.requires_grad:
                res[f"{name}.{pn}"] = p.detach().numpy().copy()
                res[f"{name}.grad.{pn}"] = (p.grad.numpy().copy() if p.grad is not None
                                            else np.zeros_like(p.detach().numpy()))
    res["E"], res["R"], res["B"], res["k"] = E, R, B, k
    np.savez_compressed(os.path.join(HERE, "strategy.npz"), **res)
    print("strategy fixture")


def repo_fixture():
    """Repo-level module/NegativeSampling.py + module/loss.py + UnifiedModel.generate."""
    install_stubs()
    import module.NegativeSampling as NSmod
    import module.loss as Lmod
    import module.model as MM
    from module.spectral_norm import spectral_norm
    from module.submodule import LayerNormalization
    import torch.nn as nn
    res = {}
    rng = np.random.default_rng(11)

    class _M:
        num_relations = 23
        dim = 48

    args = types.SimpleNamespace(image_loss_weight=0.7, text_loss_weight=0.5, gcn_loss_weight=0.7,
                                 contrastive_loss_weight=0.5)
    N, B, k = 60, 12, 10
    x = rng.standard_normal((N, 48)).astype(np.float32)
    heads = rng.integers(0, N - 1, B)
    tails = rng.integers(0, N - 1, B)
    etype = rng.integers(0, 23, B)
    # whole_triples as [h_list, r_list, t_list] of GLOBAL ids (local_global_id maps local -> global)
    glob = rng.permutation(1000)[:N]
    wh = rng.integers(0, 1000, 400).tolist() + glob[heads].tolist()
    wt = rng.integers(0, 1000, 400).tolist() + glob[tails].tolist()
    wr = rng.integers(0, 23, 400).tolist() + etype.tolist()
    torch.manual_seed(5)
    margin = Lmod.MarginLoss(margin=3.0)
    ns = NSmod.NegativeSampling(args, [wh, wr, wt], model=_M(), loss_fn=margin, regul_rate=0.5, neg_ent=k)
    # expanded edges: fixed sampled negatives (the reference's sampler uses unseeded `random`, P13)
    eh = np.concatenate([heads, rng.integers(0, N - 1, B * k)]).astype(np.int32)
    et = np.concatenate([tails, rng.integers(0, N - 1, B * k)]).astype(np.int32)
    rel = rng.standard_normal((B, 48)).astype(np.float32)
    rel_exp = torch.from_numpy(rel).repeat(1 + k, 1)
    xt = torch.from_numpy(x)
    ei = torch.from_numpy(np.stack([eh, et]))
    score = ns.scoring_fn(None, xt, rel_exp, ei, None)
    p = ns._get_positive_score(score, B)
    n = ns._get_negative_score(score, B)
    loss_res = margin(p, n)
    struct = loss_res
    struct += ns.regul_rate * ns.regularization(xt, rel_exp, ei, None)
    res.update(x=x, eh=eh, et=et, rel=rel, score=score.numpy(), p=p.numpy(), n=n.numpy(),
               struct_loss=np.array(struct.item(), np.float64), gcn_loss=np.array(loss_res.item(), np.float64))
    res["regul"] = np.array(ns.regularization(xt, rel_exp, ei, None).item(), np.float64)
    # distmult _calc, head/tail batch forms of _calc
    res["score_distmult"] = ns._calc(xt[eh], xt[et], rel_exp, score_model="distmult").numpy()
    # adversarial MarginLoss (module/loss.py:19-23)
    adv = Lmod.MarginLoss(adv_temperature=2.0, margin=3.0)
    res["adv_loss"] = np.array(adv(p, n).item(), np.float64)
    # evaluate (module/NegativeSampling.py:294-305) + main.evaluate rank rule (main.py:245-250)
    E, R, D = 500, 20, 48
    ent = rng.standard_normal((E, D)).astype(np.float32)
    relm = rng.standard_normal((R, D)).astype(np.float32)
    nq = 40
    qh = rng.integers(0, E, nq)
    qr = rng.integers(0, R, nq)
    off = [0]
    cids = []
    for q in range(nq):
        c = rng.choice(E, size=int(rng.integers(5, 120)), replace=False)
        cids.extend(c.tolist())
        off.append(len(cids))
    ranks = []
    ev_scores = []
    for q in range(nq):
        cand = cids[off[q]:off[q + 1]]
        hs = torch.from_numpy(ent[qh[q]]).repeat(len(cand), 1)
        rs = torch.from_numpy(relm[qr[q]]).repeat(len(cand), 1)
        ts = torch.from_numpy(ent[cand])
        s = ns.evaluate(h=hs, r=rs, t=ts)
        ev_scores.append(s.numpy())
        ps, nsc = s[0], s[1:]
        raw = torch.sum(nsc < ps, dim=0, dtype=torch.long)
        ties = torch.sum(nsc == ps, dim=0, dtype=torch.long)
        ranks.append(int(raw + ties // 2) + 1)
    res.update(ev_ent=ent, ev_rel=relm, ev_qh=qh, ev_qr=qr, ev_off=np.array(off), ev_cids=np.array(cids),
               ev_scores=np.concatenate(ev_scores), ev_ranks=np.array(ranks))
    # ZSL cosine ranking (zsl_module.py:699-706) with sklearn
    from sklearn.metrics.pairwise import cosine_similarity
    zs_ranks, zs_scores = [], []
    relvecs = rng.standard_normal((5, 20, 48)).astype(np.float32)
    z_off = [0]
    z_c = []
    z_rel = rng.integers(0, 5, 30)
    for q in range(30):
        c = rng.standard_normal((int(rng.integers(10, 200)), 48)).astype(np.float32)
        sc = cosine_similarity(c, relvecs[z_rel[q]]).mean(axis=1)
        order = list(np.argsort(sc))[::-1]
        zs_ranks.append(order.index(0) + 1)
        zs_scores.append(sc)
        z_c.append(c)
        z_off.append(z_off[-1] + len(c))
    res.update(zs_cand=np.concatenate(z_c), zs_off=np.array(z_off), zs_rel=z_rel, zs_relvecs=relvecs,
               zs_ranks=np.array(zs_ranks), zs_scores=np.concatenate(zs_scores))
    # UnifiedModel.generate (module/model.py:674-686) with the M3AE encoder replaced by a fixed CLS.
    for (tag, emb_dim, nrows, train) in [("g200_eval", 200, 20, False), ("g200_train", 200, 96, True),
                                        ("g256_eval", 256, 64, False)]:
        torch.manual_seed(17 if train else 13)
        um = MM.UnifiedModel.__new__(MM.UnifiedModel)
        nn.Module.__init__(um)
        red, nd = 384, 15
        um.generate_fc_layer = spectral_norm(nn.Linear(red + nd, red))
        um.des_rel_map_layer1 = spectral_norm(nn.Linear(red, emb_dim))
        um.des_rel_map_layer2 = spectral_norm(nn.Linear(emb_dim, emb_dim))
        um.layer_norm = LayerNormalization(emb_dim)
        with torch.no_grad():
            um.layer_norm.a_2.uniform_(0.5, 1.5)
            um.layer_norm.b_2.uniform_(-0.2, 0.2)
        cls = torch.randn(nrows, red)

        class _Enc(nn.Module):
            def forward_representation(self, image=None, text=None, text_padding_mask=None, deterministic=True):
                return cls, None

        um.M3AEmodel = _Enc()
        noise = 0.1 * torch.randn(nrows, nd)
        um.train(train)
        layers = []
        for ln in ["generate_fc_layer", "des_rel_map_layer1", "des_rel_map_layer2"]:
            m = getattr(um, ln)
            layers.append((m.weight_orig.detach().numpy().copy(), m.bias.detach().numpy().copy(),
                           m.weight_u.detach().numpy().copy(), m.weight_v.detach().numpy().copy()))
        out = um.generate(torch.zeros(nrows, 4, dtype=torch.int32), torch.zeros(nrows, 4), noise)
        res[f"{tag}_out"] = out.detach().numpy()
        res[f"{tag}_noise"] = noise.numpy()
        res[f"{tag}_cls"] = cls.numpy()
        res[f"{tag}_a"] = um.layer_norm.a_2.detach().numpy()
        res[f"{tag}_b"] = um.layer_norm.b_2.detach().numpy()
        for li, (w, b, u, v) in enumerate(layers):
            res[f"{tag}_W{li}"] = w
            res[f"{tag}_b{li}"] = b
            res[f"{tag}_u{li}"] = u
            res[f"{tag}_v{li}"] = v
            m = getattr(um, ["generate_fc_layer", "des_rel_map_layer1", "des_rel_map_layer2"][li])
            res[f"{tag}_u{li}_after"] = m.weight_u.detach().numpy().copy()
            res[f"{tag}_v{li}_after"] = m.weight_v.detach().numpy().copy()
        res[f"{tag}_train"] = np.array(int(train))
    np.savez_compressed(os.path.join(HERE, "repo.npz"), **res)
    print("repo fixture")


def main():
    for name, args in [("small", (257, 13, 3000, 150, 150, 1)), ("medium", (1500, 31, 20000, 500, 400, 2))]:
        p = os.path.join(DATA, name)
        write_openke_dataset(p, *args)
    lib = load_base()
    ok = import_openke()
    link_fixture(lib, ok, os.path.join(DATA, "small"), "small")
    sampler_fixture(lib, os.path.join(DATA, "small"), "small")
    sampler_fixture(lib, os.path.join(DATA, "medium"), "medium")
    strategy_fixture(ok)
    repo_fixture()


if __name__ == "__main__":
    main()
