"""The reference's main.py trainer surface (main.py:32-342) on this build's path.

* `main(args)` (main.py:32-215): dataset -> UnifiedModel -> repo NegativeSampling
  (MarginLoss(3.0), neg_ent 10) -> ZSLmodule; the per-step loop over sampled edge batches
  (GPU filtered negative sampler + fused HIP margin loss, gradients into the entity table and
  through the relation branch's spectral-norm layers), Adam + CosineAnnealingWarmRestarts, and
  every save_epochs: save_checkpoint, generate_ent_embed / generate_rel_embed('seen'),
  ZSLmodule.update_embed + ZSLmodule.train (GAN + eval). Differences forced by the path's
  scope: the entity representations come from a trainable structure table (the strategy's
  `ent_encoder`) instead of M3AE's image/text branch + RGCN (outside this path), and batches
  are drawn like torch_geometric's NeighborSampler (batch_size seed nodes, up to sample_size
  incoming edges each, main.py:93-99) by a host sampler (torch_geometric is not a dependency).
* `evaluate(args, ent_embs, rel_embs, e2id, r2id, model, mode)` (main.py:217-272): candidate
  ranking of every (head, relation) query of <mode>/<mode>_candidates.json with
  NegativeSampling.evaluate's TransE L1 score and rank = #(s < p) + #(s == p) // 2 + 1, all
  queries in one GPU launch (csrc/candidates.hip); prints the reference's lines.
* `run_evaluate(args)` + `__main__` (main.py:274-342): `python main.py [flags]` trains;
  `python main.py --evaluate [--pretrained_model_name X]` loads the checkpoint, builds the
  embedding tables, runs ZSLmodule.train and ZSLmodule.eval.
"""
import json
import os
import os.path as osp
from collections import deque

import numpy as np
import torch
import torch.nn as nn

from mmre.candidates import candidate_rank_transe

DATA_ROOT = "./origin_data"
SAVE_ROOT = "./saved_models"


def build_candidates(test_candidates, e2id, r2id):
    qh, qr, off, ids, rel_names, rel_of_q = [], [], [0], [], [], []
    for query in test_candidates.keys():
        rel_names.append(query)
        for e1_rel, tails in test_candidates[query].items():
            head, rela, _ = e1_rel.split("\t")
            qh.append(e2id[head])
            qr.append(r2id[rela])
            ids.extend(e2id[t] for t in tails)
            off.append(len(ids))
            rel_of_q.append(len(rel_names) - 1)
    return (np.array(qh, np.int64), np.array(qr, np.int64), np.array(off, np.int64), np.array(ids, np.int64),
            rel_names, np.array(rel_of_q, np.int64))


def evaluate(args, ent_embs, rel_embs, e2id, r2id, model=None, mode="test", test_candidates=None, device=None,
             data_root=DATA_ROOT):
    if test_candidates is None:
        data_path = osp.join(data_root, args.dataset)
        with open(os.path.join(data_path, f"{mode}/{mode}_candidates.json"), "r") as f:
            test_candidates = json.load(f)
    print("Start evaluation!\n")
    if model is not None:
        model.eval()
        if hasattr(model, "model") and hasattr(model.model, "set_evaluate"):
            model.model.eval()
            model.model.set_evaluate(True)
    dev = torch.device(device or "cuda:0")
    qh, qr, off, ids, rel_names, rel_of_q = build_candidates(test_candidates, e2id, r2id)
    to = lambda a: torch.as_tensor(a).to(dev)
    ent = torch.as_tensor(ent_embs, dtype=torch.float32).to(dev)
    rel = torch.as_tensor(rel_embs, dtype=torch.float32).to(dev)
    ranks = candidate_rank_transe(ent, rel, to(qh), to(qr), to(off), to(ids)).cpu().numpy().astype(np.int64)
    for i, query in enumerate(rel_names):
        tr = [int(x) for x in ranks[rel_of_q == i]]
        n = len(tr)
        print("Relation: %s| Number %d | mrr: %.4f | hit1: %.4f | hit3: %.4f | hit10: %.4f " % (
            query, len(test_candidates[query]), sum(1.0 / r for r in tr) / n,
            sum(1.0 if r <= 1 else 0.0 for r in tr) / n, sum(1.0 if r <= 3 else 0.0 for r in tr) / n,
            sum(1.0 if r <= 10 else 0.0 for r in tr) / n))
    rl = [int(x) for x in ranks]
    mrr = sum(1.0 / r for r in rl) / len(rl)
    hits = [sum(1.0 if r <= k else 0.0 for r in rl) / len(rl) for k in (1, 3, 10)]
    print(f"[Final Scores] MRR: {mrr} \tHits@1: {hits[0]} \tHits@3: {hits[1]} \tHits@10: {hits[2]}")
    return {"mrr": mrr, "hit1": hits[0], "hit3": hits[1], "hit10": hits[2], "ranks": ranks}


class EdgeBatches:
    """NeighborSampler(edge_index, sizes=[sample_size], batch_size, shuffle=True) as the loop
    consumes it (main.py:93-99, 126-151): per step, batch_size seed nodes of a shuffled node
    order, up to sample_size of each seed's incoming edges drawn without replacement; local ids
    number the seeds first, then the other endpoints in order of appearance. Yields
    (n_id int64 global ids, local edge_index (2, m), edge type (m,))."""

    def __init__(self, edge_index, edge_type, num_nodes, batch_size, sample_size, seed=0):
        ei = np.asarray(edge_index, np.int64)
        self.src, self.dst = ei[0], ei[1]
        self.etype = np.asarray(edge_type, np.int64)
        self.num_nodes, self.batch_size, self.sample_size = int(num_nodes), int(batch_size), int(sample_size)
        order = np.argsort(self.dst, kind="stable")
        self.by_dst = order
        self.start = np.searchsorted(self.dst[order], np.arange(self.num_nodes + 1))
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return (self.num_nodes + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        perm = self.rng.permutation(self.num_nodes)
        for i in range(len(self)):
            seeds = perm[i * self.batch_size:(i + 1) * self.batch_size]
            picked = []
            for s in seeds:
                a, b = self.start[s], self.start[s + 1]
                if b > a:
                    k = min(self.sample_size, b - a)
                    picked.append(self.by_dst[a + self.rng.choice(b - a, k, replace=False)])
            e = np.concatenate(picked) if picked else np.zeros(0, np.int64)
            n_id = list(seeds)
            local = {int(g): j for j, g in enumerate(n_id)}
            for g in self.src[e]:
                if int(g) not in local:
                    local[int(g)] = len(n_id)
                    n_id.append(int(g))
            src = np.array([local[int(g)] for g in self.src[e]], np.int64)
            dst = np.array([local[int(g)] for g in self.dst[e]], np.int64)
            yield np.asarray(n_id, np.int64), np.stack([src, dst]) if len(e) else np.zeros((2, 0), np.int64), \
                self.etype[e]


def _build(args, data_root, device, neg_ent):
    from module.data import ZSDataset
    from module.loss import MarginLoss
    from module.model import UnifiedModel
    from module.NegativeSampling import NegativeSampling
    from module.zsl_module import ZSLmodule
    data_path = osp.join(data_root, args.dataset)
    dataset = ZSDataset(data_path, train_file="train_tasks_zsl.json")
    print("Entity Number:", dataset.num_nodes)
    part_model = UnifiedModel(args=args, hidden_channels=200, dataset=dataset, num_relations=dataset.num_relations,
                              noise_dim=args.noise_dim)
    model = NegativeSampling(args=args, whole_triples=dataset.triples, model=part_model,
                             loss_fn=MarginLoss(margin=3.0), neg_ent=neg_ent, sampling_mode="normal").to(device)
    # the structure encoder standing in for M3AE's image/text branch + RGCN (see the docstring)
    model.ent_encoder = nn.Embedding(dataset.num_nodes, args.emb_dim).to(device)
    nn.init.xavier_uniform_(model.ent_encoder.weight.data)
    zslmodule = ZSLmodule(args=args, data_path=data_path, r2id=dataset.r2id, e2id=dataset.e2id, device=device,
                          dataset=dataset).to(device)
    return dataset, model, zslmodule


def _train_step(model, dataset, optimizer, n_id, edge_index, edge_type, device):
    """One step of main.py:126-157. Its autograd graph dies with this frame: a graph kept alive
    past the loop would keep the parameters' AccumulateGrad nodes bound to this stream, which
    the GAN step's hipGraph capture (ZSLmodule.train) cannot record."""
    batch_data = dataset.generate_batch(n_id, edge_type)
    batch_data["rel_des"] = batch_data["rel_des"].to(device)
    batch_data["rel_des_padding_mask"] = batch_data["rel_des_padding_mask"].to(device)
    batch_data["x_gcn"] = model.ent_encoder(torch.as_tensor(n_id, device=device))
    optimizer.zero_grad()
    loss, info = model(local_global_id={k: int(v) for k, v in enumerate(n_id)},
                       edge_index=torch.as_tensor(edge_index, device=device),
                       edge_type=torch.as_tensor(edge_type, device=device), batch=batch_data)
    loss.backward()
    optimizer.step()
    return loss.item()


def main(args, data_root=DATA_ROOT, save_root=SAVE_ROOT, max_steps_per_epoch=None):
    from module.utils import generate_ent_embed, generate_rel_embed, set_random_seed
    device = torch.device("cuda:" + str(args.cuda) if int(args.cuda) >= 0 else "cpu")
    set_random_seed(args.seed)
    print("Start dataset preprocessing!")
    print("Start Model Instantiation!")
    dataset, model, zslmodule = _build(args, data_root, device, neg_ent=10)
    if args.pretrained_model_name != "":
        print(f"Loading pretrained model:{args.pretrained_model_name}")
        state_dict = torch.load(f"{save_root}/{args.dataset}/{args.pretrained_model_name}.ckpt", map_location=device,
                                weights_only=True)
        del state_dict["model.generate_fc_layer.weight_orig"]
        del state_dict["model.generate_fc_layer.weight_v"]
        model.load_state_dict(state_dict, strict=False)
    print("Finish Model Instantiation!")
    graph = dataset.get_struc_dataset()
    loader = EdgeBatches(graph.edge_index, graph.edge_type, graph.num_nodes, args.batch_size, args.sample_size,
                         seed=args.seed)
    steps_per_epoch = len(loader)
    print("Average steps per epoch is:", steps_per_epoch)
    optimizer = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=args.lr_maximum)
    scheduler = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(
        optimizer, T_0=max(1, args.lr_warmup_epochs * steps_per_epoch // args.accumulate_grad_steps), T_mult=2,
        eta_min=args.lr_minimum)
    losses = deque([], steps_per_epoch)
    history = []
    os.makedirs(osp.join(save_root, args.dataset), exist_ok=True)
    print("Start Fusion Training!\n")
    for epoch in range(args.epochs):
        model.train()
        model.model.train()
        for step, (n_id, edge_index, edge_type) in enumerate(loader):
            if max_steps_per_epoch is not None and step >= max_steps_per_epoch:
                break
            if edge_index.shape[1] == 0:
                continue
            losses.append(_train_step(model, dataset, optimizer, n_id, edge_index, edge_type, device))
            scheduler.step(epoch * steps_per_epoch + step)
        print(f"epoch{epoch + args.start_epoch + 1} loss is {np.mean(losses) if losses else float('nan')}!")
        history.append(float(np.mean(losses)) if losses else float("nan"))
        losses.clear()
        if (epoch + args.start_epoch + 1) % args.save_epochs == 0:
            print(f"\n save model at epoch{epoch + args.start_epoch + 1}!")
            model.save_checkpoint(f"{save_root}/{args.dataset}/epoch{epoch + args.start_epoch + 1}_"
                                  f"{args.saved_model_name}.ckpt")
            model.model.set_evaluate(True)
            ent_embs = generate_ent_embed(args, dataset, model, device)
            rel_embs = generate_rel_embed(dataset, model, None, device, "seen")
            zslmodule.update_embed(ent_embs, rel_embs)
            zslmodule.train(model.model)
            for param in model.model.parameters():
                param.requires_grad = True
            for param in model.model.M3AEmodel.parameters():  # the text encoder stays frozen here
                param.requires_grad = False
            model.model.set_evaluate(False)
    print("Finish Training\n")
    model.save_checkpoint(f"{save_root}/{args.saved_model_name}.ckpt")
    return dict(losses=history, model=model, zslmodule=zslmodule, dataset=dataset)


def run_evaluate(args, data_root=DATA_ROOT, save_root=SAVE_ROOT):
    """The --evaluate branch (main.py:278-342)."""
    from module.utils import generate_ent_embed, generate_rel_embed
    device = torch.device("cuda:" + str(args.cuda) if int(args.cuda) >= 0 else "cpu")
    dataset, model, zslmodule = _build(args, data_root, device, neg_ent=1)
    if args.pretrained_model_name != "":
        print(f"Loading pretrained model:{args.pretrained_model_name}")
        model.load_checkpoint(f"{save_root}/{args.dataset}/{args.pretrained_model_name}.ckpt", device=device)
    ent_embs = generate_ent_embed(args, dataset, model, device)
    rel_embs = generate_rel_embed(dataset, model, None, device, "seen")
    torch.save({"ent_embs": ent_embs, "rel_embs": rel_embs}, "./temp_embs.pt")  # (main.py:328-331 pickles them)
    model.model.set_evaluate(True)
    for param in model.model.parameters():
        param.requires_grad = False
    zslmodule.update_embed(ent_embs, rel_embs)
    zslmodule.train(generate_model=model.model)
    return zslmodule.eval(generate_model=model.model, mode="test", meta=True, load_pretrain=False)


if __name__ == "__main__":
    from args import read_options
    _args = read_options()
    if not _args.evaluate:
        main(_args)
    else:
        run_evaluate(_args)
