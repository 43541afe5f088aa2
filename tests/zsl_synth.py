"""Synthetic zero-shot graphs for the Extractor tests (names, id maps, tasks, candidate lists
shaped like origin_data/FB15K-237-ZS; no reference data needed)."""
import numpy as np
import torch


def make_graph(n_ent=300, n_rel=12, n_train=900, n_test=120, n_test_rel=3, seed=0, oov=True):
    rng = np.random.default_rng(seed)
    ents = [f"/m/e{i}" for i in range(n_ent)]
    rels = [f"/r/{j}" for j in range(n_rel)]
    # id maps in a shuffled order (symbol numbering follows dict order, not ids)
    ent2id = {e: int(i) for e, i in zip(ents, rng.permutation(n_ent))}
    rel2id = {r: int(i) for r, i in zip(rels, rng.permutation(n_rel))}
    if oov:  # the reference maps carry "" / "OOV" keys that get no symbol
        ent2id = {"OOV": n_ent, **ent2id}
        rel2id = {"": n_rel, **rel2id}
    test_rels = rels[:n_test_rel]
    train_rels = rels[n_test_rel:]

    def tasks(rel_names, n):
        out = {}
        for k in range(n):
            r = rel_names[k % len(rel_names)]
            a, b = rng.choice(n_ent, 2, replace=False)
            out.setdefault(r, []).append([ents[a], r, ents[b]])
        return out

    train_tasks = tasks(train_rels, n_train)
    test_tasks = tasks(test_rels, n_test)
    n_nodes = len(ent2id)
    return dict(ents=ents, rels=rels, ent2id=ent2id, rel2id=rel2id, train_tasks=train_tasks,
                test_tasks=test_tasks, n_nodes=n_nodes, n_rel_ids=len(rel2id), rng=rng)


def embeddings(g, dim, seed=1):
    gen = torch.Generator().manual_seed(seed)
    return torch.rand((g["n_nodes"], dim), generator=gen), torch.rand((g["n_rel_ids"], dim), generator=gen)


def candidates(g, n_cand=40, seed=2):
    """test_candidates {rel: {"head\\trel\\ttrue": [true, c1, ...]}} (gen_mode_candidates.py)."""
    rng = np.random.default_rng(seed)
    ents = g["ents"]
    out = {}
    for rel, triples in g["test_tasks"].items():
        known = {}
        for h, r, t in triples:
            known.setdefault(h, set()).add(t)
        d = {}
        for h, r, t in triples:
            key = f"{h}\t{r}\t{t}"
            if key in d:
                continue
            pool = [ents[i] for i in rng.choice(len(ents), n_cand + 10, replace=False)]
            lst = [t] + [e for e in pool if e not in known[h] and e != t][:n_cand]
            d[key] = lst
        out[rel] = d
    return out


def init_extractor(ex, seed=3, bias_scale=0.1):
    """xavier_normal_ weights (module/utils.py:119-123) and small non-zero biases, so every bias
    path is exercised; LayerNorm affine randomised too."""
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in ex.named_parameters():
            if name.startswith("symbol_emb"):
                continue
            if p.dim() == 2:
                fan_out, fan_in = p.shape
                std = (2.0 / (fan_in + fan_out)) ** 0.5
                p.copy_(torch.randn(p.shape, generator=gen) * std)
            elif "layer_norm.weight" in name:
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=gen))
            else:
                p.copy_(bias_scale * torch.randn(p.shape, generator=gen))
