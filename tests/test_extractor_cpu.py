"""CPU checks of the ZSL Extractor's host side: the symbol / neighbourhood tables
(ZSLGraph, numpy) equal the oracle's literal restatement of load_embed / build_connection /
get_meta (zsl_module.py:208-287), and the C ABI exports the Extractor entry points."""
import numpy as np
import pytest
import torch

from zsl_synth import embeddings, make_graph


@pytest.mark.parametrize("max_nb", [5, 50])
def test_graph_tables_match_oracle(max_nb):
    import zsl_extractor as ox
    from module.zsl_module import ZSLGraph
    g = make_graph(seed=4)
    ent, rel = embeddings(g, 16)
    G = ZSLGraph(g["rel2id"], g["ent2id"], g["train_tasks"], g["test_tasks"], ent, rel, max_neighbor=max_nb)
    s2i, vec = ox.load_embed(g["rel2id"], g["ent2id"], ent.numpy(), rel.numpy())
    assert G.symbol2id == s2i and list(G.symbol2id) == list(s2i)
    assert G.symbol2vec.dtype == vec.dtype and np.array_equal(G.symbol2vec, vec)
    conn, deg = ox.build_connection(g["train_tasks"], g["test_tasks"], g["ent2id"], s2i, len(s2i) - 1, max_nb)
    assert np.array_equal(G.connections, conn)
    assert all(G.e1_degrees[i] == deg[i] for i in range(len(g["ent2id"])))
    assert (G.e1_degrees == 0).any()  # isolated nodes (and the OOV id)
    assert max_nb != 5 or (G.e1_degrees == max_nb).any()  # truncated lists
    left, right = [3, 7, 7, 0], [1, 2, 5, 9]
    for a, b in zip(G.get_meta(left, right), ox.get_meta(conn, deg, left, right)):
        assert a.dtype == b.dtype and torch.equal(a, b)
    for e, i in g["ent2id"].items():
        assert G.ent_sym[i] == s2i.get(e, len(s2i) - 1)


def test_extractor_symbols_exported():
    import ctypes
    from mmre import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in ("mmre_extractor_pack_size", "mmre_extractor_pack", "mmre_extractor_nodes", "mmre_extractor_encode",
              "mmre_extractor_targets", "mmre_rank_desc"):
        assert hasattr(L, n)
    lib = _lib.lib()
    assert lib.mmre_extractor_pack_size(7) == -1
    assert lib.mmre_extractor_pack_size(200) > 2 * 400 * 200


def test_extractor_requires_eval_mode():
    from mmre._lib import MMREError
    from module.zsl_module import Extractor
    ex = Extractor(64, 10, np.zeros((11, 64)))
    ex.train()
    with pytest.raises(MMREError):
        ex.encode_pairs(torch.zeros((1, 2), dtype=torch.long), None)


def test_gan_batch_generator_invariants():
    """train_generate_decription (module/utils.py:625-689): batch layout, false tails drawn from
    the relation's candidates, never a known tail of (head, rel) nor the true tail."""
    import random
    from module.zsl_module import train_generate_decription
    g = make_graph(seed=6)
    ents = g["ents"]
    tasks = g["train_tasks"]
    rng = random.Random(0)
    rel2cands = {r: rng.sample(ents, 40) for r in tasks}
    rel2cands[list(tasks)[0]] = ents[:10]  # <= 20 candidates: skipped like the reference
    e1rel_e2 = {}
    for r, tr in tasks.items():
        for h, rr, t in tr:
            e1rel_e2.setdefault(h + rr, []).append(t)
    for h, rr, t in (x for tr in tasks.values() for x in tr):
        e1rel_e2.setdefault(h + rr, [])
    rela2label = {r: i for i, r in enumerate(sorted(tasks))}
    gen = train_generate_decription(tasks, rel2cands, e1rel_e2, g["ent2id"], g["rel2id"], rela2label, 16, 2,
                                    rng=random.Random(1))
    inv = {i: e for e, i in g["ent2id"].items()}
    inv_rel = {i: r for r, i in g["rel2id"].items()}
    for _ in range(20):
        b = next(gen)
        n = len(b["rel"])
        assert n in (0, 16, 32) and all(len(v) == n for v in b.values())
        for i in range(n):
            rel = inv_rel[int(b["rel"][i])]
            h, t, f = inv[int(b["q_head"][i])], inv[int(b["q_tail"][i])], inv[int(b["f_tail"][i])]
            assert b["f_head"][i] == b["q_head"][i] and rela2label[rel] == b["labels"][i]
            assert [h, rel, t] in tasks[rel]
            assert f in rel2cands[rel] and f != t and f not in e1rel_e2[h + rel]
            assert len(rel2cands[rel]) > 20
