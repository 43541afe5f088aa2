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
