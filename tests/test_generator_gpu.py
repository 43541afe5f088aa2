"""GPU parity of the zero-shot relation generator and the candidate rankings."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["g200_eval", "g200_train", "g256_eval"])
def test_generator_matches_reference(golden, tag):
    from mmre.generator import RelationGenerator
    g = golden("repo")
    dev = torch.device("cuda:0")
    D = g[f"{tag}_W2"].shape[0]
    gen = RelationGenerator(384, 15, D).to(dev)
    with torch.no_grad():
        for i, L in enumerate([gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2]):
            L.weight_orig.copy_(torch.from_numpy(g[f"{tag}_W{i}"]))
            L.bias.copy_(torch.from_numpy(g[f"{tag}_b{i}"]))
            L.weight_u.copy_(torch.from_numpy(g[f"{tag}_u{i}"]))
            L.weight_v.copy_(torch.from_numpy(g[f"{tag}_v{i}"]))
        gen.ln_a.copy_(torch.from_numpy(g[f"{tag}_a"]))
        gen.ln_b.copy_(torch.from_numpy(g[f"{tag}_b"]))
    gen.train(bool(g[f"{tag}_train"]))
    out = gen(torch.from_numpy(g[f"{tag}_cls"]).to(dev), torch.from_numpy(g[f"{tag}_noise"]).to(dev))
    torch.cuda.synchronize()
    ref = g[f"{tag}_out"]
    assert np.abs(out.detach().cpu().numpy() - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())
    for i, L in enumerate([gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2]):
        assert np.allclose(L.weight_u.cpu().numpy(), g[f"{tag}_u{i}_after"], atol=1e-5)
        assert np.allclose(L.weight_v.cpu().numpy(), g[f"{tag}_v{i}_after"], atol=1e-5)


def test_candidate_rank_transe(golden, oracle_mod):
    from mmre.candidates import candidate_rank_transe
    g = golden("repo")
    dev = torch.device("cuda:0")
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rank, scores = candidate_rank_transe(to(g["ev_ent"]), to(g["ev_rel"]), to(g["ev_qh"].astype(np.int64)),
                                         to(g["ev_qr"].astype(np.int64)), to(g["ev_off"].astype(np.int64)),
                                         to(g["ev_cids"].astype(np.int64)), return_scores=True)
    torch.cuda.synchronize()
    o_s, o_r = oracle_mod.candidate_rank_transe(g["ev_ent"], g["ev_rel"], g["ev_qh"], g["ev_qr"], g["ev_off"],
                                                g["ev_cids"])
    assert np.array_equal(scores.cpu().numpy(), o_s)          # canonical arithmetic: bit-identical
    assert np.array_equal(rank.cpu().numpy(), g["ev_ranks"])  # reference rank rule (main.py:245-250)


def test_cosine_rank(golden):
    from mmre.candidates import cosine_rank
    g = golden("repo")
    dev = torch.device("cuda:0")
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rank, scores = cosine_rank(to(g["zs_cand"]), to(g["zs_off"].astype(np.int64)), to(g["zs_relvecs"]),
                               to(g["zs_rel"].astype(np.int64)), return_scores=True)
    torch.cuda.synchronize()
    assert np.allclose(scores.cpu().numpy(), g["zs_scores"], atol=1e-5)
    assert np.array_equal(rank.cpu().numpy(), g["zs_ranks"])
