"""Zero-shot evaluation ranking of ZSLmodule.eval (module/zsl_module.py:635-745).

`zsl_rank(candidate_vecs, cand_off, relation_vecs, rel_of_query)` runs the cosine-similarity
ranking of every query on the GPU (csrc/candidates.hip): score = mean over the test_sample
generated relation vectors of cos(candidate, relation) (sklearn cosine_similarity, :699-701),
rank of the true candidate (row 0) in descending order (:705-706). `zsl_metrics` prints and
returns Hits@10/5/1 and MRR as the reference does (:707-745). The Extractor that produces the
candidate vectors (zsl_module.py:17-110) is the next component."""
import numpy as np

from mmre.candidates import cosine_rank


def zsl_rank(candidate_vecs, cand_off, relation_vecs, rel_of_query):
    return cosine_rank(candidate_vecs, cand_off, relation_vecs, rel_of_query)


def zsl_metrics(ranks, mode="test", per_relation=None):
    r = np.asarray(ranks)
    h10 = (r <= 10).astype(float)
    h5 = (r <= 5).astype(float)
    h1 = (r <= 1).astype(float)
    mrr = 1.0 / r
    if per_relation is not None:
        for name, sel in per_relation.items():
            print("{} Hits10:{:.3f}, Hits5:{:.3f}, Hits1:{:.3f} MRR:{:.3f}".format(
                mode + name, h10[sel].mean(), h5[sel].mean(), h1[sel].mean(), mrr[sel].mean()))
    print("############   " + mode + "    #############")
    print("HITS10: {:.3f}".format(h10.mean()))
    print("HITS5: {:.3f}".format(h5.mean()))
    print("HITS1: {:.3f}".format(h1.mean()))
    print("MAP: {:.3f}".format(mrr.mean()))
    print("###################################")
    return float(h10.mean()), float(h5.mean()), float(mrr.mean())
