"""Tester (OpenKE/openke/config/Tester.py:17-91).

run_link_prediction replaces the per-query Python loop (getHeadBatch -> predict -> D2H ->
testHead, per test triple) with ONE fused evaluation on the GPU (mmre.link): every head- and
tail-batch sweep of the test set against every entity, filtered and type-constrained ranks
counted in the sweep's epilogue, then the Test.h metric reduction (test_link_prediction,
Test.h:232-327) with the reference's float order. Returns (mrr, mr, hit10, hit3, hit1) like
the reference."""
import numpy as np
import torch

from mmre.link import evaluate_link_prediction


class Tester(object):
    def __init__(self, model=None, data_loader=None, use_gpu=True):
        self.model = model
        self.data_loader = data_loader
        self.use_gpu = use_gpu
        self.last = None
        if self.use_gpu and self.model is not None:
            self.model.cuda()

    def set_model(self, model):
        self.model = model

    def set_data_loader(self, data_loader):
        self.data_loader = data_loader

    def set_use_gpu(self, use_gpu):
        self.use_gpu = use_gpu
        if self.use_gpu and self.model is not None:
            self.model.cuda()

    def to_var(self, x, use_gpu):
        t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.asarray(x))
        return t.cuda() if use_gpu else t

    def test_one_step(self, data):
        return self.model.predict({"batch_h": self.to_var(data["batch_h"], self.use_gpu),
                                   "batch_t": self.to_var(data["batch_t"], self.use_gpu),
                                   "batch_r": self.to_var(data["batch_r"], self.use_gpu),
                                   "mode": data["mode"]})

    def run_link_prediction(self, type_constrain=False):
        dl = self.data_loader
        dl.set_sampling_mode("link")
        metrics, counts = evaluate_link_prediction(self.model.score_spec(), dl.test_h, dl.test_r, dl.test_t,
                                                   index=dl.filter_index(), type_constrain=bool(type_constrain))
        self.last = {"metrics": metrics, "counts": counts}
        self._print(metrics, type_constrain)
        grp = metrics["filter_tc" if type_constrain else "filter"]
        print(grp["hit10"])
        return grp["mrr"], grp["mr"], grp["hit10"], grp["hit3"], grp["hit1"]

    @staticmethod
    def _print(m, tc):
        def line(name, g):
            return f"{name}\t {g['mrr']:f} \t {g['mr']:f} \t {g['hit10']:f} \t {g['hit3']:f} \t {g['hit1']:f} "
        print("no type constraint results:")
        print("metric:\t\t\t MRR \t\t MR \t\t hit@10 \t hit@3  \t hit@1 ")
        print(line("averaged(raw):\t\t", m["raw"]))
        print(line("averaged(filter):\t", m["filter"]))
        if tc:
            print("type constraint results:")
            print(line("averaged(raw):\t\t", m["raw_tc"]))
            print(line("averaged(filter):\t", m["filter_tc"]))

    def run_triple_classification(self, threshlod=None):
        raise NotImplementedError("triple classification is outside the MI355X hot path (SURVEY.md §2 row 7)")
