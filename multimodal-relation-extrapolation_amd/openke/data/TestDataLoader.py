"""TestDataLoader -- the openke.data contract (OpenKE Tester.py:70-82; absent from the reference
tree). Iterating in 'link' mode yields [data_head, data_tail] per test triple exactly like the
Base.so-backed loader (getHeadBatch/getTailBatch, Test.h:36-53), in testList order (sorted by
(r, h, t), Reader.h:227). The MI355X Tester does not iterate: it hands the whole test list to
the fused sweep (mmre.link)."""
import os

import numpy as np

from mmre.data import OpenKEDataset
from mmre.link import FilterIndex


class TestDataLoader(object):
    def __init__(self, in_path="./", sampling_mode="link", type_constrain=True):
        self.in_path = in_path
        self.sampling_mode = sampling_mode
        self.type_constrain = type_constrain
        self.ds = OpenKEDataset(in_path)
        self.entTotal, self.relTotal = self.ds.n_ent, self.ds.n_rel
        self.test_h, self.test_r, self.test_t = self.ds.test_list()
        self.testTotal = len(self.test_h)
        self._index = None

    def filter_index(self):
        """train + valid + test known triples (Reader.h:201-226) and type constraints."""
        if self._index is None:
            h, r, t = self.ds.all_triples()
            th, tt = (self.ds.type_heads, self.ds.type_tails) if self.type_constrain else (None, None)
            self._index = FilterIndex(h, r, t, self.entTotal, self.relTotal, th, tt)
        return self._index

    def set_sampling_mode(self, sampling_mode):
        self.sampling_mode = sampling_mode

    def get_ent_tot(self):
        return self.entTotal

    def get_rel_tot(self):
        return self.relTotal

    def get_triple_tot(self):
        return self.testTotal

    def sampling_lp(self, i):
        E = self.entTotal
        h, r, t = int(self.test_h[i]), int(self.test_r[i]), int(self.test_t[i])
        head = {"batch_h": np.arange(E, dtype=np.int64), "batch_t": np.array([t], np.int64),
                "batch_r": np.array([r], np.int64), "mode": "head_batch"}
        tail = {"batch_h": np.array([h], np.int64), "batch_t": np.arange(E, dtype=np.int64),
                "batch_r": np.array([r], np.int64), "mode": "tail_batch"}
        return [head, tail]

    def __iter__(self):
        if self.sampling_mode != "link":
            raise NotImplementedError("triple classification is outside the MI355X hot path (SURVEY.md §2 row 7)")
        for i in range(self.testTotal):
            yield self.sampling_lp(i)

    def __len__(self):
        return self.testTotal
