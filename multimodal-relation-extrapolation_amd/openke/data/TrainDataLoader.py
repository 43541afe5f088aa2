"""TrainDataLoader -- the openke.data contract the reference's examples import
(OpenKE/examples/train_transe_FB15K237.py:9-17; absent from the reference tree).

Reads an OpenKE benchmark directory (Reader.h:53-160) and samples on the GPU with
mmre.sampler.OpenKESampler: the same batches as Base.so's `sampling` (Base.cpp:161-197),
bit-for-bit, returned as device tensors."""
import os

import numpy as np

from mmre.data import OpenKEDataset, TrainIndex
from mmre.sampler import OpenKESampler


class TrainDataLoader(object):
    def __init__(self, in_path="./", tri_file=None, ent_file=None, rel_file=None, batch_size=None, nbatches=None,
                 threads=8, sampling_mode="normal", bern_flag=False, filter_flag=True, neg_ent=1, neg_rel=0,
                 device="cuda:0", seeds=None):
        self.in_path = in_path
        self.tri_file = tri_file or os.path.join(in_path, "train2id.txt")
        self.ent_file = ent_file or os.path.join(in_path, "entity2id.txt")
        self.rel_file = rel_file or os.path.join(in_path, "relation2id.txt")
        self.work_threads = threads
        self.nbatches = nbatches
        self.batch_size = batch_size
        self.bern = bool(bern_flag)
        self.filter = filter_flag  # accepted and, as in Base.cpp:116/:119, sampling is always filtered
        self.negative_ent = neg_ent
        self.negative_rel = neg_rel
        self.sampling_mode = sampling_mode
        self.cross_sampling_flag = 0
        self.device = device
        ds = OpenKEDataset(in_path, ent_file=self.ent_file, rel_file=self.rel_file, train_file=self.tri_file)
        self.relTotal, self.entTotal = ds.n_rel, ds.n_ent
        self.index = TrainIndex(ds.train[:, 0], ds.train[:, 1], ds.train[:, 2], ds.n_ent, ds.n_rel)
        self.tripleTotal = self.index.train_total
        if self.batch_size is None:
            self.batch_size = self.tripleTotal // self.nbatches
        if self.nbatches is None:
            self.nbatches = self.tripleTotal // self.batch_size
        self.sampler = OpenKESampler(self.index, device, work_threads=threads, bern=self.bern, seeds=seeds)

    def sampling(self):
        out = self.sampler.sample(self.batch_size, self.negative_ent, self.negative_rel, 0)
        out["mode"] = "normal"
        return out

    def sampling_head(self):
        out = self.sampler.sample(self.batch_size, self.negative_ent, self.negative_rel, -1)
        B = self.batch_size
        return {"batch_h": out["batch_h"], "batch_t": out["batch_t"][:B], "batch_r": out["batch_r"][:B],
                "batch_y": out["batch_y"], "mode": "head_batch"}

    def sampling_tail(self):
        out = self.sampler.sample(self.batch_size, self.negative_ent, self.negative_rel, 1)
        B = self.batch_size
        return {"batch_h": out["batch_h"][:B], "batch_t": out["batch_t"], "batch_r": out["batch_r"][:B],
                "batch_y": out["batch_y"], "mode": "tail_batch"}

    def cross_sampling(self):
        self.cross_sampling_flag = 1 - self.cross_sampling_flag
        return self.sampling_head() if self.cross_sampling_flag == 0 else self.sampling_tail()

    # setters / getters of the upstream loader
    def set_work_threads(self, work_threads):
        self.work_threads = work_threads

    def set_in_path(self, in_path):
        self.in_path = in_path

    def set_nbatches(self, nbatches):
        self.nbatches = nbatches

    def set_batch_size(self, batch_size):
        self.batch_size = batch_size
        self.nbatches = self.tripleTotal // self.batch_size

    def set_ent_neg_rate(self, rate):
        self.negative_ent = rate

    def set_rel_neg_rate(self, rate):
        self.negative_rel = rate

    def set_bern_flag(self, bern):
        self.bern = bool(bern)
        self.sampler.bern = self.bern

    def set_filter_flag(self, filter_flag):
        self.filter = filter_flag

    def get_batch_size(self):
        return self.batch_size

    def get_ent_tot(self):
        return self.entTotal

    def get_rel_tot(self):
        return self.relTotal

    def get_triple_tot(self):
        return self.tripleTotal

    def __iter__(self):
        for _ in range(self.nbatches):
            yield self.sampling() if self.sampling_mode == "normal" else self.cross_sampling()

    def __len__(self):
        return self.nbatches
