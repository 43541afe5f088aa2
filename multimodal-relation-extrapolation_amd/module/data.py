"""The parts of the reference's dataset (module/data.py: MMKGDataset, :44-339) that this path
reads, over an origin_data/<dataset> directory (entity2ids_zsl.json, relation2ids.json,
rel_description_zsl, <train_file>):

* id maps and sizes (num_nodes, num_relations) -- load_appendix_data (utils.py:194-230);
* relation-description token rows for generate_batch's 'rel_des' / 'rel_des_padding_mask'
  (data.py:274, 301-304): the BERT tokenizer MMKGDataset uses (data.py:57, 122-124, 252-270)
  cannot be loaded offline, so descriptions are split the way BERT's basic tokenizer splits
  (lower case, words and single punctuation marks) and every piece gets a stable id in
  [first_id, vocab_size) (CRC32); padding mask 1.0 on padded positions, rows of max_len;
* the structure graph of the train tasks (get_struc_dataset: edge_index (2, n) head -> tail,
  edge_type (n,)).

Entity images and texts (MultiModalInfo_zsl.pkl, not shipped with the reference) are outside
this path: generate_batch's 'image' / 'text' are empty.
"""
import json
import os
import re
import zlib
from types import SimpleNamespace

import numpy as np
import torch


def tokenize_descriptions(lines, max_len=320, vocab_size=30522, first_id=1000):
    """-> tok (R, max_len) int64 (0 on padded positions), mask (R, max_len) float32 (1.0 =
    padding), n_tok (R,) int64."""
    tok = np.zeros((len(lines), max_len), np.int64)
    n_tok = np.zeros(len(lines), np.int64)
    for i, line in enumerate(lines):
        pieces = re.findall(r"\w+|[^\w\s]", line.lower())[:max_len]
        ids = [first_id + zlib.crc32(p.encode()) % (vocab_size - first_id) for p in pieces]
        tok[i, :len(ids)] = ids
        n_tok[i] = len(ids)
    mask = (np.arange(max_len)[None, :] >= n_tok[:, None]).astype(np.float32)
    return tok, mask, n_tok


def read_descriptions(path):
    """rel_description_zsl: one description per line, by relation id (utils.py:222-229)."""
    with open(path) as fin:
        return [line[:-1] if line.endswith("\n") else line for line in fin.readlines()]


def load_tasks(path, e2id, r2id):
    """{relation: [[h, r, t], ...]} -> h, r, t id lists (load_appendix_data, utils.py:198-208)."""
    with open(path) as f:
        task = json.load(f)
    h, r, t = [], [], []
    for rel in task.keys():
        for head, rr, tail in task[rel]:
            h.append(e2id[head])
            r.append(r2id[rr])
            t.append(e2id[tail])
    return [h, r, t]


class ZSDataset:
    def __init__(self, root, train_file="train_tasks_zsl.json", max_len=320, vocab_size=30522, struct_only=False):
        self.root = root
        with open(os.path.join(root, "entity2ids_zsl.json")) as f:
            self.e2id = json.load(f)
        with open(os.path.join(root, "relation2ids.json")) as f:
            self.r2id = json.load(f)
        self.num_nodes = max(self.e2id.values()) + 1
        self.num_relations = max(self.r2id.values()) + 1
        self.rel_des = read_descriptions(os.path.join(root, "rel_description_zsl"))
        if len(self.rel_des) < self.num_relations:
            raise ValueError(f"{len(self.rel_des)} relation descriptions for {self.num_relations} relations")
        tok, mask, self.n_tok = tokenize_descriptions(self.rel_des, max_len, vocab_size)
        self.rel_tokens, self.rel_mask = torch.from_numpy(tok), torch.from_numpy(mask)
        self.vocab_size = vocab_size
        self.config = SimpleNamespace(image_only=False, text_only=False, struct_only=struct_only,
                                      tokenizer_max_length=max_len, unpaired_tokenizer_max_length=max_len)
        self.transform_image = None
        self.tokenizer = None
        tp = os.path.join(root, train_file)
        self.triples = load_tasks(tp, self.e2id, self.r2id) if os.path.exists(tp) else [[], [], []]
        h, r, t = (torch.as_tensor(x, dtype=torch.int64) for x in self.triples)
        self.edge_index = torch.stack([h, t]) if len(h) else torch.zeros((2, 0), dtype=torch.int64)
        self.edge_type = r

    def generate_batch(self, n_id, batch_rels):
        rels = torch.as_tensor(batch_rels, dtype=torch.int64)
        return dict(image=torch.empty(0), text=torch.empty(0, dtype=torch.int64), text_padding_mask=torch.empty(0),
                    rel_des=self.rel_tokens[rels], rel_des_padding_mask=self.rel_mask[rels])

    def get_struc_dataset(self):
        return SimpleNamespace(edge_index=self.edge_index, edge_type=self.edge_type, num_nodes=self.num_nodes)
