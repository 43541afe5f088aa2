"""Multi-process (gloo, CPU) test of the relation-sharded evaluation: LPT partition, one
all-gather of per-rank rank counts, metric reduction. The per-rank sweep is the oracle here
(CPU test); on the GPU box the same class runs the HIP sweep over RCCL (bench.py --gpus N)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_runner(ent, rel, hrt):
    import oracle

    def run(qh, qr, qt, qm, filt, masks_tc, events=None):
        qh, qr, qt, qm = (x.numpy() for x in (qh, qr, qt, qm))
        out = np.zeros((4, len(qh)), np.int32)
        for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
            sel = qm == mode_id
            if sel.any():
                pred = oracle.link_predict("transe", mode, ent, rel, qh[sel], qr[sel], qt[sel], norm_flag=True)
                out[:, sel] = oracle.test_rank(mode, pred, qh[sel], qr[sel], qt[sel], hrt).T
        return torch.from_numpy(out)
    return run


def _test_list(d, keep_rel):
    h, r, t = d.test_list()
    if keep_rel:  # only the first `keep_rel` test relations: ranks beyond them own no query
        sel = np.isin(r, np.unique(r)[:keep_rel])
        h, r, t = h[sel], r[sel], t[sel]
    return h, r, t


def _worker(rank, world, port, res_path, keep_rel=None):
    sys.path[:0] = [PKG, os.path.join(REPO, "oracle"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from mmre.data import OpenKEDataset
    from mmre.sharding import ShardedLinkEvaluation
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "medium"))
    rng = np.random.default_rng(0)
    ent = rng.uniform(-0.5, 0.5, (d.n_ent, 16)).astype(np.float32)
    rel = rng.uniform(-0.5, 0.5, (d.n_rel, 16)).astype(np.float32)
    trip = np.concatenate([d.train, d.valid, d.test])
    hrt = oracle.sorted_hrt(trip[:, 0], trip[:, 2], trip[:, 1])
    h, r, t = _test_list(d, keep_rel)
    ev = ShardedLinkEvaluation(None, h, r, t, device="cpu", local_runner=_oracle_runner(ent, rel, hrt))
    metrics, counts = ev.run()
    np.save(f"{res_path}_{rank}.npy", counts)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,keep_rel", [(2, None), (3, None), (3, 2)])
def test_sharded_counts_equal_single_rank(tmp_path, world, keep_rel):
    """keep_rel=2 at world 3: one rank owns no relation and joins the all-gather empty."""
    import oracle
    port = _free_port()
    res = str(tmp_path / "counts")
    mp.spawn(_worker, args=(world, port, res, keep_rel), nprocs=world, join=True)
    outs = [np.load(f"{res}_{k}.npy") for k in range(world)]
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])  # every rank holds the full table
    # single-rank reference
    sys.path[:0] = [PKG]
    from mmre.data import OpenKEDataset
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "medium"))
    rng = np.random.default_rng(0)
    ent = rng.uniform(-0.5, 0.5, (d.n_ent, 16)).astype(np.float32)
    rel = rng.uniform(-0.5, 0.5, (d.n_rel, 16)).astype(np.float32)
    trip = np.concatenate([d.train, d.valid, d.test])
    hrt = oracle.sorted_hrt(trip[:, 0], trip[:, 2], trip[:, 1])
    h, r, t = _test_list(d, keep_rel)
    single = _oracle_runner(ent, rel, hrt)(*(torch.from_numpy(np.concatenate([x, x])) for x in (h, r, t)),
                                           torch.from_numpy(np.r_[np.zeros(len(h), np.int8), np.ones(len(h), np.int8)]),
                                           None, None).numpy()
    assert np.array_equal(outs[0], single)
