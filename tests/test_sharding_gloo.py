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


@pytest.mark.parametrize("world,keep_rel", [(2, None), (3, None), (3, 2), (8, 2)])
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


# ------------------------------------------------------------------ GPU --
def _workload(dataset, model, dim, keep_triples=None):
    from mmre.workloads import synthetic_large, zs_workload
    w = synthetic_large(dim=dim) if dataset == "synthetic-1M" else zs_workload(dataset, model, dim)
    if keep_triples is not None:  # fewer queries than ranks: some ranks own an empty shard
        for k in ("test_h", "test_r", "test_t"):
            w[k] = np.asarray(w[k])[:keep_triples]
    return w


def _spec(w, model, dim, dev):
    from mmre.link import ScoreSpec, rotate_phase_denom
    pk = {"transe": 0, "distmult": 2, "complex": 2, "rotate": 3}[model]
    return ScoreSpec(model=model, ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=dim,
                     ent_im=w["ent_im"].to(dev) if "ent_im" in w else None,
                     rel_im=w["rel_im"].to(dev) if "rel_im" in w else None, norm_flag=model == "transe",
                     pred_kind=pk, margin=float(w.get("margin", 0.0)),
                     phase_denom=rotate_phase_denom(w["margin"], w["epsilon"], dim) if model == "rotate" else 0.0)


def _gpu_worker(rank, world, port, res_path, dataset, model, dim, graph, keep_triples=None, cost=None, streams=1):
    """Each rank: the HIP sweep on cuda:0 through ShardedLinkEvaluation.launch/finish (counts
    exchanged over gloo through host memory); rank 0 also runs the single-process evaluation
    and the out-of-order ticket sequence."""
    sys.path[:0] = [PKG, os.path.join(REPO, "oracle"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmre.link import FilterIndex, evaluate_link_prediction
    from mmre.sharding import ShardedLinkEvaluation
    dev = torch.device("cuda:0")
    w = _workload(dataset, model, dim, keep_triples)
    E = w["n_ent"]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, w["n_rel"])
    spec = _spec(w, model, dim, dev)
    ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev, graph=graph,
                               cost=cost, streams=streams)
    assert (ev._streams is not None) == (streams == 2)
    assert (ev.weights is not None) == (cost == "undecided" and model == "transe")
    a = ev.launch()
    b = ev.launch()
    mb, cb = ev.finish(b)        # out of order: b first, then a third launch while a is pending
    c = ev.launch()
    ma, ca = ev.finish(a)
    mc, cc = ev.finish(c)
    out = dict(counts_a=ca, counts_b=cb, counts_c=cc, n_local=np.array(int(ev.masks[rank].sum())),
               masks=np.stack(ev.masks))
    if rank == 0:
        m1, (h1, t1) = evaluate_link_prediction(spec, w["test_h"], w["test_r"], w["test_t"], index=index)
        out["single"] = np.concatenate([h1, t1], 1)
        out["metrics_equal"] = np.array(all(ma[g][k] == m1[g][k] for g in m1 for k in m1[g]))
    np.savez(f"{res_path}_{rank}.npz", **out)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("dataset,model,dim,world,graph,keep,cost,streams", [
    ("FB15K-237-ZS", "transe", 200, 2, False, None, None, 1),
    ("FB15K-237-ZS", "transe", 200, 2, True, None, None, 1),
    ("DB15K-ZS", "complex", 200, 3, True, None, None, 2),
    ("FB15K-237-ZS", "rotate", 512, 8, True, None, None, 1),
    ("FB15K-237-ZS", "transe", 200, 8, True, 3, None, 2),
    ("FB15K-237-ZS", "transe", 200, 1, True, None, "undecided", 2),
    ("FB15K-237-ZS", "transe", 200, 2, True, None, "undecided", 1),
    ("FB15K-237-ZS", "transe", 200, 8, True, None, "undecided", 2)])
def test_sharded_hip_sweep_equals_single_rank(tmp_path, dataset, model, dim, world, graph, keep, cost, streams):
    """The multi-rank path with the real HIP sweep at full size (C2; C3 with its largest
    relation split across ranks; C4 RotatE d 512 at world 8, the driver's node size, every
    rank on the one GPU of the box), eager and with each rank's local evaluation replayed from
    a hipGraph: every rank's gathered counts -- for three overlapping evaluations finished out
    of order -- and rank 0's metrics are bit-equal to one process. keep=3: three test triples
    (6 sweeps) over 8 ranks, so two ranks own an empty shard and still join the all-gather.
    cost="undecided": the partition packed by calibrated per-query cost (rank 0's calibration
    broadcast: every rank holds the same masks) and each rank's queries swept heaviest first
    (world 1: the whole set reordered, the counts put back in query order by one gather).
    streams=2: two evaluation slots on two HIP streams, so the three overlapping evaluations
    run on alternating buffers / graphs / exchange buffers."""
    port = _free_port()
    res = str(tmp_path / "hip")
    mp.spawn(_gpu_worker, args=(world, port, res, dataset, model, dim, graph, keep, cost, streams), nprocs=world,
             join=True)
    outs = [dict(np.load(f"{res}_{k}.npz")) for k in range(world)]
    single = outs[0]["single"]
    assert bool(outs[0]["metrics_equal"])
    for o in outs:
        for key in ("counts_a", "counts_b", "counts_c"):
            assert np.array_equal(o[key], single), key
        assert np.array_equal(o["masks"], outs[0]["masks"])   # every rank packed the same partition
    assert sum(int(o["n_local"]) for o in outs) == single.shape[1]
    if cost is None:
        assert max(int(o["n_local"]) for o in outs) <= -(-single.shape[1] // world)


def _entity_worker(rank, world, port, res_path, dataset, model, dim):
    """Each rank: the HIP sweep of ALL queries against its entity slice on cuda:0, counts summed
    over gloo (host memory); rank 0 also runs the single-process evaluation."""
    sys.path[:0] = [PKG, os.path.join(REPO, "oracle"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmre.link import FilterIndex, evaluate_link_prediction
    from mmre.sharding import EntityShardedLinkEvaluation
    dev = torch.device("cuda:0")
    w = _workload(dataset, model, dim)
    E = w["n_ent"]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, w["n_rel"])
    spec = _spec(w, model, dim, dev)
    ev = EntityShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev)
    a = ev.launch()
    b = ev.launch()
    mb, cb = ev.finish(b)
    ma, ca = ev.finish(a)
    out = dict(counts_a=ca, counts_b=cb, e0=np.array(ev.entity_range[0]), e1=np.array(ev.entity_range[1]))
    if rank == 0:
        m1, (h1, t1) = evaluate_link_prediction(spec, w["test_h"], w["test_r"], w["test_t"], index=index)
        out["single"] = np.concatenate([h1, t1], 1)
        out["metrics_equal"] = np.array(all(ma[g][k] == m1[g][k] for g in m1 for k in m1[g]))
    np.savez(f"{res_path}_{rank}.npz", **out)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("dataset,model,dim,world", [("FB15K-237-ZS", "transe", 200, 2),
                                                      ("DB15K-ZS", "complex", 200, 3),
                                                      ("synthetic-1M", "distmult", 256, 8)])
def test_entity_sharded_hip_sweep_equals_single_rank(tmp_path, dataset, model, dim, world):
    """SURVEY 8(e)'s alternative for huge E: each rank sweeps every query against a contiguous
    slice of the entity tiles (VALU TransE and MFMA ComplEx / DistMult kernels), counts summed
    by one all-reduce: every rank's counts and rank 0's metrics are bit-equal to one process --
    C5 (1 M entities, DistMult d 256) at world 8, every rank on the one GPU of the box."""
    port = _free_port()
    res = str(tmp_path / "ent")
    mp.spawn(_entity_worker, args=(world, port, res, dataset, model, dim), nprocs=world, join=True)
    outs = [dict(np.load(f"{res}_{k}.npz")) for k in range(world)]
    single = outs[0]["single"]
    assert bool(outs[0]["metrics_equal"])
    for o in outs:
        assert np.array_equal(o["counts_a"], single) and np.array_equal(o["counts_b"], single)
    assert outs[0]["e0"] == 0 and all(outs[k]["e1"] == outs[k + 1]["e0"] for k in range(world - 1))
