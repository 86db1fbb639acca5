"""The N>1 paths on CPU with the gloo backend at world sizes 2, 4 and 8:
gradient averaging over the flat gradient buffer (ddp.py), rank-0 parameter
and BN-buffer broadcast, and the gallery-sharded retrieval protocol of
knn.knn_sharded itself (owner's positive key -> all_reduce MAX, per-shard
exact top-k + rank counts -> all_gather_into_tensor / all_reduce SUM -> merge),
with CPU stand-ins for the GPU kernels, against the unsharded oracle."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLDS = [2, 4, 8]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(fn, *args, world=2):
    port = _free_port()
    mp.spawn(_entry, args=(fn, port, world, args), nprocs=world, join=True)


def _entry(rank, fn, port, world, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _mean_rank1():
    """mean of rank + 1 over the ranks: what averaging a per-rank (rank + 1) gives"""
    return (dist.get_world_size() + 1) / 2.0


def _allreduce(rank):
    import ddp
    n = 1000
    flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
    model = types.SimpleNamespace(_hip_engine=types.SimpleNamespace(_grads=types.SimpleNamespace(flat=flat)))
    ddp.allreduce_gradients(model, bucket_bytes=256)  # 64-element buckets, last one ragged
    want = torch.arange(n, dtype=torch.float32) * _mean_rank1()
    assert torch.allclose(flat, want), (flat - want).abs().max()


@pytest.mark.parametrize("world", WORLDS)
def test_allreduce_gradients_averages_flat_buffer(world):
    _run(_allreduce, world=world)


def _broadcast(rank):
    import ddp
    import models
    torch.manual_seed(100 + rank)  # ranks start from different weights
    m = models.ModifiedResNet((1, 1, 1, 1), 32, heads=8, input_resolution=64, width=16)
    for b in m.buffers():
        if b.dtype.is_floating_point:
            b.fill_(float(rank))
    ddp.broadcast_parameters(m)
    ddp.broadcast_buffers(m)
    torch.manual_seed(100)
    m0 = models.ModifiedResNet((1, 1, 1, 1), 32, heads=8, input_resolution=64, width=16)
    for (k, p), (_, q) in zip(m.named_parameters(), m0.named_parameters()):
        assert torch.equal(p, q), k
    for b in m.buffers():
        if b.dtype.is_floating_point:
            assert torch.all(b == 0)


@pytest.mark.parametrize("world", [2, 4])
def test_broadcast_parameters_and_buffers(world):
    _run(_broadcast, world=world)


def _cpu_local_search(queries, shard, k, positives, compute, g_base=0, dpos=None, metric="euclidean"):
    """CPU stand-in of knn.knn for one shard (the oracle's exact keys): the same
    return contract — global indices padded with -1 / +inf, per-shard rank counts"""
    from oracle import retrieval as oret
    qs, g = queries.numpy(), shard.numpy()
    n = len(g)
    Q = len(qs)
    idx = np.full((Q, k), -1, np.int64)
    dd = np.full((Q, k), np.inf)
    cnt = np.zeros(Q, np.int64)
    for i, q in enumerate(qs):
        d = oret.distances(q, g, metric)
        ti, td = oret.topk(d, min(k, n))
        idx[i, :len(ti)] = ti + g_base
        dd[i, :len(td)] = td
        if positives is not None and dpos[i] >= 0:
            gi = np.arange(g_base, g_base + n)
            p = int(positives[i])
            cnt[i] = int(((d < dpos[i].item()) | ((d == dpos[i].item()) & (gi < p))).sum())
    rank = torch.from_numpy(cnt) if positives is not None else None
    return torch.from_numpy(idx), torch.from_numpy(dd), rank, dpos


def _cpu_positive_keys(queries, shard, g_base, positives, metric="euclidean"):
    from oracle import retrieval as oret
    out = torch.full((len(queries),), -1.0, dtype=torch.float64)
    for i, p in enumerate(positives.tolist()):
        if g_base <= p < g_base + len(shard):
            out[i] = float(oret.distances(queries[i].numpy(), shard[p - g_base:p - g_base + 1].numpy(), metric)[0])
    return out


def _ragged_bounds(n, world):
    """shard boundaries of n rows over world ranks, ragged as a 1,000,000-row
    gallery split 8 ways by whole batches is: odd sizes, and at world 8 one shard
    shorter than the top-k list (5 rows)"""
    b = [0] + [i * n // world + (13 if i % 2 else -21) for i in range(1, world)] + [n]
    if world == 8:
        b[3] = b[2] + 5
    return b


def _sharded(rank, k, metric):
    """knn.knn_sharded's own collective code (all_reduce MAX of the positives' keys,
    all_gather_into_tensor of the lists, merge, all_reduce SUM of the ranks) over
    gloo, with CPU stand-ins for the GPU search and merge"""
    import knn
    from oracle import retrieval as oret
    world = dist.get_world_size()
    g, qs, pos = oret.synthetic_gallery(1000, 16, 32, seed_g=5, seed_q=6)
    g[900:910] = g[0:10]  # duplicate rows in three shards (two at world 2) -> cross-shard ties
    g[480:490] = g[0:10]
    qs[:4] = g[:4]
    pos = pos.copy()
    pos[5] = -1  # a query without a positive
    pos[6] = 903  # positives among the duplicates
    pos[7] = 484
    bounds = _ragged_bounds(1000, world)
    lo, hi = bounds[rank], bounds[rank + 1]
    mi, md, rk = knn.knn_sharded(torch.from_numpy(qs), torch.from_numpy(g[lo:hi]), lo, k, torch.from_numpy(pos),
                                 metric=metric, local_search=_cpu_local_search, positive_keys=_cpu_positive_keys,
                                 merge=lambda d, i, kk: knn.merge_topk(list(i), list(d), kk))
    for i, q in enumerate(qs):
        d_full = oret.distances(q, g, metric)
        ri, rd = oret.topk(d_full, k)
        np.testing.assert_array_equal(mi[i].numpy(), ri)
        np.testing.assert_array_equal(md[i].numpy(), rd)
        if pos[i] >= 0:
            assert rk[i].item() == oret.rank_of(d_full, pos[i])


@pytest.mark.parametrize("world", WORLDS)
def test_sharded_retrieval_protocol_matches_unsharded_oracle(world):
    _run(_sharded, 10, "euclidean", world=world)


@pytest.mark.parametrize("world", WORLDS)
def test_sharded_retrieval_protocol_cosine_short_shard(world):
    """cosine keys and k = 20 (the lists of every shard are merged by (key, index))"""
    _run(_sharded, 20, "cosine", world=world)


def test_merge_topk_short_shards():
    import knn
    a_i = torch.tensor([[3, -1, -1]])
    a_d = torch.tensor([[0.5, 0.0, 0.0]], dtype=torch.float64)
    b_i = torch.tensor([[7, 1, 9]])
    b_d = torch.tensor([[0.5, 0.7, 0.9]], dtype=torch.float64)
    i, d = knn.merge_topk([a_i, b_i], [a_d, b_d], 3)
    assert i.tolist() == [[3, 7, 1]] and d.tolist() == [[0.5, 0.5, 0.7]]


def _overlapped(rank):
    """ddp.OverlappedReducer: ranges reported out of order, in pieces, some
    never reported (swept by end()); every element is all-reduced exactly once
    (a second reduction would show as a wrong scale) and buckets launch as soon
    as bucket_bytes are pending, before end()."""
    import ddp
    n = 1000
    flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
    r = ddp.OverlappedReducer(bucket_bytes=400)  # 100 floats
    r.begin(flat)
    r.ready([(900, 1000)])                 # the end of the buffer first (the attention pool)
    assert r.launches == [(900, 1000)]     # one full bucket pending -> launched immediately
    r.ready([(850, 900), (700, 760)])      # 110 pending -> launched, adjacent ranges kept apart
    assert len(r.launches) == 3
    r.ready([(0, 10)])                     # 10 pending: below the bucket, waits
    assert len(r.launches) == 3
    r.end()                                # (0,10) plus the unreported [10,700) and [760,850)
    covered = sorted(r.launches)
    lo = 0
    for a, b in covered:
        assert a == lo, covered
        lo = b
    assert lo == n
    r.finish()
    want = torch.arange(n, dtype=torch.float32) * _mean_rank1()
    assert torch.allclose(flat, want), (flat - want).abs().max()
    # a step whose backward never drove the reducer: finish() falls back to the plain all-reduce
    flat2 = torch.ones(50) * (rank + 1)
    model = types.SimpleNamespace(_hip_engine=types.SimpleNamespace(_grads=types.SimpleNamespace(flat=flat2)))
    r2 = ddp.OverlappedReducer(bucket_bytes=64, model=model)
    r2.finish()
    assert torch.allclose(flat2, torch.full((50,), _mean_rank1()))


@pytest.mark.parametrize("world", WORLDS)
def test_overlapped_reducer_protocol(world):
    _run(_overlapped, world=world)


class _ProjModel(torch.nn.Module):
    """CPU stand-in encoder for the sharded-inference protocol: 4x4 average pool
    then a fixed random projection (the protocol is model-agnostic)."""

    def __init__(self, res, dim=8):
        super().__init__()
        g = torch.Generator().manual_seed(7)
        self.w = torch.randn(3 * (res // 4) ** 2, dim, generator=g)
        self.transform = None

    def forward(self, x):
        return torch.nn.functional.avg_pool2d(x, 4).flatten(1) @ self.w


def _sharded_inference(rank, tmp, metric):
    import data_preparation
    import inference
    import knn
    from oracle import retrieval as oret
    os.chdir(tmp)
    res = 16
    model = _ProjModel(res)
    _, test = data_preparation.get_datasets("SyntheticKaggle", n=130, resolution=res)  # 13 photos, 3+ shards ragged
    out = inference.run_inference_sharded(
        model, test, metric, local_search=_cpu_local_search, positive_keys=_cpu_positive_keys,
        merge=lambda d, i, kk: knn.merge_topk(list(i), list(d), kk))
    assert set(out) == {"image_features", "drawing_stats", "sketch_stats"}  # Kaggle -> second pass
    # unsharded expectation: every photo / sketch embedded in one process, exact oracle search
    ids = data_preparation.InferenceDataset(test.photo_paths, None, res)
    with torch.no_grad():
        g = torch.cat([model(ids[i][None]) for i in range(len(ids))]).numpy()
    feats = np.load(os.path.join("data/image_features", out["image_features"], "image_features.npy"))
    np.testing.assert_allclose(feats, g, rtol=1e-6, atol=1e-6)  # rank 0 saved the gathered gallery
    _, kag = data_preparation.get_datasets("KaggleInferenceV1", sketch_type="sketches")
    for ds, stats in ((test, out["drawing_stats"]), (kag, out["sketch_stats"])):
        with torch.no_grad():
            q = torch.cat([model(inference._Sketches(ds)[i][None]) for i in range(len(ds))]).numpy()
        pos = inference._positives(ds, ids.image_paths)
        ranks = []
        for i in range(len(ds)):
            d = oret.distances(q[i], g, metric)
            ranks.append(oret.rank_of(d, pos[i]) if pos[i] >= 0 else len(g))
        want = inference.retrieval_stats(ranks, 10)
        assert stats["mean_reciprocal_rank"] == pytest.approx(want["mean_reciprocal_rank"], rel=1e-12)
        assert stats["topk_acc"] == pytest.approx(want["topk_acc"])
        assert stats["size"] == len(g)
        for sample in stats["retrieval_samples"]:
            (sp, top), = sample.items()
            i = [str(p) for p in ds.sketch_paths].index(sp)
            ti, td = oret.topk(oret.distances(q[i], g, metric), min(10, len(g)))
            assert [p for p, _ in top] == [str(ids.image_paths[j]) for j in ti]
            np.testing.assert_allclose([d for _, d in top], td, rtol=1e-9)
    assert any(p < 0 for p in inference._positives(kag, ids.image_paths))  # sketches without a gallery photo


@pytest.mark.parametrize("world,metric", [(2, "euclidean"), (2, "cosine"), (4, "euclidean"), (8, "euclidean")])
def test_sharded_gallery_inference_matches_unsharded(tmp_path, world, metric):
    """13 gallery photos over 2 / 4 / 8 ranks: ragged, at world 8 some ranks hold one"""
    _run(_sharded_inference, str(tmp_path), metric, world=world)


def _allreduce_autograd_model(rank):
    """a model without the HIP engine's flat buffer (vit.VisionTransformer's
    gradients are autograd's param.grad): coalesced buckets of mixed sizes and
    dtypes, every tensor averaged exactly once"""
    import ddp
    m = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    for i, p in enumerate(m.parameters()):
        p.grad = torch.full(p.shape, float((rank + 1) * (i + 1)))
    m[1].bias.grad = None  # a parameter without a gradient is skipped
    ddp.allreduce_gradients(m, bucket_bytes=64)  # several buckets, split at tensor boundaries
    mr = _mean_rank1()
    for i, p in enumerate(m.parameters()):
        if p.grad is not None:
            assert torch.allclose(p.grad, torch.full(p.shape, mr * (i + 1))), i
    ts = [torch.arange(5, dtype=torch.float64) * (rank + 1), torch.ones(3, dtype=torch.bfloat16) * (rank + 1)]
    ddp.allreduce_tensors(ts, bucket_bytes=1 << 20)  # a dtype change starts a new bucket
    assert torch.allclose(ts[0], torch.arange(5, dtype=torch.float64) * mr)
    assert torch.allclose(ts[1].float(), torch.full((3,), mr), rtol=1e-2)
    r = ddp.attach_overlapped_reducer(m)  # no engine: finish() is the plain coalesced all-reduce
    for p in m.parameters():
        if p.grad is not None:
            p.grad.fill_(float(rank))
    r.finish()
    assert all(torch.allclose(p.grad, torch.full(p.shape, mr - 1)) for p in m.parameters() if p.grad is not None)


@pytest.mark.parametrize("world", WORLDS)
def test_allreduce_gradients_without_engine(world):
    _run(_allreduce_autograd_model, world=world)
