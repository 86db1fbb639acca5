"""The N>1 paths on CPU with the gloo backend, world_size 2:
gradient averaging over the flat gradient buffer (ddp.py), rank-0 parameter
and BN-buffer broadcast, and the gallery-sharded retrieval protocol of
knn.knn_sharded (per-shard exact top-k + rank counts -> all_gather/all_reduce
-> merge_topk) against the unsharded oracle."""
import os
import socket
import types

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(fn, *args):
    port = _free_port()
    mp.spawn(_entry, args=(fn, port, args), nprocs=WORLD, join=True)


def _entry(rank, fn, port, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _allreduce(rank):
    import ddp
    n = 1000
    flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
    model = types.SimpleNamespace(_hip_engine=types.SimpleNamespace(_grads=types.SimpleNamespace(flat=flat)))
    ddp.allreduce_gradients(model, bucket_bytes=256)  # 64-element buckets, last one ragged
    want = torch.arange(n, dtype=torch.float32) * 1.5
    assert torch.allclose(flat, want), (flat - want).abs().max()


def test_allreduce_gradients_averages_flat_buffer():
    _run(_allreduce)


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


def test_broadcast_parameters_and_buffers():
    _run(_broadcast)


def _sharded(rank, k):
    import knn
    from oracle import retrieval as oret
    g, qs, pos = oret.synthetic_gallery(1000, 16, 32, seed_g=5, seed_q=6)
    g[900:910] = g[0:10]  # duplicates straddling the shard boundary -> cross-shard ties
    qs[:4] = g[:4]
    bounds = [0, 537, 1000]  # ragged shards
    lo, hi = bounds[rank], bounds[rank + 1]
    idx = np.zeros((len(qs), k), np.int64)
    dd = np.full((len(qs), k), np.inf)
    cnt = np.zeros(len(qs), np.int64)
    for i, q in enumerate(qs):
        d_full = oret.l2_distances(q, g)
        dpos = d_full[pos[i]]  # exact positive distance, shared by the owner shard (all_reduce MAX)
        d = d_full[lo:hi]
        ti, td = oret.topk(d, min(k, hi - lo))
        idx[i, :len(ti)] = ti + lo
        dd[i, :len(td)] = td
        if len(ti) < k:
            idx[i, len(ti):] = -1
        gi = np.arange(lo, hi)
        cnt[i] = int(((d < dpos) | ((d == dpos) & (gi < pos[i]))).sum())
    ti, td, c = torch.from_numpy(idx), torch.from_numpy(dd), torch.from_numpy(cnt)
    all_i = [torch.empty_like(ti) for _ in range(WORLD)]
    all_d = [torch.empty_like(td) for _ in range(WORLD)]
    dist.all_gather(all_i, ti)
    dist.all_gather(all_d, td)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    mi, md = knn.merge_topk(all_i, all_d, k)
    for i, q in enumerate(qs):
        d_full = oret.l2_distances(q, g)
        ri, rd = oret.topk(d_full, k)
        np.testing.assert_array_equal(mi[i].numpy(), ri)
        np.testing.assert_array_equal(md[i].numpy(), rd)
        assert c[i].item() == oret.rank_of(d_full, pos[i])


def test_sharded_retrieval_protocol_matches_unsharded_oracle():
    _run(_sharded, 10)


def test_merge_topk_short_shards():
    import knn
    a_i = torch.tensor([[3, -1, -1]])
    a_d = torch.tensor([[0.5, 0.0, 0.0]], dtype=torch.float64)
    b_i = torch.tensor([[7, 1, 9]])
    b_d = torch.tensor([[0.5, 0.7, 0.9]], dtype=torch.float64)
    i, d = knn.merge_topk([a_i, b_i], [a_d, b_d], 3)
    assert i.tolist() == [[3, 7, 1]] and d.tolist() == [[0.5, 0.5, 0.7]]
