"""Batched exact retrieval on libartsbir_hip (single GPU and gallery-sharded).

Replaces the per-query loop of inference.py:30-69: model(sketch) ->
utils.euclidean_distance(q[1,D], G[N,D]) (or utils.cosine_distance) ->
distances.topk(N, largest=False) -> position of the positive, and
get_topk_images' topk(k).  All queries are answered by ONE library call,
artsbir_pairwise_l2_topk (include/artsbir.h): a fused bf16 MFMA scan over the
gallery, then exact f64 decisions — distances of the f32 features, ties broken
by the lower gallery index (oracle/retrieval.py) — with every fallback on the
device and no host synchronisation.

Sharding: every rank holds rows [g_base, g_base + n) of the
gallery.  The positive's exact key comes from its owning shard (all_reduce MAX),
every rank answers all queries on its shard, one all_gather of the per-shard
(k indices, k keys) lists is merged on the device (artsbir_topk_merge) and the
per-shard ranks are summed (all_reduce SUM).
"""
from __future__ import annotations

import torch

import _hip
from _hip import call, ptr

METRICS = {"euclidean": 0, "cosine": 1}
KMAX = 64


def _s():
    return _hip.stream()


def _metric(metric) -> int:
    if metric not in METRICS:
        raise Exception(f"loss type not correct {metric}")  # inference.py:48
    return METRICS[metric]


def knn(queries: torch.Tensor, gallery: torch.Tensor, k: int = 10, positives: torch.Tensor | None = None,
        compute: str = "bf16", g_base: int = 0, dpos: torch.Tensor | None = None,
        tiles_per_chunk: int | None = None, metric: str = "euclidean"):
    """Exact top-k and rank of the positive, one library call.

    queries [Q, D], gallery [N, D] (float, CUDA).  positives: int64 [Q] global
    gallery index of each query's positive (-1: none) or None.  Returns
    (idx int64 [Q, k] global indices, dist float64 [Q, k], rank int64 [Q] or
    None, dpos float64 [Q] or None).  metric "euclidean" orders by
    ||q - g + 1e-6|| (utils.py:42), "cosine" by 1 - cos (utils.py:31-40); dist
    holds that key.  With g_base / dpos this is one shard of a larger gallery
    (dpos: the exact key of positives living in other shards, -1 otherwise) and
    a shard shorter than k pads with index -1 / distance +inf."""
    if not (queries.is_cuda and gallery.is_cuda):
        raise RuntimeError("knn on libartsbir_hip needs CUDA tensors")
    m = _metric(metric)
    q = queries.detach().contiguous().float()
    g = gallery.detach().contiguous().float()
    Q, D = q.shape
    N = g.shape[0]
    shard = g_base != 0 or dpos is not None
    if k > N and not shard:
        raise ValueError(f"k={k} > gallery size {N}")  # torch.topk(k) on N < k raises too
    if not 1 <= k <= KMAX:
        raise ValueError(f"k={k} outside 1..{KMAX}")
    dev = q.device
    dt = _hip.DT_BF16 if compute == "bf16" else _hip.DT_F32
    tpc = int(tiles_per_chunk or 0)
    out_i = torch.empty(Q, k, dtype=torch.int64, device=dev)
    out_d = torch.empty(Q, k, dtype=torch.float64, device=dev)
    rank = out_dp = pos = None
    if N == 0:
        out_i.fill_(-1)
        out_d.fill_(float("inf"))
        if positives is not None:
            rank = torch.zeros(Q, dtype=torch.int64, device=dev)
            out_dp = dpos.to(dev, torch.float64).clone() if dpos is not None else torch.full(
                (Q,), -1.0, dtype=torch.float64, device=dev)
        return out_i, out_d, rank, out_dp
    if positives is not None:
        pos = positives.to(dev, torch.int64).contiguous()
        rank = torch.empty(Q, dtype=torch.int64, device=dev)
        out_dp = torch.empty(Q, dtype=torch.float64, device=dev)
        if dpos is not None:
            dpos = dpos.to(dev, torch.float64).contiguous()
    nbytes = int(_hip.lib().artsbir_pairwise_l2_topk_workspace(dt, Q, N, D, k, tpc))
    if nbytes < 0:
        raise _hip.HipError(_hip.lib().artsbir_last_error().decode())
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    call("artsbir_pairwise_l2_topk", dt, m, ptr(q), Q, ptr(g), N, D, k, ptr(pos), ptr(dpos), g_base, tpc,
         ptr(out_i), ptr(out_d), ptr(rank), ptr(out_dp), ptr(ws), nbytes, _s(),
         kernel="auto", flops=2.0 * Q * N * D)
    return out_i, out_d, rank, out_dp


def shard_positive_distances(queries, gallery_shard, g_base: int, positives, metric: str = "euclidean"):
    """f64 [Q]: the exact key of each query's positive if it lies in this shard's
    rows [g_base, g_base + n), -1 for the others (and for no positive)."""
    q = queries.detach().contiguous().float()
    g = gallery_shard.detach().contiguous().float()
    Q, D = q.shape
    pos = positives.to(q.device, torch.int64).contiguous()
    out = torch.empty(Q, dtype=torch.float64, device=q.device)
    call("artsbir_positive_key", _metric(metric), ptr(q), Q, ptr(g), g.shape[0], D, ptr(pos), g_base, ptr(out), _s())
    return out


def merge_topk_device(all_d: torch.Tensor, all_i: torch.Tensor, k: int):
    """[nshard, Q, k] gathered lists -> global top-k by (distance, index) on the GPU"""
    ns, Q, _ = all_d.shape
    out_i = torch.empty(Q, k, dtype=torch.int64, device=all_d.device)
    out_d = torch.empty(Q, k, dtype=torch.float64, device=all_d.device)
    call("artsbir_topk_merge", ns, Q, k, ptr(all_d.contiguous()), ptr(all_i.contiguous()), ptr(out_i), ptr(out_d),
         _s())
    return out_i, out_d


def merge_topk(all_i, all_d, k):
    """Host restatement of artsbir_topk_merge (CPU tensors; the gloo tests):
    per-shard top-k lists ([Q, k] each) -> global top-k ordered by (distance,
    global index); entries with index -1 (short shards) sort last."""
    ci = torch.cat(list(all_i), 1)
    cd = torch.cat(list(all_d), 1).clone()
    cd[ci < 0] = float("inf")
    o1 = torch.sort(ci, dim=1, stable=True).indices  # by index, then stably by distance
    ci, cd = torch.gather(ci, 1, o1), torch.gather(cd, 1, o1)
    o2 = torch.sort(cd, dim=1, stable=True).indices[:, :k]
    return torch.gather(ci, 1, o2), torch.gather(cd, 1, o2)


def knn_sharded(queries, gallery_shard, g_base: int, k: int = 10, positives=None, compute="bf16",
                metric: str = "euclidean", *, local_search=None, positive_keys=None, merge=None):
    """Gallery sharded over the ranks of the default process group (RCCL on the
    GPUs): every rank passes ITS shard [g_base, g_base + n) and the same queries.
    The collective protocol is: all_reduce(MAX) of the positives' keys, the
    local search, all_gather of (k keys, k indices) per query, merge, and
    all_reduce(SUM) of the per-shard ranks.  local_search / positive_keys / merge
    default to the library (knn, shard_positive_distances, merge_topk_device);
    the gloo tests substitute CPU stand-ins to run this same protocol code."""
    import torch.distributed as dist
    local_search = local_search or knn
    positive_keys = positive_keys or shard_positive_distances
    merge = merge or merge_topk_device
    world = dist.get_world_size()
    dpos = None
    if positives is not None:
        dpos = positive_keys(queries, gallery_shard, g_base, positives, metric=metric)
        dist.all_reduce(dpos, op=dist.ReduceOp.MAX)  # -1 everywhere but the owner
    idx, dd, rank, _ = local_search(queries, gallery_shard, k, positives, compute, g_base=g_base, dpos=dpos,
                                    metric=metric)
    Q = idx.shape[0]
    all_i = torch.empty(world * Q, k, dtype=idx.dtype, device=idx.device)  # rank-major [world][Q][k]
    all_d = torch.empty(world * Q, k, dtype=dd.dtype, device=dd.device)
    dist.all_gather_into_tensor(all_i, idx.contiguous())
    dist.all_gather_into_tensor(all_d, dd.contiguous())
    out_i, out_d = merge(all_d.view(world, Q, k), all_i.view(world, Q, k), k)
    if rank is not None:
        dist.all_reduce(rank, op=dist.ReduceOp.SUM)
    return out_i, out_d, rank
