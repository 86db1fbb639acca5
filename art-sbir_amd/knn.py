"""Batched exact L2 retrieval on libartsbir_hip (single GPU and gallery-sharded).

Replaces the per-query loop of inference.py:104-121 (model(sketch) ->
utils.euclidean_distance(q[1,D], G[N,D]) -> distances.topk(N) -> position of
the positive; get_topk_images topk(k)).  All queries are scored at once by the
fused MFMA scan (retrieval.hip); the final order is exact: f64 distances of
the f32 features, ties broken by the lower gallery index (oracle/retrieval.py).

Sharding: every rank holds rows [g_base, g_base + n) of the
gallery, computes its local exact top-k and its count of items closer than the
positive; one all_gather of (k indices, k distances) per query and one
all_reduce of the counts give the global answer.
"""
from __future__ import annotations

import torch

import _hip
from _hip import call, ptr

# |approx d^2 - exact d^2| <= REL * |q| * max|g| + 1e-3 for the approximate squared
# distance |q|^2+|g|^2-2q.g (bf16 operands + f32 accumulation, or exact f32
# MFMA); derivation in csrc/retrieval.hip
REL = {_hip.DT_BF16: 2.0 ** -6 + 2.0 ** -12, _hip.DT_F32: 2.0 ** -14}
TILES_PER_CHUNK = {"v1": 64, "v2": 256}  # gallery chunk = tiles_per_chunk * 128 rows (measured best)
UNC_CAP = 1 << 20
PREPASS_ROWS = 0  # off: see knn() docstring


def _s():
    return _hip.stream()


def knn(queries: torch.Tensor, gallery: torch.Tensor, k: int = 10, positives: torch.Tensor | None = None,
        compute: str = "bf16", g_base: int = 0, dpos: torch.Tensor | None = None,
        tiles_per_chunk: int | None = None, scan: str = "auto", prepass_rows: int = PREPASS_ROWS,
        share_bound: bool = False):
    """Exact top-k and rank of the positive.

    queries [Q, D], gallery [N, D] (float, CUDA).  positives: int64 [Q] global
    gallery index of each query's positive (-1: none) or None.  Returns
    (idx int64 [Q, k] global indices, dist float64 [Q, k], rank int64 [Q] or None,
    dpos float64 [Q] or None).  With g_base/dpos this is one shard of a larger
    gallery: dpos must then hold the exact positive distance (or -1) for rows
    whose positive lives in another shard.  scan: "auto" (the register-resident
    bf16 scan knn_scan_v2 on an augmented gallery copy when D pads to 64, 128,
    256 or 512, else knn_scan_kernel), "v1" (always knn_scan_kernel).
    prepass_rows: with the v2 scan, k <= 16 and N >= 4 * prepass_rows, a pre-pass
    over the first prepass_rows gallery rows seeds every query's list threshold
    with (its k-th smallest approximate d^2 there) + 2 eps: an upper bound of
    (k-th smallest over the whole gallery) + 2 eps, which is all the exact merge
    needs, so the lists stay exact.  Off by default: on the C4 workload the 2 eps
    margin leaves that bound looser than each chunk's own 16th-smallest value, so
    more items pass the scan's prefilter (measured 41 ms vs 24 ms).
    share_bound: with the v2 scan and k <= 16, the chunks of one launch publish
    their k-th smallest approximate d^2 per query and tighten each other's list
    thresholds to (best published) + 2 eps while they run — the same bound as the
    pre-pass, but from the whole gallery as it is scanned.  Off by default: it
    cuts list insertions 3x but not the scan's slow-path entries (measured 20.4
    vs 19.8 ms at 1M x 512).
    """
    if not (queries.is_cuda and gallery.is_cuda):
        raise RuntimeError("knn on libartsbir_hip needs CUDA tensors")
    q = queries.detach().contiguous().float()
    g = gallery.detach().contiguous().float()
    Q, D = q.shape
    N = g.shape[0]
    dev = q.device
    dt = _hip.DT_BF16 if compute == "bf16" else _hip.DT_F32
    tdt = torch.bfloat16 if dt == _hip.DT_BF16 else torch.float32
    rel = REL[dt]
    if k > N:
        raise ValueError(f"k={k} > gallery size {N}")
    step = 64 if dt == _hip.DT_BF16 else 32
    Dp = (D + step - 1) // step * step  # MFMA scan: zero-padded compute copies
    use_v2 = (scan == "auto" and dt == _hip.DT_BF16 and bool(_hip.lib().artsbir_knn_scan_aug_supported(Dp)))
    if tiles_per_chunk is None:
        tiles_per_chunk = TILES_PER_CHUNK["v2" if use_v2 else "v1"]
    if k > _hip.lib().artsbir_knn_candidates_per_query(N, tiles_per_chunk):
        tiles_per_chunk = 1  # more chunks -> more candidates per query (k <= 16 * chunks)
        if k > _hip.lib().artsbir_knn_candidates_per_query(N, 1):
            raise ValueError(f"k={k} exceeds the candidate capacity for a gallery of {N}")
    qsq = torch.empty(Q, dtype=torch.float32, device=dev)
    gsq = torch.empty(N, dtype=torch.float32, device=dev)
    qc = torch.empty(Q, Dp, dtype=tdt, device=dev)
    call("artsbir_rows_prep", dt, ptr(q), Q, D, ptr(qsq), ptr(qc), Dp, _s())
    if use_v2:  # [N][Dp + 8] bf16 rows carrying their f32 |g|^2 (one DMA block per tile)
        gc = torch.empty(N, Dp + 8, dtype=tdt, device=dev)
        call("artsbir_rows_prep_aug", ptr(g), N, D, Dp, ptr(gsq), ptr(gc), _s())
    else:
        gc = torch.empty(N, Dp, dtype=tdt, device=dev)
        call("artsbir_rows_prep", dt, ptr(g), N, D, ptr(gsq), ptr(gc), Dp, _s())
    gsq_max = float(gsq.max().item()) if N else 0.0

    lo = hi = pos = None
    if positives is not None:
        pos = positives.to(dev, torch.int64).contiguous()
        if dpos is None:
            dpos = torch.full((Q,), -1.0, dtype=torch.float64, device=dev)
        else:
            dpos = dpos.to(dev, torch.float64).contiguous().clone()
        lo = torch.empty(Q, dtype=torch.float32, device=dev)
        hi = torch.empty(Q, dtype=torch.float32, device=dev)
        call("artsbir_knn_band", ptr(q), ptr(g), ptr(pos), g_base, N, ptr(qsq), gsq_max, Q, D, rel, ptr(dpos),
             ptr(lo), ptr(hi), _s())
    cnt = torch.zeros(Q, dtype=torch.int32, device=dev)
    unc = torch.zeros(2 * UNC_CAP + 1, dtype=torch.int32, device=dev)
    ncand = _hip.lib().artsbir_knn_candidates_per_query(N, tiles_per_chunk)
    nchunks = ncand // 16
    cand_d = torch.empty(Q, ncand, dtype=torch.float32, device=dev)
    cand_i = torch.empty(Q, ncand, dtype=torch.int32, device=dev)
    if use_v2:
        thr0 = None
        if k <= 16 and prepass_rows >= 128 and N >= 4 * prepass_rows:
            S = prepass_rows // 128 * 128
            tpc0 = 8 if S % 1024 == 0 else 1
            nc0 = _hip.lib().artsbir_knn_candidates_per_query(S, tpc0)
            cd0 = torch.empty(Q, nc0, dtype=torch.float32, device=dev)
            ci0 = torch.empty(Q, nc0, dtype=torch.int32, device=dev)
            call("artsbir_knn_scan_aug", ptr(qc), ptr(gc), ptr(qsq), gsq_max, Q, S, Dp, tpc0, None, None, 0, 0.0,
                 None, None, ptr(cnt), ptr(unc), UNC_CAP, ptr(cd0), ptr(ci0), _s(), kernel="knn_scan_v2_kernel(prepass)",
                 flops=2.0 * Q * S * D)
            # k-th smallest approximate d^2 of the subset (its k smallest are in the chunk lists)
            kth = torch.where(ci0 >= 0, cd0.double(), torch.inf).kthvalue(k, dim=1).values
            eps = rel * torch.sqrt(qsq.double() * gsq_max) + 1e-3
            thr0 = ((kth + 2.0 * eps) * (1.0 + 1e-6) + 1e-3).float()
        # chunks share their k-th smallest approximate d^2 (tighter list thresholds, same exact result)
        kbound = torch.full((Q,), -8388608, dtype=torch.int32, device=dev) if (share_bound and k <= 16) else None
        call("artsbir_knn_scan_aug", ptr(qc), ptr(gc), ptr(qsq), gsq_max, Q, N, Dp, tiles_per_chunk, ptr(thr0),
             ptr(kbound), k, rel, ptr(lo), ptr(hi), ptr(cnt), ptr(unc), UNC_CAP, ptr(cand_d), ptr(cand_i), _s(),
             kernel="knn_scan_v2_kernel", flops=2.0 * Q * N * D)
    else:
        call("artsbir_knn_scan", dt, ptr(qc), ptr(gc), ptr(qsq), ptr(gsq), Q, N, Dp, tiles_per_chunk, ptr(lo),
             ptr(hi), ptr(cnt), ptr(unc), UNC_CAP, ptr(cand_d), ptr(cand_i), _s(), kernel="knn_scan_kernel",
             flops=2.0 * Q * N * D)
    out_i = torch.empty(Q, k, dtype=torch.int64, device=dev)
    out_d = torch.empty(Q, k, dtype=torch.float64, device=dev)
    flag = torch.empty(Q, dtype=torch.int32, device=dev)
    call("artsbir_knn_merge", ptr(q), ptr(g), D, Q, nchunks, ptr(cand_d), ptr(cand_i), ptr(qsq), gsq_max, rel,
         g_base, k, ptr(out_i), ptr(out_d), ptr(flag), _s())
    rank = None
    if positives is not None:
        call("artsbir_knn_uncertain", ptr(q), ptr(g), D, ptr(unc), UNC_CAP, ptr(dpos), ptr(pos), g_base, ptr(cnt),
             _s())
        if int(unc[2 * UNC_CAP].item()) > UNC_CAP:
            cnt = _exact_counts(q, g, pos, dpos, g_base)
        rank = cnt.to(torch.int64)
    # rare: a chunk list could have hidden a true top-k item -> exhaustive exact pass
    bad = torch.nonzero(flag).flatten().tolist()
    for qi in bad:
        d = torch.empty(N, dtype=torch.float64, device=dev)
        call("artsbir_knn_exact_all", ptr(q[qi]), ptr(g), D, N, ptr(d), _s())
        order = _stable_order(d)[:k]
        out_i[qi] = order + g_base
        out_d[qi] = d[order]
    return out_i, out_d, rank, dpos


def _stable_order(d: torch.Tensor) -> torch.Tensor:
    return torch.sort(d, stable=True).indices


def _exact_counts(q, g, pos, dpos, g_base):
    """exhaustive exact rank counts (uncertain-queue overflow fallback)."""
    Q, D = q.shape
    N = g.shape[0]
    cnt = torch.zeros(Q, dtype=torch.int32, device=q.device)
    d = torch.empty(N, dtype=torch.float64, device=q.device)
    idx = torch.arange(N, device=q.device) + g_base
    for qi in range(Q):
        if dpos[qi].item() < 0:
            continue
        call("artsbir_knn_exact_all", ptr(q[qi]), ptr(g), D, N, ptr(d), _s())
        dp = dpos[qi]
        cnt[qi] = int(((d < dp) | ((d == dp) & (idx < pos[qi]))).sum().item())
    return cnt


def shard_positive_distances(queries, gallery_shard, g_base: int, positives):
    """f64 [Q]: the exact ||q - g_pos + 1e-6|| for queries whose positive lies in this
    shard's rows [g_base, g_base + n), -1 for the others (and for no positive).  One
    knn_band launch: the same exact_l2 as every other exact decision of the scan."""
    q = queries.detach().contiguous().float()
    g = gallery_shard.detach().contiguous().float()
    Q, D = q.shape
    dev = q.device
    pos = positives.to(dev, torch.int64).contiguous()
    dpos = torch.full((Q,), -1.0, dtype=torch.float64, device=dev)
    qsq = torch.zeros(Q, dtype=torch.float32, device=dev)  # only feeds lo/hi, unused here
    lo = torch.empty(Q, dtype=torch.float32, device=dev)
    hi = torch.empty(Q, dtype=torch.float32, device=dev)
    call("artsbir_knn_band", ptr(q), ptr(g), ptr(pos), g_base, g.shape[0], ptr(qsq), 0.0, Q, D, 0.0, ptr(dpos),
         ptr(lo), ptr(hi), _s())
    return dpos


def knn_sharded(queries, gallery_shard, g_base: int, k: int = 10, positives=None, compute="bf16"):
    """Gallery sharded over the ranks of the default process group (RCCL):
    every rank passes ITS shard [g_base, g_base + n) and the same queries."""
    import torch.distributed as dist
    world = dist.get_world_size()
    Q = queries.shape[0]
    dpos = None
    if positives is not None:
        # exact positive distance from the owning shard, then shared (max of -1s)
        dpos = shard_positive_distances(queries, gallery_shard, g_base, positives)
        dist.all_reduce(dpos, op=dist.ReduceOp.MAX)
    idx, dd, rank, _ = knn(queries, gallery_shard, k, positives, compute, g_base=g_base, dpos=dpos)
    all_i = [torch.empty_like(idx) for _ in range(world)]
    all_d = [torch.empty_like(dd) for _ in range(world)]
    dist.all_gather(all_i, idx)
    dist.all_gather(all_d, dd)
    out_i, out_d = merge_topk(all_i, all_d, k)
    if rank is not None:
        dist.all_reduce(rank, op=dist.ReduceOp.SUM)
    return out_i, out_d, rank


def merge_topk(all_i, all_d, k):
    """Merge per-shard top-k lists ([Q, k] each) into the global top-k ordered by
    (distance, global index); entries with index -1 (short shards) sort last."""
    ci = torch.cat(list(all_i), 1)
    cd = torch.cat(list(all_d), 1).clone()
    cd[ci < 0] = float("inf")
    # stable sort by index, then stable sort by distance == lexicographic (distance, index)
    o1 = torch.sort(ci, dim=1, stable=True).indices
    ci, cd = torch.gather(ci, 1, o1), torch.gather(cd, 1, o1)
    o2 = torch.sort(cd, dim=1, stable=True).indices[:, :k]
    return torch.gather(ci, 1, o2), torch.gather(cd, 1, o2)
