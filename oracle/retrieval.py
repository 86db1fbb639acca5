"""Retrieval metrics on CPU in numpy (TEST ORACLE).

Follows /root/reference/inference.py and utils.py:
  get_ranking_position  inference.py:30-57 (name parsing, first matching gallery
                        path, distance, full sort, position of the positive)
  get_topk_images       inference.py:60-69
  process_inference     inference.py:94-136 (rank+1, MRR, topk_acc[rank:] += 1,
                        pandas describe() of ranks)
  find_image_index      utils.py:22-25
  euclidean_distance    utils.py:42  nn.PairwiseDistance(p=2, eps=1e-6): ||x1-x2+eps||
  cosine_distance       utils.py:31-40  1 - cos(x1,x2) (CosineSimilarity eps=1e-8)
  InferenceDataset      data_preparation.py:24-41 (dedup, then sort the gallery paths)

"Exact" distances here are evaluated in float64 from float32 inputs and the
sort is stable on (distance, gallery index): this is the total order the HIP
retrieval path must reproduce bit-exactly (torch.topk leaves the order of
equal distances unspecified, so a tie rule has to be fixed somewhere).
"""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np

EPS = 1e-6


def l2_distances(q: np.ndarray, g: np.ndarray) -> np.ndarray:
    """||q - g_i + eps||_2 for every gallery row, float64.  q [D], g [N, D]."""
    d = (q.astype(np.float64)[None, :] - g.astype(np.float64)) + EPS
    return np.sqrt(np.einsum("nd,nd->n", d, d))


def cosine_distances(q: np.ndarray, g: np.ndarray, eps: float = 1e-8) -> np.ndarray:
    """1 - cos(q, g_i) in float64 with nn.CosineSimilarity's eps: each norm is
    clamped separately, x1.x2 / (max(|x1|, eps) max(|x2|, eps)) (torch 2.10)."""
    q64, g64 = q.astype(np.float64), g.astype(np.float64)
    num = np.einsum("nd,d->n", g64, q64)
    den = np.maximum(np.sqrt(np.einsum("nd,nd->n", g64, g64)), eps) * max(np.sqrt(q64 @ q64), eps)
    return 1.0 - num / den


def distances(q: np.ndarray, g: np.ndarray, metric: str = "euclidean") -> np.ndarray:
    """the reference's distance of inference.py:43-48 for loss_type `metric`"""
    if metric == "euclidean":
        return l2_distances(q, g)
    if metric == "cosine":
        return cosine_distances(q, g)
    raise Exception(f"loss type not correct {metric}")


def order(dist: np.ndarray) -> np.ndarray:
    """Ascending order with ties broken by lower index (stable sort)."""
    return np.argsort(dist, kind="stable")


def topk(dist: np.ndarray, k: int):
    idx = order(dist)[:k]
    return idx, dist[idx]


def rank_of(dist: np.ndarray, pos: int) -> int:
    """0-based position of gallery item `pos` in the stable ascending order."""
    d = dist[pos]
    return int(np.count_nonzero(dist < d) + np.count_nonzero(dist[:pos] == d))


def topk_rank_large(qs: np.ndarray, g: np.ndarray, pos, k: int, metric: str = "euclidean", chunk: int = 16):
    """topk(distances(q, g), k) and rank_of(..., pos) for every query, for
    galleries too large for the per-query float64 loop (1M x 512).  Candidate
    sets come from the float64 GEMM form; every decision is re-made with the
    direct form above, so the answers are those of distances() + stable sort:
      euclidean: |GEMM d^2 - direct d^2| <= 2e-6 sqrt(D) |q - g| + D e-12 + f64
                 rounding, covered by the margin m below;
      cosine:    the GEMM and direct forms differ by f64 rounding only."""
    import torch
    G = torch.from_numpy(np.ascontiguousarray(g)).double()
    gsq = (G * G).sum(1)
    N, D = G.shape
    gn = gsq.sqrt().clamp_min(1e-8)
    out_i = np.zeros((len(qs), k), np.int64)
    out_d = np.zeros((len(qs), k))
    ranks = np.full(len(qs), -1, np.int64)
    for c0 in range(0, len(qs), chunk):
        Qc = torch.from_numpy(np.ascontiguousarray(qs[c0:c0 + chunk])).double()
        dot = Qc @ G.T
        qsq = (Qc * Qc).sum(1, keepdim=True)
        if metric == "euclidean":
            a = qsq + gsq[None, :] - 2.0 * dot                       # ~ key^2
            m = 4e-6 * torch.sqrt(D * (qsq + gsq.max())) + 1e-9 * (qsq + gsq.max()) + 1e-9
        else:
            a = 1.0 - dot / (qsq.sqrt().clamp_min(1e-8) * gn[None, :])  # ~ key
            m = torch.full_like(qsq, 1e-9)
        kth = torch.kthvalue(a, k, dim=1).values[:, None]
        for j in range(Qc.shape[0]):
            qi = c0 + j
            cand = torch.nonzero(a[j] <= kth[j] + 2 * m[j]).flatten().numpy()
            d = distances(qs[qi], g[cand], metric)
            o = np.lexsort((cand, d))[:k]
            out_i[qi], out_d[qi] = cand[o], d[o]
            p = int(pos[qi])
            if p >= 0:
                dp = distances(qs[qi], g[p:p + 1], metric)[0]
                ap = (dp * dp) if metric == "euclidean" else dp
                sure = int((a[j] < ap - m[j]).sum())
                band = torch.nonzero((a[j] >= ap - m[j]) & (a[j] <= ap + m[j])).flatten().numpy()
                db = distances(qs[qi], g[band], metric)
                ranks[qi] = sure + int(((db < dp) | ((db == dp) & (band < p))).sum())
    return out_i, out_d, ranks


def find_image_index(image_paths, name: str) -> int:
    """utils.py:22-25 — first path whose stem equals `name`, else -1."""
    for i, p in enumerate(image_paths):
        if Path(p).stem == name:
            return i
    return -1


def positive_name(sketch_path, image_paths) -> str:
    """inference.py:33-37 sketch-name parsing."""
    stem = Path(sketch_path).stem
    parts = re.split('-', stem)
    if len(parts) <= 2:
        return stem if "artworks" in str(image_paths[0]) else parts[0]
    if len(parts) == 3:
        return parts[1]
    return parts  # the reference leaves a list here; it never matches a stem


def inference_dataset_paths(paths):
    """data_preparation.py:30-31 — dedup keeping first occurrence, then sort."""
    return sorted(dict.fromkeys(paths))


def describe(ranks) -> dict:
    """pandas DataFrame.describe() of the 1-based ranks (ddof=1 std, linear quantiles)."""
    r = np.asarray(ranks, np.float64)
    out = {"count": float(len(r)), "mean": float(r.mean())}
    out["std"] = float(r.std(ddof=1)) if len(r) > 1 else float("nan")
    out["min"] = float(r.min())
    for q, key in ((0.25, "25%"), (0.5, "50%"), (0.75, "75%")):
        out[key] = float(np.quantile(r, q))
    out["max"] = float(r.max())
    return out


def metrics(ranks0, k: int = 10) -> dict:
    """inference.py:116-134 from 0-based ranks; adds mAP@k (one relevant item per
    query => mean of 1/rank over queries whose rank <= k)."""
    ranks1 = [r + 1 for r in ranks0]
    mrr = float(np.mean([1.0 / r for r in ranks1]))
    acc = np.zeros(k)
    for r in ranks0:
        if r < k:
            acc[r:] += 1
    acc /= len(ranks0)
    out = {"mean_reciprocal_rank": mrr}
    out.update(describe(ranks1))
    out["topk_acc"] = [float(a) for a in acc]
    out[f"map@{k}"] = float(np.mean([1.0 / r if r <= k else 0.0 for r in ranks1]))
    return out


def synthetic_gallery(n: int, d: int, q: int, seed_g: int = 7, seed_q: int = 8, noise: float = 0.5):
    """G ~ N(0,1) [n,d]; query i = G[p_i] + noise*N(0,1), p_i = (i*7919) mod n."""
    g = np.random.Generator(np.random.PCG64(seed_g)).standard_normal((n, d), dtype=np.float32)
    pos = (np.arange(q, dtype=np.int64) * 7919) % n
    qs = g[pos] + noise * np.random.Generator(np.random.PCG64(seed_q)).standard_normal((q, d), dtype=np.float32)
    return g, qs.astype(np.float32), pos


def fp32_reference_order(qs: np.ndarray, g: np.ndarray, pos, k: int, metric: str = "euclidean",
                         rows_per_chunk: int = 131072):
    """The reference's own float32 op sequence (inference.py:43-56 and 60-66 on
    the CPU): utils.euclidean_distance = nn.PairwiseDistance(p=2) (or the
    CosineLoss of utils.py:31-40) of one sketch feature against every gallery
    row, distances.topk(k, largest=False) for the top-k list and
    distances.topk(N, largest=False) + position of the positive for the rank.
    Rows are evaluated in chunks (each row's norm is its own reduction, so the
    values equal the one-call result).  Returns (topk idx [Q,k], topk dist
    [Q,k] float32, ranks [Q], -1 without a positive, and the per-query float32
    distance of every top-k / positive item for the tie analysis)."""
    import torch
    G = torch.from_numpy(np.ascontiguousarray(g))
    if metric == "euclidean":
        fn = torch.nn.PairwiseDistance(p=2)
    else:
        cs = torch.nn.CosineSimilarity(dim=1)
        fn = lambda a, b: cs(a, b) * -1 + 1  # noqa: E731  (utils.py:37-38)
    n = G.shape[0]
    out_i = np.zeros((len(qs), k), np.int64)
    out_d = np.zeros((len(qs), k), np.float32)
    ranks = np.full(len(qs), -1, np.int64)
    dists = []
    with torch.no_grad():
        for qi, q in enumerate(qs):
            qt = torch.from_numpy(np.ascontiguousarray(q))[None, :]
            d = torch.cat([fn(qt, G[c0:c0 + rows_per_chunk]) for c0 in range(0, n, rows_per_chunk)])
            v, i = d.topk(k, largest=False)
            out_i[qi], out_d[qi] = i.numpy(), v.numpy()
            p = int(pos[qi])
            if p >= 0:
                _, full = d.topk(n, largest=False)
                ranks[qi] = int((full == p).nonzero().flatten()[0])
            dists.append(d.numpy())
    return out_i, out_d, ranks, dists
