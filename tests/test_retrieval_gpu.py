"""Retrieval vs the float64 oracle (oracle/retrieval.py): bit-exact top-k indices and ranks.

knn.knn is one call of artsbir_pairwise_l2_topk (include/artsbir.h); compute
"bf16" runs the register-resident knn_scan_v2 when D pads to 64/128/256/512 and
knn_scan_kernel otherwise (D = 768 here), "f32" runs knn_scan_kernel in f32."""
import numpy as np
import pytest
import torch

from oracle import retrieval as oret

pytestmark = pytest.mark.gpu


def _oracle(g, qs, pos, k, metric="euclidean"):
    idx, dist, ranks = [], [], []
    for i, q in enumerate(qs):
        d = oret.distances(q, g, metric)
        ti, td = oret.topk(d, k)
        idx.append(ti)
        dist.append(td)
        ranks.append(oret.rank_of(d, pos[i]) if pos[i] >= 0 else -1)
    return np.array(idx), np.array(dist), np.array(ranks)


@pytest.mark.parametrize("metric", ["euclidean", "cosine"])
@pytest.mark.parametrize("compute", ["bf16", "f32"])
@pytest.mark.parametrize("N,D,Q,k", [(5000, 64, 300, 10), (20000, 512, 200, 10), (300, 128, 50, 10),
                                     (4000, 768, 100, 10)])
def test_knn_matches_oracle(compute, metric, N, D, Q, k, dev):
    import knn
    g, qs, pos = oret.synthetic_gallery(N, D, Q)
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), k,
                                 torch.from_numpy(pos).to(dev), compute=compute, metric=metric)
    ri, rd, rr = _oracle(g, qs, pos, k, metric)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_allclose(dist.cpu().numpy(), rd, rtol=1e-12)
    np.testing.assert_array_equal(rank.cpu().numpy(), rr)


def test_knn_ties_and_duplicates(dev):
    """exact duplicate gallery rows: equal distances, order by lower index; ranks follow the same rule."""
    import knn
    rng = np.random.Generator(np.random.PCG64(5))
    base = rng.standard_normal((400, 64), dtype=np.float32)
    g = np.concatenate([base, base[:50], base[:50]])  # rows 400.. duplicate rows 0..49 twice
    perm = rng.permutation(len(g))
    g = g[perm]
    qs = g[[3, 17, 200, 401]] + 0.01 * rng.standard_normal((4, 64), dtype=np.float32)
    pos = np.array([3, 17, 200, 401], dtype=np.int64)
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), 10,
                                 torch.from_numpy(pos).to(dev))
    ri, rd, rr = _oracle(g, qs, pos, 10)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_array_equal(rank.cpu().numpy(), rr)


def test_knn_no_positive_and_far_positive(dev):
    import knn
    g, qs, pos = oret.synthetic_gallery(3000, 64, 40, noise=3.0)  # positives not the nearest
    pos = pos.copy()
    pos[::7] = -1
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), 10,
                                 torch.from_numpy(pos).to(dev))
    ri, rd, rr = _oracle(g, qs, pos, 10)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    r = rank.cpu().numpy()
    np.testing.assert_array_equal(r[pos >= 0], rr[pos >= 0])


def test_pairwise_l2_matches_torch(dev):
    import utils
    a = torch.randn(1, 256)
    b = torch.randn(777, 256)
    ref = torch.nn.PairwiseDistance(p=2)(a, b)
    out = utils.euclidean_distance(a.to(dev), b.to(dev)).cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5)
    c = torch.randn(777, 256)
    assert torch.allclose(utils.euclidean_distance(b.to(dev), c.to(dev)).cpu(),
                          torch.nn.PairwiseDistance(p=2)(b, c), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("compute", ["bf16", "f32"])
@pytest.mark.parametrize("N,D,Q,tpc", [(5000, 100, 300, 1), (9000, 256, 520, 2), (20, 64, 3, 64), (1000, 512, 257, 1)])
def test_knn_chunks_ragged(compute, N, D, Q, tpc, dev):
    """many gallery chunks (small tiles_per_chunk), ragged D (zero-padded), partial query tiles
    (Q not a multiple of 256 / 128) and a gallery smaller than one 32-row tile."""
    import knn
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=1.5)
    pos = pos.copy()
    pos[::5] = -1
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), min(10, N),
                                 torch.from_numpy(pos).to(dev), compute=compute, tiles_per_chunk=tpc)
    ri, rd, rr = _oracle(g, qs, pos, min(10, N))
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_allclose(dist.cpu().numpy(), rd, rtol=1e-12)
    r = rank.cpu().numpy()
    np.testing.assert_array_equal(r[pos >= 0], rr[pos >= 0])


def test_knn_scan_v2_candidates_equal_v1(dev):
    """the two scans produce the same per-(query, chunk) candidate lists and counts (same
    d2 formula and (value, index) order) — compared through the C-ABI directly."""
    import _hip
    from _hip import call, ptr
    N, D, Q, tpc = 6000, 512, 300, 4
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=2.0)
    q = torch.from_numpy(qs).to(dev)
    gg = torch.from_numpy(g).to(dev)
    qsq = torch.empty(Q, device=dev)
    gsq = torch.empty(N, device=dev)
    qc = torch.empty(Q, D, dtype=torch.bfloat16, device=dev)
    gc = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    ga = torch.empty(N, D + 8, dtype=torch.bfloat16, device=dev)
    call("artsbir_rows_prep", _hip.DT_BF16, ptr(q), Q, D, ptr(qsq), ptr(qc), D, _hip.stream())
    call("artsbir_rows_prep", _hip.DT_BF16, ptr(gg), N, D, ptr(gsq), ptr(gc), D, _hip.stream())
    gsq2 = torch.empty(N, device=dev)
    call("artsbir_rows_prep_aug", ptr(gg), N, D, D, ptr(gsq2), ptr(ga), _hip.stream())
    assert torch.equal(gsq, gsq2)
    assert torch.equal(ga[:, :D], gc)
    assert torch.equal(ga[:, D:D + 2].contiguous().view(torch.float32).flatten(), gsq)
    ncand = _hip.lib().artsbir_knn_candidates_per_query(N, tpc)
    # rank band around the 30th-nearest item's approximate distance: exercises counts and the queue
    d2 = (qsq[:, None] + gsq[None, :] - 2.0 * (qc.float() @ gc.float().T))
    lo = d2.kthvalue(30, dim=1).values - 5.0
    hi = lo + 10.0
    out = []
    for v2 in (False, True):
        cnt = torch.zeros(Q, dtype=torch.int32, device=dev)
        unc = torch.zeros(2 * 4096 + 1, dtype=torch.int32, device=dev)
        cd = torch.empty(Q, ncand, device=dev)
        ci = torch.empty(Q, ncand, dtype=torch.int32, device=dev)
        if v2:
            call("artsbir_knn_scan_aug", ptr(qc), ptr(ga), ptr(qsq), float(gsq.max()), Q, N, D, tpc, None, None, 0, 0.0,
                 ptr(lo), ptr(hi),
                 ptr(cnt), ptr(unc), 4096, ptr(cd), ptr(ci), _hip.stream())
        else:
            call("artsbir_knn_scan", _hip.DT_BF16, ptr(qc), ptr(gc), ptr(qsq), ptr(gsq), Q, N, D, tpc, ptr(lo),
                 ptr(hi), ptr(cnt), ptr(unc), 4096, ptr(cd), ptr(ci), _hip.stream())
        n = int(unc[-1])
        pairs = sorted(map(tuple, unc[:2 * min(n, 4096)].view(-1, 2).cpu().tolist()))
        out.append((cd.cpu(), ci.cpu(), cnt.cpu(), n, pairs))
    (cd1, ci1, c1, n1, p1), (cd2, ci2, c2, n2, p2) = out
    # the two MFMA shapes sum the dot products in different orders (f32 rounding), so a
    # near-tie may land on the other side of a list end or band edge; otherwise equal
    same_lists = (ci1.view(Q, -1, 16) == ci2.view(Q, -1, 16)).all(dim=2).float().mean().item()
    assert same_lists >= 0.99, same_lists
    assert (c1 == c2).float().mean().item() >= 0.99
    assert n1 > 0 and abs(n1 - n2) <= max(2, n1 // 100)
    assert len(set(p1) ^ set(p2)) <= max(2, n1 // 50)
    m = ci1 == ci2
    np.testing.assert_allclose(cd1[m].numpy(), cd2[m].numpy(), rtol=1e-5, atol=1e-3)


def test_knn_shards_on_one_gpu_match_oracle(dev):
    """the sharded protocol of knn.knn_sharded run shard by shard on one GPU (uneven
    row shards, positives in every shard and some missing): owner dpos, max-combine,
    per-shard exact top-k and counts, merge_topk, summed ranks == the oracle."""
    import knn
    N, D, Q, k = 7000, 512, 300, 10
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=1.5)
    pos = pos.copy()
    pos[::9] = -1
    q = torch.from_numpy(qs).to(dev)
    gg = torch.from_numpy(g).to(dev)
    p = torch.from_numpy(pos).to(dev)
    bounds = [0, 1234, 4000, N]
    shards = [(b0, gg[b0:b1].contiguous()) for b0, b1 in zip(bounds[:-1], bounds[1:])]
    dpos = torch.stack([knn.shard_positive_distances(q, sh, b0, p) for b0, sh in shards]).max(dim=0).values
    outs = [knn.knn(q, sh, k, p, g_base=b0, dpos=dpos) for b0, sh in shards]
    mi, md = knn.merge_topk_device(torch.stack([o[1] for o in outs]), torch.stack([o[0] for o in outs]), k)
    rank = sum(o[2] for o in outs)
    ri, rd, rr = _oracle(g, qs, pos, k)
    np.testing.assert_array_equal(mi.cpu().numpy(), ri)
    np.testing.assert_allclose(md.cpu().numpy(), rd, rtol=1e-12)
    r = rank.cpu().numpy()
    np.testing.assert_array_equal(r[pos >= 0], rr[pos >= 0])


def test_knn_shard_shorter_than_k(dev):
    """a shard with fewer rows than k pads its list with index -1 / +inf, and the
    device merge of the shards still gives the oracle's top-k"""
    import knn
    N, D, Q, k = 300, 64, 40, 10
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=1.0)
    q, gg, p = torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), torch.from_numpy(pos).to(dev)
    bounds = [0, 4, 293, N]  # 4 and 7 rows
    shards = [(b0, gg[b0:b1].contiguous()) for b0, b1 in zip(bounds[:-1], bounds[1:])]
    dpos = torch.stack([knn.shard_positive_distances(q, sh, b0, p) for b0, sh in shards]).max(dim=0).values
    outs = [knn.knn(q, sh, k, p, g_base=b0, dpos=dpos) for b0, sh in shards]
    short = outs[0][0].cpu().numpy()
    assert (short[:, 4:] == -1).all() and np.isinf(outs[0][1].cpu().numpy()[:, 4:]).all()
    mi, md = knn.merge_topk_device(torch.stack([o[1] for o in outs]), torch.stack([o[0] for o in outs]), k)
    ri, rd, rr = _oracle(g, qs, pos, k)
    np.testing.assert_array_equal(mi.cpu().numpy(), ri)
    np.testing.assert_array_equal(sum(o[2] for o in outs).cpu().numpy(), rr)


@pytest.mark.parametrize("metric", ["euclidean", "cosine"])
def test_knn_near_ties_duplicates_and_scaled_rows(metric, dev):
    """planted exact duplicates (equal keys: lower index first), near-ties one ulp
    apart, positively scaled copies (equal cosine keys up to rounding) and a zero
    row (cos eps clamp): the exact (key, index) order of the oracle"""
    import knn
    rng = np.random.Generator(np.random.PCG64(11))
    base = rng.standard_normal((3000, 128), dtype=np.float32)
    g = base.copy()
    g[1000:1040] = base[0:40]                         # exact duplicates
    g[1040:1080] = base[0:40] * np.float32(2.5)       # scaled copies
    g[1080:1120] = np.nextafter(base[0:40], np.float32(np.inf))  # one-ulp neighbours
    g[1200] = 0.0
    qs = base[0:40] + np.float32(0.05) * rng.standard_normal((40, 128), dtype=np.float32)
    qs[5] = 0.0
    pos = np.arange(40, dtype=np.int64)
    pos[7] = 1200
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), 10,
                                 torch.from_numpy(pos).to(dev), metric=metric)
    ri, rd, rr = _oracle(g, qs, pos, 10, metric)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_allclose(dist.cpu().numpy(), rd, rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(rank.cpu().numpy(), rr)


def test_knn_fallbacks_on_device(dev):
    """the device fallbacks of the one-call path: k larger than the chunk lists can
    hold (exhaustive exact top-k of flagged queries) and an uncertain-queue overflow
    (exhaustive exact recount) both give the oracle's answers"""
    import _hip
    import knn
    g, qs, pos = oret.synthetic_gallery(100, 64, 30, noise=2.0)
    q, gg, p = torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), torch.from_numpy(pos).to(dev)
    idx, dist, rank, _ = knn.knn(q, gg, 40, p)  # one 128-row tile -> 16 candidates < 40
    ri, rd, rr = _oracle(g, qs, pos, 40)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_allclose(dist.cpu().numpy(), rd, rtol=1e-12)
    g, qs, pos = oret.synthetic_gallery(5000, 128, 64, noise=4.0)
    old = _hip.lib().artsbir_knn_set_unc_cap(8)
    try:
        idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), 10,
                                     torch.from_numpy(pos).to(dev))
    finally:
        _hip.lib().artsbir_knn_set_unc_cap(old)
    ri, rd, rr = _oracle(g, qs, pos, 10)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_array_equal(rank.cpu().numpy(), rr)


def test_topk_merge_device_vs_host(dev):
    """artsbir_topk_merge == the host restatement merge_topk, with cross-list ties
    and empty (-1) entries"""
    import knn
    rng = np.random.Generator(np.random.PCG64(3))
    ns, Q, k = 5, 70, 12
    d = np.round(rng.random((ns, Q, k)) * 8) / 8  # many exact ties
    i = rng.permutation(ns * Q * k).reshape(ns, Q, k).astype(np.int64)
    i[1, :, 7:] = -1
    d[1, :, 7:] = np.inf
    td, ti = torch.from_numpy(d), torch.from_numpy(i)
    hi, hd = knn.merge_topk(list(ti), list(td), k)
    di, dd = knn.merge_topk_device(td.to(dev), ti.to(dev), k)
    np.testing.assert_array_equal(di.cpu().numpy(), hi.numpy())
    np.testing.assert_array_equal(dd.cpu().numpy(), hd.numpy())


@pytest.mark.parametrize("metric", ["euclidean", "cosine"])
def test_knn_c4_gallery_sampled_queries(metric, dev):
    """C4's full gallery (1M x 512, N(0,1), seed 7) with queries at noise 3.0, so that
    ranks spread (mAP@10 < 1): 64 sampled queries' top-10 and ranks vs the oracle"""
    import knn
    N, D, Q, k = 1_000_000, 512, 64, 10
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=3.0)
    ri, rd, rr = oret.topk_rank_large(qs, g, pos, k, metric)
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), k,
                                 torch.from_numpy(pos).to(dev), metric=metric)
    np.testing.assert_array_equal(idx.cpu().numpy(), ri)
    np.testing.assert_allclose(dist.cpu().numpy(), rd, rtol=1e-12)
    np.testing.assert_array_equal(rank.cpu().numpy(), rr)
    r1 = rr + 1
    assert np.mean(np.where(r1 <= k, 1.0 / r1, 0.0)) < 1.0  # a workload where ranks spread


@pytest.mark.parametrize("compute", ["bf16", "f32"])
def test_knn_against_committed_golden_fixture(compute, dev):
    """tests/golden/retrieval.npz (duplicates at rows 0 / 4000, queries without a
    positive) through the library: top-10, distances and ranks as committed."""
    import os
    import sys
    import knn
    golden = os.path.join(os.path.dirname(__file__), "golden")
    sys.path.insert(0, golden)
    import make_golden
    gold = np.load(os.path.join(golden, "retrieval.npz"), allow_pickle=False)
    g, qs, pos = make_golden.golden_gallery()
    np.testing.assert_array_equal(gold["positives"], pos)
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), 10,
                                 torch.from_numpy(pos).to(dev), compute=compute)
    np.testing.assert_array_equal(idx.cpu().numpy(), gold["topk_idx"])
    np.testing.assert_allclose(dist.cpu().numpy(), gold["topk_dist"], rtol=1e-12)
    r = rank.cpu().numpy()
    want = gold["ranks"]
    np.testing.assert_array_equal(np.where(pos >= 0, r, len(g)), want)
