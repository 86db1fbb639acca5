"""Retrieval kernels vs the float64 oracle (oracle/retrieval.py): bit-exact top-k indices and ranks."""
import numpy as np
import pytest
import torch

from oracle import retrieval as oret

pytestmark = pytest.mark.gpu


def _oracle(g, qs, pos, k):
    idx, dist, ranks = [], [], []
    for i, q in enumerate(qs):
        d = oret.l2_distances(q, g)
        ti, td = oret.topk(d, k)
        idx.append(ti)
        dist.append(td)
        ranks.append(oret.rank_of(d, pos[i]) if pos[i] >= 0 else -1)
    return np.array(idx), np.array(dist), np.array(ranks)


@pytest.mark.parametrize("compute", ["bf16", "f32"])
@pytest.mark.parametrize("N,D,Q,k", [(5000, 64, 300, 10), (20000, 512, 200, 10), (300, 128, 50, 10)])
def test_knn_matches_oracle(compute, N, D, Q, k, dev):
    import knn
    g, qs, pos = oret.synthetic_gallery(N, D, Q)
    idx, dist, rank, _ = knn.knn(torch.from_numpy(qs).to(dev), torch.from_numpy(g).to(dev), k,
                                 torch.from_numpy(pos).to(dev), compute=compute)
    ri, rd, rr = _oracle(g, qs, pos, k)
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
