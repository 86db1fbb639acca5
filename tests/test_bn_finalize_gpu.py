"""BatchNorm slot finalizes (artsbir_bn_finalize_seg / artsbir_bn_bwd_finalize_seg,
csrc/elementwise.hip) against an f64 numpy restatement of the same sums: per channel
the ARTSBIR_NSLOT replica slots in four quarters of eight, the quarters added in
order.  Forward: mean, var = E[y^2] - mean^2 (clamped at 0), istd, scale, beta and
the running-statistics update per segment in order (nn.BatchNorm2d train mode,
models.py:199,203,209,220); backward: dbeta += sum g, dgamma += sum g*xhat,
coef = gamma*istd, sum g / n, sum g*xhat / n.  Channel counts off the 64-channel
block and segment counts past the kernel's four-segment chunk are included."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [(1, 64), (3, 72), (3, 2048), (5, 136), (9, 256)]


def _quarter_sums(slots, C):
    """slots [NSLOT][2][C] f32 -> (s1, s2) f64 with the kernel's association."""
    import _hip
    kq = _hip.NSLOT // 4
    s = slots.astype(np.float64).reshape(4, kq, 2, C)
    q = np.zeros((4, 2, C))
    for k in range(kq):  # each quarter: a sequential sum over its 8 slots
        q += s[:, k]
    tot = np.zeros((2, C))
    for u in range(4):
        tot += q[u]
    return tot[0], tot[1]


@pytest.mark.parametrize("nseg,C", CASES)
def test_bn_finalize_seg(dev, nseg, C):
    import _hip
    rng = np.random.default_rng(nseg * 1000 + C)
    count = 4096.0
    mean_true = rng.normal(0, 2, (nseg, C))
    var_true = rng.uniform(0.1, 3, (nseg, C))
    # slot sums that reproduce those moments, split unevenly over the slots
    w = rng.dirichlet(np.ones(_hip.NSLOT), size=(nseg, C)).transpose(0, 2, 1)  # [nseg][NSLOT][C]
    s1 = (mean_true * count)[:, None, :] * w
    s2 = ((var_true + mean_true ** 2) * count)[:, None, :] * w
    stats = np.stack([s1, s2], axis=2).astype(np.float32)  # [nseg][NSLOT][2][C]
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    beta = rng.normal(0, 0.5, C).astype(np.float32)
    rmean = rng.normal(0, 1, C).astype(np.float32)
    rvar = rng.uniform(0.5, 2, C).astype(np.float32)
    mom, eps = float(np.float32(0.1)), float(np.float32(1e-5))  # the kernel takes f32 momentum / eps

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_stats, d_g, d_b, d_rm, d_rv = t(stats), t(gamma), t(beta), t(rmean), t(rvar)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty(nseg, 4, C, device=dev)
    _hip.call("artsbir_bn_finalize_seg", d_stats.data_ptr(), nseg, 2 * _hip.NSLOT * C, C, count, d_g.data_ptr(),
              d_b.data_ptr(), d_rm.data_ptr(), d_rv.data_ptr(), nbt.data_ptr(), mom, eps, 1, out.data_ptr(),
              _hip.stream())
    torch.cuda.synchronize()

    rm, rv = rmean.astype(np.float64).copy(), rvar.astype(np.float64).copy()
    exp = np.zeros((nseg, 4, C))
    for s in range(nseg):
        a, b = _quarter_sums(stats[s], C)
        mean = a / count
        var = np.maximum(b / count - mean * mean, 0.0)
        rm = ((1 - mom) * rm.astype(np.float32).astype(np.float64) + mom * mean).astype(np.float32)
        rv = ((1 - mom) * rv.astype(np.float32).astype(np.float64) + mom * var * count / (count - 1)).astype(np.float32)
        istd = (1.0 / np.sqrt(var + eps)).astype(np.float32)
        exp[s] = [mean.astype(np.float32), istd, gamma * istd, beta]
    o = out.cpu().numpy()
    np.testing.assert_allclose(o, exp, rtol=2e-7, atol=0)
    np.testing.assert_allclose(d_rm.cpu().numpy(), rm, rtol=2e-7, atol=1e-30)
    np.testing.assert_allclose(d_rv.cpu().numpy(), rv, rtol=2e-7, atol=1e-30)
    assert int(nbt.item()) == nseg


@pytest.mark.parametrize("nseg,C", CASES)
def test_bn_bwd_finalize_seg(dev, nseg, C):
    import _hip
    rng = np.random.default_rng(nseg * 7 + C)
    count = 1024.0
    slots = rng.normal(0, 3, (nseg, _hip.NSLOT, 2, C)).astype(np.float32)
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    istd = rng.uniform(0.2, 4, (nseg, C)).astype(np.float32)
    dgamma0 = rng.normal(0, 1, C).astype(np.float32)
    dbeta0 = rng.normal(0, 1, C).astype(np.float32)

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_sl, d_g, d_is, d_dg, d_db = t(slots), t(gamma), t(istd), t(dgamma0), t(dbeta0)
    coef = torch.empty(nseg, 3, C, device=dev)
    _hip.call("artsbir_bn_bwd_finalize_seg", d_sl.data_ptr(), nseg, 2 * _hip.NSLOT * C, C, count, d_g.data_ptr(),
              d_is.data_ptr(), C, d_dg.data_ptr(), d_db.data_ptr(), coef.data_ptr(), _hip.stream())
    torch.cuda.synchronize()

    dg, db = dgamma0.copy(), dbeta0.copy()
    exp = np.zeros((nseg, 3, C), np.float32)
    for s in range(nseg):
        a, b = _quarter_sums(slots[s], C)
        db = (db + a.astype(np.float32)).astype(np.float32)
        dg = (dg + b.astype(np.float32)).astype(np.float32)
        exp[s] = [gamma * istd[s], (a / count).astype(np.float32), (b / count).astype(np.float32)]
    np.testing.assert_array_equal(coef.cpu().numpy(), exp)
    np.testing.assert_array_equal(d_db.cpu().numpy(), db)
    np.testing.assert_array_equal(d_dg.cpu().numpy(), dg)
