"""The CPU oracle against the committed golden fixtures and against its
independent float64 numpy restatement (the cross-pinning that stands in for
reference golden vectors, which do not exist — SURVEY §4/§8c)."""
import json
import os
import sys

import numpy as np
import torch

from oracle import encoder as oenc
from oracle import numpy_ref
from oracle import retrieval as oret
from oracle import steps as osteps

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLDEN)
import make_golden  # noqa: E402


def _npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_encoder_golden():
    gold = _npz("encoder_tiny.npz")
    torch.manual_seed(0)
    T = make_golden.TINY
    m = osteps.build(T["layers"], T["output_dim"], T["heads"], T["res"], T["width"], seed=1234)
    el = list(oenc.synthetic_triplet(4, T["res"], seed=3))
    opt = osteps.make_optimizer(m, lr=1e-3, weight_decay=0.002)
    m.train()
    loss, embs = osteps.get_loss(osteps.make_loss(0.2), m, el)
    opt.zero_grad()
    loss.backward()
    assert abs(loss.item() - gold["loss"][0]) < 1e-5
    for name, e in zip(("emb_s", "emb_p", "emb_n"), embs):
        np.testing.assert_allclose(e.detach().numpy(), gold[name], rtol=1e-4, atol=1e-5)
    for k, p in m.named_parameters():
        s, _ = make_golden.summary(p.grad, "grad/" + k)
        np.testing.assert_allclose(s, gold["grad/" + k], rtol=1e-3, atol=1e-6)
    opt.step()
    for k, v in m.state_dict().items():
        if v.dtype.is_floating_point:
            s, _ = make_golden.summary(v, "state/" + k)
            np.testing.assert_allclose(s, gold["state/" + k], rtol=1e-4, atol=1e-6)
        else:
            np.testing.assert_array_equal(v.numpy().reshape(-1), gold["state/" + k])


def test_retrieval_golden():
    gold = _npz("retrieval.npz")
    g, qs, pos = make_golden.golden_gallery()
    np.testing.assert_allclose(gold["gallery_checksum"], [g.sum(), qs.sum()], rtol=1e-6)
    np.testing.assert_array_equal(gold["positives"], pos)
    for i, q in enumerate(qs):
        d = oret.l2_distances(q, g)
        ti, td = oret.topk(d, 10)
        np.testing.assert_array_equal(ti, gold["topk_idx"][i])
        np.testing.assert_allclose(td, gold["topk_dist"][i], rtol=1e-12)
        r = oret.rank_of(d, pos[i]) if pos[i] >= 0 else len(g)
        assert r == gold["ranks"][i]
    # duplicates are ordered by the lower index
    d = oret.l2_distances(qs[0], g)
    assert d[0] == d[4000] and oret.rank_of(d, 0) < oret.rank_of(d, 4000)
    with open(os.path.join(GOLDEN, "retrieval_metrics.json")) as f:
        gm = json.load(f)
    m = oret.metrics([int(r) for r, p in zip(gold["ranks"], pos) if p >= 0], 10)
    for k, v in gm.items():
        np.testing.assert_allclose(m[k], v, rtol=1e-12)


def test_loss_and_adam_golden_and_numpy_pin():
    gold = _npz("loss_adam.npz")
    a, p, n = (torch.from_numpy(gold[k]).requires_grad_(True) for k in ("a", "p", "n"))
    loss = osteps.make_loss(0.2)(a, p, n)
    loss.backward()
    assert abs(loss.item() - gold["loss"][0]) < 1e-6
    np.testing.assert_allclose(a.grad.numpy(), gold["da"], atol=1e-7)
    # independent float64 numpy restatements
    ln = numpy_ref.triplet_margin_loss(gold["a"].astype(np.float64), gold["p"].astype(np.float64),
                                       gold["n"].astype(np.float64))
    assert abs(ln - gold["loss"][0]) < 1e-5
    w, mm, vv = gold["w0"].astype(np.float64), np.zeros(257), np.zeros(257)
    for s in range(3):
        w, mm, vv = numpy_ref.adam_step(w, gold["grads"][s].astype(np.float64), mm, vv, s + 1, lr=1e-3, wd=0.002)
    np.testing.assert_allclose(w, gold["w3"], atol=2e-6)
    np.testing.assert_allclose(mm, gold["m3"], atol=1e-6)
    np.testing.assert_allclose(vv, gold["v3"], rtol=1e-4, atol=1e-8)


def test_numpy_cross_pins_torch_oracle():
    """two independent restatements of models.py agree (train-mode BN, attention pool)."""
    T = make_golden.TINY
    m = osteps.build((2, 1, 1, 1), 32, 8, 64, 16, seed=7)
    x, _, _ = oenc.synthetic_triplet(3, 64, seed=5)
    m.train()
    with torch.no_grad():
        e = m(x).numpy()
    sd = {k: v.detach().double().numpy() for k, v in m.state_dict().items()}
    e2, stats = numpy_ref.encoder_forward(x.double().numpy(), sd, (2, 1, 1, 1), 8)
    np.testing.assert_allclose(e, e2, rtol=1e-4, atol=1e-5)
    # running-stat update of one train forward: momentum 0.1, unbiased variance
    for bn, (mean, uvar) in stats.items():
        np.testing.assert_allclose(m.state_dict()[bn + ".running_mean"].numpy(), 0.1 * mean, atol=1e-5)
        np.testing.assert_allclose(m.state_dict()[bn + ".running_var"].numpy(), 0.9 + 0.1 * uvar, rtol=1e-4)
    # eval mode
    m.eval()
    with torch.no_grad():
        e = m(x).numpy()
    sd = {k: v.detach().double().numpy() for k, v in m.state_dict().items()}
    e3, _ = numpy_ref.encoder_forward(x.double().numpy(), sd, (2, 1, 1, 1), 8, train=False)
    np.testing.assert_allclose(e, e3, rtol=1e-4, atol=1e-5)
