"""Encoder forward / triplet step on libartsbir_hip vs the CPU oracle (f32 parity mode)."""
import copy

import numpy as np
import pytest
import torch

from oracle import encoder as oenc
from oracle import steps as osteps

pytestmark = pytest.mark.gpu

TINY = dict(layers=(1, 1, 1, 1), output_dim=32, heads=8, res=64, width=16)
SMALL = dict(layers=(2, 2, 2, 2), output_dim=128, heads=8, res=64, width=16)


def _pair(cfg, dev, dtype=torch.float32, seed=1234):
    import models
    ref = osteps.build(cfg["layers"], cfg["output_dim"], cfg["heads"], cfg["res"], cfg["width"], seed=seed)
    mine = models.ModifiedResNet(cfg["layers"], cfg["output_dim"], heads=cfg["heads"],
                                 input_resolution=cfg["res"], width=cfg["width"])
    mine.load_state_dict(ref.state_dict(), strict=True)
    mine.compute_dtype = dtype
    return ref, mine.to(dev)


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("cfg", [TINY, SMALL], ids=["tiny", "small"])
def test_forward_train_and_eval_f32(cfg, dev):
    ref, mine = _pair(cfg, dev)
    s, p, n = oenc.synthetic_triplet(4, cfg["res"])
    ref.train(); mine.train()
    with torch.no_grad():
        for x in (s, p, n):
            e_ref = ref(x)
            e = mine(x.to(dev)).cpu()
            assert torch.allclose(e, e_ref, atol=1e-3, rtol=1e-3), _rel(e, e_ref)
    # running statistics after three train-mode forwards
    sd_ref, sd = ref.state_dict(), mine.state_dict()
    for k in sd_ref:
        if "running" in k or "num_batches" in k:
            assert torch.allclose(sd[k].cpu().double(), sd_ref[k].double(), atol=1e-4, rtol=1e-4), k
    ref.eval(); mine.eval()
    with torch.no_grad():
        e_ref = ref(s)
        e = mine(s.to(dev)).cpu()
    assert torch.allclose(e, e_ref, atol=1e-3, rtol=1e-3), _rel(e, e_ref)


@pytest.mark.parametrize("cfg", [TINY, SMALL], ids=["tiny", "small"])
def test_triplet_step_f32(cfg, dev):
    import losses
    import optim
    ref, mine = _pair(cfg, dev)
    # batch 4 for the tiny net; the deeper net at batch 4 sits on ReLU/hinge
    # decision boundaries where f32 rounding flips masks, so it uses batch 16
    batch = 4 if cfg is TINY else 16
    elements = oenc.synthetic_triplet(batch, cfg["res"], seed=3)
    opt_ref = osteps.make_optimizer(ref, lr=1e-3, weight_decay=0.002)
    loss_ref, emb_ref = osteps.train_step(ref, opt_ref, osteps.make_loss(0.2), list(elements))

    opt = optim.Adam(mine.parameters(), lr=1e-3, weight_decay=0.002)
    mine.train()
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    outs = [mine(e.to(dev)) for e in elements]
    loss = loss_fn(*outs)
    opt.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    before = {k: p.detach().cpu().clone() for k, p in mine.named_parameters()}
    opt.step()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * max(1.0, abs(loss_ref.item()))
    # gradients: the triplet loss at batch 4 is ill-conditioned (the oracle's own
    # f32 gradients differ from its f64 gradients by up to a few 1e-2 relative), so
    # the bar is "as accurate as the reference's f32 path": error vs the f64 oracle
    # within max(4e-3, 4 x the f32 oracle's own error).
    def ref_grads(dtype):
        r = osteps.build(cfg["layers"], cfg["output_dim"], cfg["heads"], cfg["res"], cfg["width"]).to(dtype)
        r.train()
        l, _ = osteps.get_loss(osteps.make_loss(0.2), r, [e.to(dtype) for e in elements])
        l.backward()
        return {k: q.grad.double() for k, q in r.named_parameters()}
    g64, g32 = ref_grads(torch.float64), ref_grads(torch.float32)
    # BN statistics are summed with f32 atomics (run-to-run order varies), so a
    # pre-activation within ~1e-7 of zero can land on either side of a ReLU; one
    # such flip moves one element's contribution and shows up as a ~1e-2 error in
    # a few small parameters (seen on MI355X: 2 of 4 runs of this exact case).
    # Allowed: at most 6 such outliers, each within 2e-2, and the whole gradient
    # vector within 1e-3 relative L2 of the f64 oracle.
    floor = 1e-4 * max(g.abs().max().item() for g in g64.values())
    outliers = []
    for k, g_ref in g64.items():
        scale = max(g_ref.abs().max().item(), floor)
        e_ref = (g32[k] - g_ref).abs().max().item() / scale
        e_mine = (grads[k].double() - g_ref).abs().max().item() / scale
        if e_mine > max(4e-3, 4 * e_ref):
            outliers.append((k, e_mine, e_ref))
            assert e_mine <= 2e-2, (k, e_mine, e_ref)
    assert len(outliers) <= 6, outliers
    # the rest of the gradient vector (the flip outliers are bounded above)
    flipped = {k for k, _, _ in outliers}
    flat_ref = torch.cat([g.flatten() for k, g in g64.items() if k not in flipped])
    flat = torch.cat([grads[k].double().flatten() for k in g64 if k not in flipped])
    assert ((flat - flat_ref).norm() / flat_ref.norm()).item() < 1e-3
    # parameters after one Adam step: the HIP Adam vs the float64 restatement of
    # torch.optim.Adam applied to the same gradients (first-step Adam is ~lr*sign(g),
    # so comparing against the reference parameters would test sign noise of ~0 grads)
    from oracle import numpy_ref
    for k, p in mine.named_parameters():
        z = np.zeros(p.shape)
        want, _, _ = numpy_ref.adam_step(before[k].double().numpy(), grads[k].double().numpy(), z, z, 1,
                                         lr=1e-3, wd=0.002)
        assert np.allclose(p.detach().cpu().double().numpy(), want, atol=1e-6, rtol=1e-5), k
    # and the BN running statistics of the three train-mode forwards
    sd_ref = ref.state_dict()
    for k, v in mine.state_dict().items():
        if "running" in k or "num_batches" in k:
            assert torch.allclose(v.cpu().double(), sd_ref[k].double(), atol=1e-4, rtol=1e-4), k


def test_forward_bf16_close(dev):
    ref, mine = _pair(SMALL, dev, dtype=torch.bfloat16)
    s, _, _ = oenc.synthetic_triplet(8, SMALL["res"])
    ref.train(); mine.train()
    with torch.no_grad():
        e_ref = ref(s)
        e = mine(s.to(dev)).cpu()
    cos = torch.nn.functional.cosine_similarity(e, e_ref, dim=1)
    assert cos.min() > 0.98, cos  # bf16 activations through 8 blocks of batch-8 BN


def test_triplet_step_against_golden_fixture(dev):
    """embeddings, loss and post-Adam parameter summaries vs tests/golden/encoder_tiny.npz"""
    import os
    import sys
    import losses
    import optim
    golden = os.path.join(os.path.dirname(__file__), "golden")
    sys.path.insert(0, golden)
    import make_golden
    gold = np.load(os.path.join(golden, "encoder_tiny.npz"), allow_pickle=False)
    ref, mine = _pair(TINY, dev)
    elements = oenc.synthetic_triplet(4, TINY["res"], seed=3)
    mine.train()
    opt = optim.Adam(mine.parameters(), lr=1e-3, weight_decay=0.002)
    outs = [mine(e.to(dev)) for e in elements]
    loss = losses.TripletMarginLoss(margin=0.2)(*outs)
    opt.zero_grad()
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert abs(loss.item() - gold["loss"][0]) < 1e-4
    for name, e in zip(("emb_s", "emb_p", "emb_n"), outs):
        np.testing.assert_allclose(e.detach().cpu().numpy(), gold[name], rtol=1e-3, atol=1e-3)
    for k, v in mine.state_dict().items():
        if "running" in k or "num_batches" in k:
            if v.dtype.is_floating_point:
                s, _ = make_golden.summary(v.cpu(), "state/" + k)
                np.testing.assert_allclose(s, gold["state/" + k], rtol=1e-3, atol=1e-4)
            else:
                np.testing.assert_array_equal(v.cpu().numpy().reshape(-1), gold["state/" + k])
    mine.eval()
    with torch.no_grad():
        e = mine(elements[0].to(dev)).cpu().numpy()
    np.testing.assert_allclose(e, gold["emb_eval"], rtol=1e-3, atol=1e-3)
