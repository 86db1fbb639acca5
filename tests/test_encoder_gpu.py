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
    """three separate train-mode forwards + TripletMarginLoss + backward + Adam
    (train.py:27-37,59-70) in the deterministic f32 mode.  Gradients against the
    float64 oracle evaluated on the HIP forward's ReLU decisions (tests/_parity.py):
    every parameter within max(4e-4, 4x the float32 oracle's error) — no outliers;
    the decisions themselves differ from float64 only at f32 rounding distance."""
    import engine
    import losses
    import optim
    from _parity import conditioned_grads, hip_relu_masks, max_rel_errors
    ref, mine = _pair(cfg, dev)
    # batch 4 for the tiny net; the deeper net at batch 4 sits on ReLU/hinge
    # decision boundaries, so it uses batch 16
    batch = 4 if cfg is TINY else 16
    elements = oenc.synthetic_triplet(batch, cfg["res"], seed=3)
    opt_ref = osteps.make_optimizer(ref, lr=1e-3, weight_decay=0.002)
    loss_ref, emb_ref = osteps.train_step(ref, opt_ref, osteps.make_loss(0.2), list(elements))

    old = engine.set_deterministic(True)
    try:
        masks = hip_relu_masks(mine, elements, dev, batched=False)
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
    finally:
        engine.set_deterministic(old)
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * max(1.0, abs(loss_ref.item()))

    def build():
        return osteps.build(cfg["layers"], cfg["output_dim"], cfg["heads"], cfg["res"], cfg["width"])
    _, g64, feed = conditioned_grads(build, elements, torch.float64, masks)
    _, g32, _ = conditioned_grads(build, elements, torch.float32, masks)
    assert feed.flip_mag < 1e-5 and feed.flips <= max(2, 1e-5 * feed.total), (feed.flips, feed.flip_mag)
    errs = max_rel_errors(grads, g64, g32)
    bad = [(k, e, r) for k, (e, r) in errs.items() if e > max(4e-4, 4 * r)]
    assert not bad, bad
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


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
def test_fused_eval_matches_unfused(dtype, tol, dev):
    """inference with every BatchNorm folded into its conv and applied with the
    ReLU / residual add in the conv epilogue (engine._forward_eval) = the
    training-path kernels with eval BatchNorm (separate BN / activation passes),
    on non-trivial running statistics; the f32 path also against the oracle"""
    import engine
    cfg = SMALL
    ref, mine = _pair(cfg, dev, dtype=dtype)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():  # non-trivial BN affine and running statistics
        for mod_r, mod_m in zip(ref.modules(), mine.modules()):
            if isinstance(mod_m, torch.nn.BatchNorm2d):
                C = mod_m.num_features
                vals = [1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g),
                        0.2 * torch.randn(C, generator=g), 0.5 + torch.rand(C, generator=g)]
                for mod in (mod_r, mod_m):
                    for t, v in zip((mod.weight, mod.bias, mod.running_mean, mod.running_var), vals):
                        t.copy_(v.to(t.device))
    ref.eval(); mine.eval()
    s, _, _ = oenc.synthetic_triplet(6, cfg["res"])
    old = engine.FUSED_EVAL
    try:
        with torch.no_grad():
            engine.FUSED_EVAL = True
            e_fused = mine(s.to(dev)).float().cpu()
            engine.FUSED_EVAL = False
            e_plain = mine(s.to(dev)).float().cpu()
    finally:
        engine.FUSED_EVAL = old
    rel = ((e_fused - e_plain).norm() / e_plain.norm()).item()
    assert rel < tol, rel
    if dtype == torch.float32:
        with torch.no_grad():
            e_ref = ref(s)
        assert torch.allclose(e_fused, e_ref, atol=1e-3, rtol=1e-3), _rel(e_fused, e_ref)


def test_fused_eval_refolds_after_train_forward_without_step(dev):
    """the folded eval weights cache the BN running statistics; a train-mode
    forward with no optimizer step (BN recalibration under no_grad) updates those
    statistics through raw pointers, so the next eval must refold: it must equal
    the unfused eval path and the oracle run through the same sequence"""
    import engine
    cfg = TINY
    ref, mine = _pair(cfg, dev)
    s, p, _ = oenc.synthetic_triplet(4, cfg["res"])
    ref.eval(); mine.eval()
    with torch.no_grad():
        mine(s.to(dev))  # builds the folded cache
        ref.train(); mine.train()
        ref(p); mine(p.to(dev))  # running statistics move, no parameter changes
        ref.eval(); mine.eval()
        e_ref = ref(s)
        e = mine(s.to(dev)).float().cpu()
        old = engine.FUSED_EVAL
        try:
            engine.FUSED_EVAL = False
            e_plain = mine(s.to(dev)).float().cpu()
        finally:
            engine.FUSED_EVAL = old
    assert torch.allclose(e, e_plain, atol=1e-4, rtol=1e-4), _rel(e, e_plain)
    assert torch.allclose(e, e_ref, atol=1e-3, rtol=1e-3), _rel(e, e_ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_batched_repack_matches_fresh_packs(dtype, dev):
    """the one-launch re-pack after a weight update (artsbir_pack_weights) writes
    exactly what a first-time per-tensor pack of the same weights writes"""
    import engine
    _, mine = _pair(SMALL, dev, dtype)
    eng = engine.Engine(mine)
    eng.dtype = dtype
    eng.packed()  # first pack: records the plan
    assert eng._plan is not None and eng._plan[2] > 50
    with torch.no_grad():
        for i, p in enumerate(mine.parameters()):
            p.add_(0.01 * (i % 7 + 1) * torch.randn_like(p))
    got = eng.packed()  # batched path
    assert eng._plan is not None
    fresh = engine.Engine(mine)
    fresh.dtype = dtype
    want = fresh.packed()
    torch.cuda.synchronize()

    def leaves(x):
        if isinstance(x, dict):
            for k in sorted(x):
                yield from leaves(x[k])
        elif isinstance(x, (list, tuple)):
            for v in x:
                yield from leaves(v)
        elif x is not None:
            yield x
    a, b = list(leaves(got)), list(leaves(want))
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
