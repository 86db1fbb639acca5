"""Batched branches (BN segments) and the BN-backward reduction fused into the
data-gradient GEMM: kernel-level checks against torch fp32 (CPU), and the
encoder-level check that forward_branches / fused backward give the same
embeddings, running statistics and gradients as three separate calls with the
unfused backward."""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

import _hip
import _kernels

pytestmark = pytest.mark.gpu

CFGS = ["auto", "0", "1", "2", "3", "4", "5", "10", "11", "12", "13", "14", "15", "16", "18", "19", "20", "21", "22", "26",
        "-2"]


@pytest.fixture
def cfg_env():
    old = os.environ.get("ARTSBIR_PGEMM_CFG")
    yield
    if old is None:
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    else:
        os.environ["ARTSBIR_PGEMM_CFG"] = old


def _set(cfg):
    if cfg == "auto":
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    else:
        os.environ["ARTSBIR_PGEMM_CFG"] = cfg


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


SEG_CASES = [
    # N (= nseg x images), nseg, H, W, C, Cout, R, pad
    (6, 3, 16, 16, 64, 128, 3, 1),     # 256 px / segment
    (12, 3, 8, 8, 256, 64, 1, 0),      # 256 px / segment
    (6, 3, 32, 16, 32, 64, 3, 1),      # multi-tap C=32, 1024 px / segment
    (6, 3, 16, 16, 32, 32, 3, 1),      # stem conv2 shape family
    (6, 2, 7, 7, 512, 256, 3, 1),      # 147 px / segment: not a multiple of 64 -> per-segment fallback
]


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("case", SEG_CASES)
def test_conv_fwd_segment_stats(case, cfg, dev, cfg_env):
    _set(cfg)
    N, G, H, W, C, Co, R, pd = case
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g)
    x[N // G:] += 0.5  # segments with different statistics
    x = x.bfloat16().float()
    w = (torch.randn(Co, C, R, R, generator=g) / (C * R * R) ** 0.5).bfloat16().float()
    ref = F.conv2d(x, w, padding=pd)
    y = torch.empty(N * H * W, Co, device=dev, dtype=torch.bfloat16)
    stats = torch.zeros(G, _hip.NSLOT, 2, Co, device=dev)
    d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, 1, pd)
    xd = _nhwc(x).to(dev, torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    _hip.call("artsbir_conv2d_fwd_seg", d, xd.data_ptr(), wd.data_ptr(), y.data_ptr(), G, stats.data_ptr(),
              _hip.stream())
    torch.cuda.synchronize()
    _kernels.require(cfg)
    out = y.float().cpu().view(N, H, W, Co).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=3e-2, rtol=1e-2), (out - ref).abs().max()
    s = stats.sum(1).cpu()
    for k in range(G):
        r2 = ref[k * N // G:(k + 1) * N // G].permute(0, 2, 3, 1).reshape(-1, Co)
        assert torch.allclose(s[k, 0], r2.sum(0), atol=5e-2, rtol=1e-3), k
        assert torch.allclose(s[k, 1], (r2 * r2).sum(0), atol=5e-2, rtol=1e-3), k


BNB_CASES = [
    # N, nseg, H, W, Cin (= BN channels), Cout (of the forward conv), R, pad, kind, ntarget, res_mode
    (4, 1, 8, 8, 64, 64, 3, 1, 1, 1, 0),       # ACT, 3x3
    (6, 3, 16, 16, 128, 64, 1, 0, 1, 1, 0),    # ACT, segments
    (4, 2, 16, 16, 256, 64, 1, 0, 0, 2, 1),    # RES (bn3 + downsample), residual add
    (6, 3, 16, 16, 256, 64, 1, 0, 0, 1, 2),    # RES, avg-unpool residual
    (4, 2, 16, 16, 32, 64, 3, 1, 1, 1, 0),     # stem-like: 64-ch dY -> 32-ch dX
    (6, 3, 16, 16, 32, 32, 3, 1, 1, 1, 0),     # stem conv2 data gradient, segments
    (3, 1, 9, 13, 64, 64, 3, 1, 1, 1, 0),      # layer-1 3x3, image-crossing tiles
    (4, 2, 16, 16, 512, 128, 1, 0, 0, 2, 1),   # RES, K 128 (layer-2 conv1 family), two targets
    (6, 3, 8, 8, 256, 128, 1, 0, 0, 1, 2),     # RES, K 128, avg-unpool residual
]


def _bnb_reference(d, kind, ys, means, istds, msc, msh, mask):
    """g = d*mask, sum g, sum g*xhat_t (f64) for one segment; tensors [n, C];
    kind 1 masks with the ReLU's BN applied as (y - mean) * scale + beta"""
    if kind == 1:
        keep = ((ys[0] - means[0]) * msc + msh) > 0
    else:
        keep = mask > 0
    g = torch.where(keep, d, torch.zeros_like(d))
    sums = []
    for y, m, s in zip(ys, means, istds):
        xhat = (y - m) * s
        sums.append((g.sum(0), (g * xhat).sum(0)))
    return g, sums


def _pack_bits(mask_nhwc):
    """[..., C] -> uint8 [..., C/8]: bit e of byte c = mask[..., 8c+e] > 0"""
    m = (mask_nhwc > 0).to(torch.uint8).reshape(*mask_nhwc.shape[:-1], -1, 8)
    return (m << torch.arange(8, dtype=torch.uint8, device=m.device)).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("bits", [False, True])
@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("case", BNB_CASES)
def test_dgrad_fused_bn_reduce(case, cfg, bits, dev, cfg_env):
    _set(cfg)
    N, G, H, W, Ci, Co, R, pd, kind, nt, rm = case
    if bits and kind != 0:
        pytest.skip("mask bits replace the block-output mask (kind 0) only")
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(N, Co, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Co, Ci, R, R, generator=g) / (Co * R * R) ** 0.5).bfloat16().float()
    draw = torch.nn.grad.conv2d_input((N, Ci, H, W), w, dy, stride=1, padding=pd)
    res = None
    if rm == 1:
        res = torch.randn(N, Ci, H, W, generator=g).bfloat16().float()
        draw = draw + res
    elif rm == 2:
        res = torch.randn(N, Ci, H // 2, W // 2, generator=g).bfloat16().float()
        draw = draw + 0.25 * F.interpolate(res, scale_factor=2, mode="nearest")
    ys = [torch.randn(N, Ci, H, W, generator=g).bfloat16().float() for _ in range(nt)]
    mask = torch.randn(N, Ci, H, W, generator=g).bfloat16().float()
    params = torch.randn(G, 4, Ci, generator=g)  # BN parameter block per segment: mean, istd, scale, beta
    params[:, 1] = params[:, 1].abs() + 0.5
    params2 = torch.randn(G, 4, Ci, generator=g)
    params2[:, 1] = params2[:, 1].abs() + 0.5
    # device buffers
    wdflip = w.flip(2, 3).permute(1, 2, 3, 0).contiguous().to(dev, torch.bfloat16)
    dyd = _nhwc(dy).to(dev, torch.bfloat16)
    resd = _nhwc(res).to(dev, torch.bfloat16) if res is not None else None
    yds = [_nhwc(y).to(dev, torch.bfloat16) for y in ys]
    maskd = _nhwc(mask).to(dev, torch.bfloat16)
    pd_ = [params.to(dev), params2.to(dev)]
    slots = [torch.zeros(G, _hip.NSLOT, 2, Ci, device=dev) for _ in range(nt)]
    dx = torch.full((N * H * W, Ci), float("nan"), device=dev, dtype=torch.bfloat16)
    desc = _hip.BnBwdDesc()
    desc.dtype = _hip.DT_BF16
    desc.kind = 3 if bits else kind
    desc.pool = 0
    maskb = _pack_bits(maskd) if bits else None
    desc.mask = (maskb.data_ptr() if bits else maskd.data_ptr()) if kind == 0 else None
    desc.mask_bn = pd_[0][0].data_ptr() if kind == 1 else None
    desc.ntarget = nt
    for t in range(nt):
        desc.y[t] = yds[t].data_ptr()
        desc.mean[t] = pd_[t][0, 0].data_ptr()
        desc.istd[t] = pd_[t][0, 1].data_ptr()
        desc.slots[t] = slots[t].data_ptr()
    d = _hip.conv_desc(torch.bfloat16, N, H, W, Ci, Co, R, R, 1, pd)
    _hip.call("artsbir_conv2d_dgrad_bnb", d, dyd.data_ptr(), wdflip.data_ptr(), dx.data_ptr(),
              resd.data_ptr() if resd is not None else None, rm, desc, G, 4 * Ci, _hip.stream())
    torch.cuda.synchronize()
    _kernels.require(cfg)
    got = dx.float().cpu()
    flat = lambda t: t.permute(0, 2, 3, 1).reshape(-1, Ci)  # noqa: E731
    per = N // G * H * W
    for s in range(G):
        sl = slice(s * per, (s + 1) * per)
        dseg = flat(draw)[sl]
        yseg = [flat(y)[sl] for y in ys]
        gref, sums = _bnb_reference(dseg, kind, yseg, [params[s, 0], params2[s, 0]], [params[s, 1], params2[s, 1]],
                                    params[s, 2], params[s, 3], flat(mask)[sl])
        # masks decided on identical bf16 inputs; g within bf16 rounding of the f32 GEMM
        assert torch.allclose(got[sl], gref, atol=3e-2, rtol=1e-2), (s, (got[sl] - gref).abs().max())
        for t in range(nt):
            st = slots[t][s].sum(0).cpu()
            scale = gref.abs().sum(0) + 1.0
            assert ((st[0] - sums[t][0]).abs() / scale).max() < 2e-2, (s, t)
            assert ((st[1] - sums[t][1]).abs() / (scale * 4)).max() < 2e-2, (s, t)


def _models(dev, dtype):
    import models
    torch.manual_seed(11)
    a = models.ModifiedResNet((1, 2, 1, 1), 32, heads=8, input_resolution=64, width=16)
    b = copy.deepcopy(a)
    a.compute_dtype = b.compute_dtype = dtype
    return a.to(dev), b.to(dev)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_forward_branches_matches_separate_calls(dtype, dev):
    import engine
    import losses
    batched, separate = _models(dev, dtype)
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randn(8, 3, 64, 64, device=dev, generator=g) + i for i in range(3)]
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    old = engine.FUSE_BNB
    try:
        engine.FUSE_BNB = True
        batched.train()
        ob = batched.forward_branches(xs)
        lb = loss_fn(*ob)
        lb.backward()
        engine.FUSE_BNB = False
        separate.train()
        os_ = [separate(x) for x in xs]
        ls = loss_fn(*os_)
        ls.backward()
    finally:
        engine.FUSE_BNB = old
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    for a, b in zip(ob, os_):
        assert torch.allclose(a, b, atol=tol, rtol=tol), (a - b).abs().max()
    sa, sb = batched.state_dict(), separate.state_dict()
    for k in sa:
        if "running" in k or "num_batches" in k:
            assert torch.allclose(sa[k].double(), sb[k].double(), atol=tol, rtol=tol), k
    if dtype != torch.float32:
        # bf16 gradients of the default mode differ run to run by ~15 % on this tiny
        # net (atomic order -> ReLU flips); the deterministic mode makes the batched
        # and the separate calls take the same ReLU decisions, so their gradients
        # must agree up to the weight gradients' split-K summation order
        _bf16_det_gradients_agree(dev, xs, loss_fn)
        return
    # per parameter, relative to max(|g|, 1e-4 * the largest gradient anywhere):
    # mathematically-zero gradients (k_proj.bias, c_proj.bias of a triplet loss)
    # are rounding noise of ~1e-8 and must not dominate a global norm
    grads_b = {k: p.grad for k, p in batched.named_parameters()}
    grads_s = {k: p.grad for k, p in separate.named_parameters()}
    # BN sums use f32 atomics, so a pre-activation within ~1e-7 of zero can land
    # on either side of a ReLU between two runs.  On this net two identical
    # separate-call runs already differ by up to ~6e-3 (per-parameter relative
    # L2) in a few dozen BN parameters (measured on MI355X), so the bar here is
    # that noise level; the fused kernels themselves are checked exactly above.
    floor = 1e-4 * max(g.norm().item() for g in grads_s.values())
    for k, gs in grads_s.items():
        err = (grads_b[k] - gs).norm().item() / max(gs.norm().item(), floor)
        assert err < 2e-2, (k, err)


def _bf16_det_gradients_agree(dev, xs, loss_fn):
    import engine
    batched, separate = _models(dev, torch.bfloat16)
    old = engine.set_deterministic(True)
    try:
        batched.train()
        lb = loss_fn(*batched.forward_branches(xs))
        lb.backward()
        separate.train()
        ls = loss_fn(*[separate(x) for x in xs])
        ls.backward()
        torch.cuda.synchronize()
    finally:
        engine.set_deterministic(old)
    assert abs(lb.item() - ls.item()) <= 1e-6 * max(1.0, abs(ls.item())), (lb.item(), ls.item())
    gb = {k: p.grad for k, p in batched.named_parameters()}
    gs = {k: p.grad for k, p in separate.named_parameters()}
    floor = 1e-4 * max(g.norm().item() for g in gs.values())
    for k, g in gs.items():
        err = (gb[k] - g).norm().item() / max(g.norm().item(), floor)
        assert err < 1e-2, (k, err)


@pytest.mark.parametrize("C", [64, 256])
def test_block_out_mask_bits(C, dev):
    """artsbir_block_out_mask: the same output as artsbir_block_out plus its
    ReLU mask as bits (the fused backward's kind-3 mask)"""
    g = torch.Generator(device=dev).manual_seed(3)
    rows = 3 * 7 * 5
    y3 = torch.randn(rows, C, device=dev, generator=g).bfloat16()
    idn = torch.randn(rows, C, device=dev, generator=g).bfloat16()
    bn = torch.randn(4, C, device=dev, generator=g)  # mean, istd (unused), scale, beta
    out0 = torch.empty_like(y3)
    out1 = torch.empty_like(y3)
    bits = torch.full((rows, C // 8), 77, dtype=torch.uint8, device=dev)
    _hip.call("artsbir_block_out", _hip.DT_BF16, y3.data_ptr(), bn.data_ptr(), None, None,
              idn.data_ptr(), rows, C, 1, out0.data_ptr(), _hip.stream())
    _hip.call("artsbir_block_out_mask", _hip.DT_BF16, y3.data_ptr(), bn.data_ptr(), None, None,
              idn.data_ptr(), rows, C, 1, out1.data_ptr(), bits.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    assert torch.equal(out0, out1)
    ref = torch.relu((y3.float() - bn[0]) * bn[2] + bn[3] + idn.float()).bfloat16()
    assert torch.allclose(out1.float(), ref.float(), atol=3e-2, rtol=1e-2)
    assert torch.equal(bits, _pack_bits(out1))
