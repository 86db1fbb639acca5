"""The pipelined LDS-DMA conv kernel (pgemm.hip): bf16 forward with BN statistics
and bf16 data-gradient with residual epilogues, every tile shape forced in turn,
against torch fp32 (CPU) on the same bf16-rounded operands."""
import os

import pytest
import torch
import torch.nn.functional as F

import _hip
import _kernels

pytestmark = pytest.mark.gpu

CASES = [
    # N, H, W, C, Cout, R, S, stride, pad
    (2, 9, 7, 8, 32, 3, 3, 2, 1),       # stem-1 like: 8-channel multi-tap K-steps, stride 2
    (2, 8, 8, 32, 64, 3, 3, 1, 1),      # 32 channels: two taps per K-step
    (3, 7, 5, 64, 256, 1, 1, 1, 0),
    (2, 14, 14, 128, 128, 3, 3, 1, 1),
    (1, 5, 5, 256, 96, 1, 1, 1, 0),     # partial channel tile
    (8, 28, 28, 64, 128, 3, 3, 1, 1),   # many pixel tiles
    (3, 12, 12, 512, 64, 1, 1, 2, 0),   # strided 1x1
    (2, 12, 10, 32, 32, 3, 3, 1, 1),    # stem conv2 (direct small-channel kernel)
    (3, 9, 13, 64, 64, 3, 3, 1, 1),     # layer-1 3x3, image-crossing pixel tiles
    (2, 12, 10, 64, 32, 3, 3, 1, 1),
    (3, 11, 7, 8, 32, 3, 3, 2, 1),      # stem conv1, odd sizes
    (2, 32, 48, 64, 64, 3, 3, 1, 1),    # halo-tiled kernel, 16 x 16 tiles
    (2, 32, 16, 32, 64, 3, 3, 1, 1),    # halo-tiled, 16 x 16 tiles, 32 -> 64 channels
    (3, 17, 23, 64, 32, 3, 3, 1, 1),    # halo-tiled, 8 x 16 tiles with row and column tails
]
CFGS = ["auto", "0", "1", "2", "3", "4", "5", "10", "15", "16", "19", "20", "21", "22", "24", "25"]


@pytest.fixture
def cfg_env(request):
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


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("case", CASES)
def test_pgemm_fwd_stats(case, cfg, dev, cfg_env):
    _set(cfg)
    N, H, W, C, Co, R, S, st, pd = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Co, C, R, S, generator=g) / (C * R * S) ** 0.5).bfloat16().float()
    ref = F.conv2d(x, w, stride=st, padding=pd)
    Ho, Wo = ref.shape[2:]
    xd = _nhwc(x).to(dev, torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    y = torch.full((N * Ho * Wo, Co), float("nan"), device=dev, dtype=torch.bfloat16)
    stats = torch.zeros(_hip.NSLOT, 2, Co, device=dev)
    d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, S, st, pd)
    _hip.call("artsbir_conv2d_fwd", d, xd.data_ptr(), wd.data_ptr(), y.data_ptr(), Co, 0, 0, None, None, None, 0,
              stats.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    _kernels.require(cfg)
    out = y.float().cpu().view(N, Ho, Wo, Co).permute(0, 3, 1, 2)
    assert torch.isfinite(out).all()
    assert torch.allclose(out, ref, atol=2e-2, rtol=1e-2), (out - ref).abs().max()
    s = stats.sum(0).cpu()
    r2 = ref.permute(0, 2, 3, 1).reshape(-1, Co)
    assert torch.allclose(s[0], r2.sum(0), atol=1e-2, rtol=1e-3)
    assert torch.allclose(s[1], (r2 * r2).sum(0), atol=1e-2, rtol=1e-3)


DG_CASES = [
    # N, H, W, Cin, Cout, R, pad, res_mode
    (2, 8, 8, 64, 64, 3, 1, 0),
    (2, 8, 8, 64, 64, 3, 1, 1),
    (2, 8, 8, 256, 64, 1, 0, 2),
    (3, 14, 14, 128, 256, 1, 0, 1),
    (2, 10, 6, 32, 64, 3, 1, 0),        # dY with 64 channels -> 32-channel dX (stem)
    (2, 10, 6, 32, 32, 3, 1, 0),        # 32-channel dY: multi-tap
    (8, 28, 28, 128, 128, 3, 1, 2),
    (3, 9, 13, 64, 64, 3, 1, 0),        # layer-1 3x3 data gradient
    (2, 12, 10, 64, 32, 3, 1, 1),
    (2, 16, 32, 32, 64, 3, 1, 0),       # halo-tiled data gradient, 16 x 16 tiles
]


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("case", DG_CASES)
def test_pgemm_dgrad_residual(case, cfg, dev, cfg_env):
    _set(cfg)
    N, H, W, Ci, Co, R, pd, rm = case
    g = torch.Generator().manual_seed(2)
    dy = torch.randn(N, Co, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Co, Ci, R, R, generator=g) / (Co * R * R) ** 0.5).bfloat16().float()
    ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w, dy, stride=1, padding=pd)
    res = None
    if rm == 1:
        res = torch.randn(N, Ci, H, W, generator=g).bfloat16().float()
        ref = ref + res
    elif rm == 2:
        res = torch.randn(N, Ci, H // 2, W // 2, generator=g).bfloat16().float()
        ref = ref + 0.25 * F.interpolate(res, scale_factor=2, mode="nearest")
    wdflip = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Ci][R][S][Co]
    dyd = _nhwc(dy).to(dev, torch.bfloat16)
    wdd = wdflip.to(dev, torch.bfloat16)
    dx = torch.full((N * H * W, Ci), float("nan"), device=dev, dtype=torch.bfloat16)
    resd = _nhwc(res).to(dev, torch.bfloat16) if res is not None else None
    d = _hip.conv_desc(torch.bfloat16, N, H, W, Ci, Co, R, R, 1, pd)
    _hip.call("artsbir_conv2d_dgrad", d, dyd.data_ptr(), wdd.data_ptr(), dx.data_ptr(),
              resd.data_ptr() if resd is not None else None, rm, _hip.stream())
    torch.cuda.synchronize()
    _kernels.require(cfg)
    out = dx.float().cpu().view(N, H, W, Ci).permute(0, 3, 1, 2)
    assert torch.isfinite(out).all()
    assert torch.allclose(out, ref, atol=2e-2, rtol=1e-2), (out - ref).abs().max()


WG_CASES = [
    # N, H, W, C, Cout, R, S, stride, pad
    (2, 9, 7, 8, 32, 3, 3, 2, 1),        # stem-1 like (8 channels, stride 2)
    (2, 12, 12, 32, 32, 3, 3, 1, 1),     # 32 -> 32 (Cout tile 32)
    (2, 12, 12, 32, 64, 3, 3, 1, 1),     # 32 -> 64 (Cout tile 64)
    (3, 7, 5, 64, 256, 1, 1, 1, 0),      # dense 1x1
    (2, 14, 14, 128, 128, 3, 3, 1, 1),
    (4, 28, 28, 64, 64, 3, 3, 1, 1),     # many K-steps, split over workgroups
    (3, 12, 12, 512, 64, 1, 1, 2, 0),    # strided 1x1 (not dense)
    (1, 5, 5, 256, 96, 1, 1, 1, 0),      # partial Cout tile
    (2, 32, 48, 32, 32, 3, 3, 1, 1),     # halo-tiled wgrad, 16 x 16 tiles
    (3, 17, 23, 64, 64, 3, 3, 1, 1),     # halo-tiled, 8 x 16 tiles with tails, two output-channel passes
    (2, 16, 16, 64, 32, 3, 3, 1, 1),
    (3, 14, 14, 128, 192, 3, 3, 1, 1),   # halo-tiled, 64-channel slices of input and output
]


# candidates (gemm.hip tune_wgrad): -1 register-staged kernel, c + 9 * level the
# pipelined kernel's 9 tile shapes at 4 split levels, 36-39 the halo-tiled kernel variants
@pytest.mark.parametrize("cfg", ["-1", "0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "16", "20", "34", "36", "37",
                                 "38", "39", "auto"])
@pytest.mark.parametrize("case", WG_CASES)
def test_wgrad_accumulates(case, cfg, dev):
    old = os.environ.get("ARTSBIR_WGRAD_CFG")
    if cfg == "auto":
        os.environ.pop("ARTSBIR_WGRAD_CFG", None)
    else:
        os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    try:
        N, H, W, C, Co, R, S, st, pd = case
        g = torch.Generator().manual_seed(3)
        x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
        w = torch.randn(Co, C, R, S, generator=g)
        Ho = (H + 2 * pd - R) // st + 1
        Wo = (W + 2 * pd - S) // st + 1
        dy = torch.randn(N, Co, Ho, Wo, generator=g).bfloat16().float()
        wr = w.clone().requires_grad_(True)
        F.conv2d(x, wr, stride=st, padding=pd).backward(dy)
        init = torch.randn(Co, R, S, C, generator=g)
        ref = init + wr.grad.permute(0, 2, 3, 1)
        dw = init.clone().to(dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, S, st, pd)
        dyd, xd = _nhwc(dy).to(dev, torch.bfloat16), _nhwc(x).to(dev, torch.bfloat16)
        _hip.call("artsbir_conv2d_wgrad", d, dyd.data_ptr(), xd.data_ptr(), None, None, 0, dw.data_ptr(),
                  _hip.stream())
        torch.cuda.synchronize()
        _kernels.require(cfg, wgrad=True)
        assert torch.allclose(dw.cpu(), ref, atol=2e-2, rtol=1e-3), (dw.cpu() - ref).abs().max()
    finally:
        if old is None:
            os.environ.pop("ARTSBIR_WGRAD_CFG", None)
        else:
            os.environ["ARTSBIR_WGRAD_CFG"] = old


@pytest.mark.parametrize("cus", [96, 224])
@pytest.mark.parametrize("cfg", ["0", "9", "34", "38", "100", "101"])
@pytest.mark.parametrize("case", [WG_CASES[3], WG_CASES[5], WG_CASES[-1]])
def test_wgrad_grids_sized_for_fewer_cus(case, cfg, cus, dev):
    """artsbir_set_wgrad_cus (the grids of a CU-masked weight-gradient stream):
    the split-K targets and the halo kernel's persistent groups scale with the
    CU count, the result does not change"""
    lib = _hip.lib()
    old_env = os.environ.get("ARTSBIR_WGRAD_CFG")
    os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    old = lib.artsbir_set_wgrad_cus(cus)
    try:
        N, H, W, C, Co, R, S, st, pd = case
        g = torch.Generator().manual_seed(5)
        x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
        w = torch.randn(Co, C, R, S, generator=g)
        Ho = (H + 2 * pd - R) // st + 1
        Wo = (W + 2 * pd - S) // st + 1
        dy = torch.randn(N, Co, Ho, Wo, generator=g).bfloat16().float()
        wr = w.clone().requires_grad_(True)
        F.conv2d(x, wr, stride=st, padding=pd).backward(dy)
        ref = wr.grad.permute(0, 2, 3, 1)
        dw = torch.zeros(Co, R, S, C, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, S, st, pd)
        dyd, xd = _nhwc(dy).to(dev, torch.bfloat16), _nhwc(x).to(dev, torch.bfloat16)
        _hip.call("artsbir_conv2d_wgrad", d, dyd.data_ptr(), xd.data_ptr(), None, None, 0, dw.data_ptr(),
                  _hip.stream())
        torch.cuda.synchronize()
        _kernels.require(cfg, wgrad=True)
        assert torch.allclose(dw.cpu(), ref, atol=2e-2, rtol=1e-3), (dw.cpu() - ref).abs().max()
    finally:
        lib.artsbir_set_wgrad_cus(old)
        if old_env is None:
            os.environ.pop("ARTSBIR_WGRAD_CFG", None)
        else:
            os.environ["ARTSBIR_WGRAD_CFG"] = old_env


@pytest.mark.parametrize("cfg", ["-1", "0", "1", "2", "3", "6", "7", "8"])
@pytest.mark.parametrize("M,N,K,ldd,ldx", [(100, 96, 64, 96, 64), (3000, 512, 2048, 512, 2048), (77, 40, 24, 48, 32)])
def test_gemm_tn_strided(M, N, K, ldd, ldx, cfg, dev):
    os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    try:
        g = torch.Generator().manual_seed(4)
        dy = torch.randn(M, ldd, generator=g).bfloat16().float()
        x = torch.randn(M, ldx, generator=g).bfloat16().float()
        ref = dy[:, :N].t() @ x[:, :K]
        dw = torch.zeros(N, K, device=dev)
        dyd, xd = dy.to(dev, torch.bfloat16), x.to(dev, torch.bfloat16)
        _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dyd.data_ptr(), ldd, xd.data_ptr(), ldx, dw.data_ptr(),
                  _hip.stream())
        torch.cuda.synchronize()
        _kernels.require(cfg, wgrad=True)
        assert torch.allclose(dw.cpu(), ref, atol=2e-2, rtol=1e-3), (dw.cpu() - ref).abs().max()
    finally:
        os.environ.pop("ARTSBIR_WGRAD_CFG", None)


@pytest.mark.parametrize("cfg", ["auto", "0", "1", "2", "3", "4", "5", "10", "15", "19", "21"])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode", ["bias", "bias_relu", "bias_res_relu"])
def test_conv_fwd_act(case, cfg, mode, dev, cfg_env):
    """artsbir_conv2d_fwd_act (eval conv + folded BN + ReLU + residual) on every
    kernel that takes the bias / ReLU epilogue, vs torch fp32 on bf16 operands;
    shapes a candidate does not take fall back to the auto choice"""
    N, H, W, C, Co, R, S, st, pd = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Co, C, R, S, generator=g) * 0.1).bfloat16().float()
    bias = torch.randn(Co, generator=g)
    ref = F.conv2d(x, w, stride=st, padding=pd) + bias[None, :, None, None]
    res = None
    if mode == "bias_res_relu":
        res = torch.randn(ref.shape, generator=g).bfloat16().float()
        ref = ref + res
    if mode != "bias":
        ref = ref.clamp_min(0)
    Ho, Wo = ref.shape[2], ref.shape[3]
    d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, S, st, pd)
    xd = _nhwc(x).to(dev, torch.bfloat16)
    wp = torch.empty(Co, R, S, C, dtype=torch.bfloat16, device=dev)
    wd, biasd = w.to(dev), bias.to(dev)  # alive through the calls
    _hip.call("artsbir_pack_weight", _hip.DT_BF16, wd.data_ptr(), Co, C, R, S, C, 0, 0, wp.data_ptr(),
              _hip.stream())
    y = torch.empty(N, Ho, Wo, Co, dtype=torch.bfloat16, device=dev)
    resd = _nhwc(res).to(dev, torch.bfloat16) if res is not None else None
    _set(cfg)
    try:
        _hip.call("artsbir_conv2d_fwd_act", d, xd.data_ptr(), wp.data_ptr(), y.data_ptr(), biasd.data_ptr(),
                  resd.data_ptr() if resd is not None else None, 1 if resd is not None else 0,
                  0 if mode == "bias" else 1, _hip.stream())
    except _hip.HipError:
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)  # candidate not applicable to this shape / epilogue
        _hip.call("artsbir_conv2d_fwd_act", d, xd.data_ptr(), wp.data_ptr(), y.data_ptr(), biasd.data_ptr(),
                  resd.data_ptr() if resd is not None else None, 1 if resd is not None else 0,
                  0 if mode == "bias" else 1, _hip.stream())
    torch.cuda.synchronize()
    _kernels.require(cfg)
    out = y.float().cpu().permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=3e-2, rtol=1e-2), (out - ref).abs().max()


@pytest.mark.parametrize("M,N,K", [(600, 512, 256), (300, 1024, 2048), (57, 96, 64)])
def test_gemm_nt_bf16_bias(M, N, K, dev):
    """biased dense GEMM with a bf16 output (the attention-pool k|v projection) on
    the pipelined kernel, vs torch fp32"""
    g = torch.Generator().manual_seed(12)
    a = torch.randn(M, K, generator=g).bfloat16().float()
    b = (torch.randn(N, K, generator=g) * 0.05).bfloat16().float()
    bias = torch.randn(N, generator=g)
    ref = a @ b.T + bias
    c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ad, bd, biasd = a.to(dev, torch.bfloat16), b.to(dev, torch.bfloat16), bias.to(dev)  # alive through the call
    _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, ad.data_ptr(), K, bd.data_ptr(), c.data_ptr(), N, 0, 0,
              biasd.data_ptr(), None, _hip.stream())
    torch.cuda.synchronize()
    assert torch.allclose(c.float().cpu(), ref, atol=3e-2, rtol=1e-2), (c.float().cpu() - ref).abs().max()


@pytest.mark.parametrize("M,N,K,lda,ldc", [(600, 512, 256, 256, 512), (1000, 768, 768, 800, 776), (4096, 2304, 768, 768, 2304),
                                           (57, 96, 64, 64, 96), (3000, 768, 2304, 2304, 768)])
@pytest.mark.parametrize("with_bias", [False, True], ids=["plain", "bias"])
def test_gemm_nt_pp256_candidate(M, N, K, lda, ldc, with_bias, dev, cfg_env):
    """candidate 22 (pp256.hip, the ping-pong 256x256 tile that replaced the
    hipBLASLt candidate for the dense GEMMs: attention-pool k|v projection, ViT
    projection data gradients) on strided operands with an optional f32 bias per
    output column, vs torch fp32 on the same bf16 operands"""
    g = torch.Generator().manual_seed(13)
    a = torch.randn(M, lda, generator=g).bfloat16()
    b = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, generator=g)
    ref = a[:, :K].float() @ b.float().T + (bias if with_bias else 0)
    c = torch.full((M, ldc), 7.0, dtype=torch.bfloat16, device=dev)
    ad, bd, biasd = a.to(dev), b.to(dev), bias.to(dev)
    _set("22")
    _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, ad.data_ptr(), lda, bd.data_ptr(), c.data_ptr(), ldc, 0, 0,
              biasd.data_ptr() if with_bias else None, None, _hip.stream())
    torch.cuda.synchronize()
    assert _hip.lib().artsbir_last_kernel().decode() == "pp256_kernel"
    out = c.float().cpu()
    assert torch.allclose(out[:, :N], ref, atol=3e-2, rtol=1e-2), (out[:, :N] - ref).abs().max()
    assert torch.all(out[:, N:] == 7.0)  # the row padding beyond N is untouched


PW256_CASES = [
    # N, H, W, C, Cout, R, S, stride, pad
    (2, 14, 14, 128, 256, 3, 3, 1, 1),   # 3x3, a 256-k tile spans two taps
    (16, 28, 28, 128, 256, 3, 3, 1, 1),  # many m-splits
    (2, 7, 7, 512, 512, 3, 3, 1, 1),     # 7x7 images (49 pixels): a K-tile of 32 rows crosses images
    (3, 10, 9, 256, 512, 1, 1, 1, 0),    # dense 1x1
    (3, 12, 12, 512, 256, 1, 1, 2, 0),   # strided 1x1 (implicit im2col)
    (2, 9, 11, 64, 200, 3, 3, 1, 1),     # Cout and K tails (200 co, 576 k)
]


@pytest.mark.parametrize("cfg", ["100", "101", "102"])
@pytest.mark.parametrize("case", PW256_CASES)
def test_wgrad_pw256(case, cfg, dev):
    """wgrad candidates 100-102 (pw256.hip, the ping-pong 256x256 weight-gradient
    tile at three m-split levels): dW accumulated onto an existing gradient vs
    torch fp32 autograd on the same bf16 operands"""
    os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    try:
        N, H, W, C, Co, R, S, st, pd = case
        g = torch.Generator().manual_seed(21)
        x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
        w = torch.randn(Co, C, R, S, generator=g)
        Ho = (H + 2 * pd - R) // st + 1
        Wo = (W + 2 * pd - S) // st + 1
        dy = torch.randn(N, Co, Ho, Wo, generator=g).bfloat16().float()
        wr = w.clone().requires_grad_(True)
        F.conv2d(x, wr, stride=st, padding=pd).backward(dy)
        init = torch.randn(Co, R, S, C, generator=g)
        ref = init + wr.grad.permute(0, 2, 3, 1)
        dw = init.clone().to(dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, S, st, pd)
        dyd, xd = _nhwc(dy).to(dev, torch.bfloat16), _nhwc(x).to(dev, torch.bfloat16)
        _hip.call("artsbir_conv2d_wgrad", d, dyd.data_ptr(), xd.data_ptr(), None, None, 0, dw.data_ptr(),
                  _hip.stream())
        torch.cuda.synchronize()
        assert _hip.lib().artsbir_last_kernel().decode().startswith("pw256_kernel")
        assert torch.allclose(dw.cpu(), ref, atol=2e-2, rtol=1e-3), (dw.cpu() - ref).abs().max()
    finally:
        os.environ.pop("ARTSBIR_WGRAD_CFG", None)


@pytest.mark.parametrize("cfg", ["100", "102"])
@pytest.mark.parametrize("M,N,K,ldd,ldx", [(3000, 512, 2048, 512, 2048), (5001, 768, 2304, 776, 2304),
                                           (40000, 256, 768, 256, 800)])
def test_gemm_tn_pw256(M, N, K, ldd, ldx, cfg, dev):
    """artsbir_gemm_tn (the dense weight gradients of the attention pool and the
    ViT projections) on pw256, strided rows, vs torch fp32"""
    os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    try:
        g = torch.Generator().manual_seed(22)
        dy = torch.randn(M, ldd, generator=g).bfloat16().float()
        x = torch.randn(M, ldx, generator=g).bfloat16().float()
        ref = dy[:, :N].t() @ x[:, :K]
        dw = torch.zeros(N, K, device=dev)
        dyd, xd = dy.to(dev, torch.bfloat16), x.to(dev, torch.bfloat16)
        _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dyd.data_ptr(), ldd, xd.data_ptr(), ldx, dw.data_ptr(),
                  _hip.stream())
        torch.cuda.synchronize()
        assert _hip.lib().artsbir_last_kernel().decode() == "pw256_kernel<dense>"
        assert torch.allclose(dw.cpu(), ref, atol=5e-2, rtol=1e-3), (dw.cpu() - ref).abs().max()
    finally:
        os.environ.pop("ARTSBIR_WGRAD_CFG", None)
