"""Every entry of the committed autotuner table (profiles/tune_r6.txt, the table
bench.py loads, so every bench / profiling run launches these kernels) at its
exact shape: the entry's candidate forced (ARTSBIR_PGEMM_CFG / ARTSBIR_WGRAD_CFG),
the kernel that ran asserted by name — a candidate that does not take its own
table shape FAILS here, it is not skipped — and the result checked against an
fp32/f64 reference on the same bf16 operands:

  conv / GEMM keys   sampled output rows (every output channel) against the
                     im2col product on the CPU, with the entry's epilogue: BN
                     segment statistics (conv2d_fwd_seg), bias / residual / ReLU
                     (conv2d_fwd_act), residual data gradients (conv2d_dgrad),
                     the fused BN-backward masks of kinds 1 and 3 (conv2d_dgrad_bnb),
                     the folded BN backward's two operands (conv1x1_dgrad_fold)
                     and the QuickGELU gate (gemm_nt_gate);
  weight-gradient keys  sampled output rows (every column) against a torch fp32
                     GEMM per filter tap over the whole reduction, including the
                     split levels 14 and 27-31 and the two-part dY of gemm_tn2.

The reference's layers these shapes come from: models.py:191-272 (C2 step /
embed pass), models.py:396-417 (C5 blocks)."""
import os
import re

import pytest
import torch
import torch.nn.functional as F

import _hip
import _kernels

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "profiles", "tune_r6.txt")
BF = torch.bfloat16
NSAMPLE = 48


def _entries():
    out = []
    with open(TABLE) as f:
        for line in f:
            t = line.split()
            if t and t[0] in ("c", "w"):
                out.append((t[0], [int(v) for v in t[1:]]))
    return out


ENTRIES = _entries()
IDS = [f"{k}:" + "_".join(str(v) for v in vals) for k, vals in ENTRIES]


@pytest.fixture
def forced():
    keys = ("ARTSBIR_PGEMM_CFG", "ARTSBIR_WGRAD_CFG")
    old = {k: os.environ.get(k) for k in keys}
    yield
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _rnd(*shape, dev, gen, scale=1.0):
    return (torch.randn(*shape, device=dev, generator=gen) * scale).to(BF)


def _rows(M, gen_cpu):
    idx = torch.randint(0, M, (NSAMPLE,), generator=gen_cpu)
    return torch.cat([torch.tensor([0, M - 1]), idx]).unique()


def _patches(x, idx, Ho, Wo, R, S, stride, pad):
    """im2col rows of the NHWC tensor x for output pixels idx: [P][R*S*C] f64 (CPU)"""
    N, H, W, C = x.shape
    n, r = idx // (Ho * Wo), idx % (Ho * Wo)
    ho, wo = r // Wo, r % Wo
    out = torch.zeros(len(idx), R, S, C, dtype=torch.float64)
    for dr in range(R):
        for ds in range(S):
            hi, wi = ho * stride + dr - pad, wo * stride + ds - pad
            ok = (hi >= 0) & (hi < H) & (wi >= 0) & (wi < W)
            if ok.any():
                v = x[n[ok].to(x.device), hi[ok].to(x.device), wi[ok].to(x.device)]
                out[ok, dr, ds] = v.double().cpu()
    return out.reshape(len(idx), -1)


def _close(got, ref, what):
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    rel = ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()
    assert rel < 1.2e-2 and err < 4e-2 * scale, (what, rel, err, scale)


# the two-operand (fold) form of each candidate that has one
FOLD_PREFIX = {"2": "pgemm_kernel<256,64,", "16": "pgemm_kernel<128,128,k32,glb,", "19": "pgemm_kernel<256,128,k32,glb,",
               "10": "pstream_kernel<", "14": "pstream_kernel<64,bnbk,", "22": "pp256_kernel<"}


def _check_name(cfg, name, fold=False):
    if fold:
        assert cfg in FOLD_PREFIX and name.startswith(FOLD_PREFIX[cfg]) and name.endswith("fold>"), (cfg, name)
        return
    assert re.match(_kernels.CONV[cfg], name), (cfg, name, _kernels.CONV[cfg])


def _bn_params(G, C, dev, gen):
    prm = torch.zeros(G, 4, C, device=dev)
    prm[:, 0] = torch.randn(G, C, device=dev, generator=gen) * 0.1
    prm[:, 1] = torch.rand(G, C, device=dev, generator=gen) + 0.5
    prm[:, 2] = prm[:, 1] * (torch.rand(G, C, device=dev, generator=gen) + 0.5)
    prm[:, 3] = torch.randn(G, C, device=dev, generator=gen) * 0.2
    return prm


def _conv_entry(vals, dev):
    M, H, W, C, Cout, R, S, stride, pad, Ho, Wo, res_mode, flags, nseg, bnb, choice = vals
    cfg = str(choice)
    os.environ["ARTSBIR_PGEMM_CFG"] = cfg
    gen = torch.Generator(device=dev).manual_seed(M % 1000003 + C * 7 + Cout)
    gcpu = torch.Generator().manual_seed(M % 997 + Cout)
    N = M // (Ho * Wo)
    st = _hip.stream()
    rows = _rows(M, gcpu)
    x2 = flags & 8
    if x2:  # folded BN backward: [g | x] w_s^T + bias_s (conv1x1_dgrad_fold), key C = Co + Ci, Cout = Ci
        Ci, Co = Cout, C - Cout
        g = _rnd(N, H, W, Co, dev=dev, gen=gen)
        x = _rnd(N, H, W, Ci, dev=dev, gen=gen)
        w = _rnd(nseg, Ci, Co + Ci, dev=dev, gen=gen, scale=(Co + Ci) ** -0.5)
        bias = torch.randn(nseg, Ci, device=dev, generator=gen)
        dx = torch.full((N, H, W, Ci), float("nan"), dtype=BF, device=dev)
        d = _hip.conv_desc(BF, N, H, W, Ci, Co, 1, 1, 1, 0)
        desc, keep = None, None
        if bnb:
            y2 = _rnd(N, H, W, Ci, dev=dev, gen=gen)
            prm = _bn_params(nseg, Ci, dev, gen)
            slots = torch.zeros(nseg, _hip.NSLOT, 2, Ci, device=dev)
            desc = _hip.BnBwdDesc()
            desc.dtype, desc.kind, desc.pool, desc.ntarget = _hip.DT_BF16, 1, 0, 1
            desc.mask_bn = prm.data_ptr()
            desc.y[0], desc.mean[0], desc.istd[0], desc.slots[0] = y2.data_ptr(), prm.data_ptr(), prm[0, 1].data_ptr(), \
                slots.data_ptr()
            desc.B, desc.H, desc.W, desc.C = N, H, W, Ci
            keep = (y2, prm, slots)
        _hip.call("artsbir_conv1x1_dgrad_fold", d, g.data_ptr(), x.data_ptr(), w.data_ptr(), bias.data_ptr(),
                  dx.data_ptr(), desc, nseg, 4 * Ci, st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel(), fold=True)
        seg = rows // (M // nseg)
        pa = torch.cat([_patches(g, rows, H, W, 1, 1, 1, 0), _patches(x, rows, H, W, 1, 1, 1, 0)], 1)
        wc, bc = w.double().cpu(), bias.double().cpu()
        ref = torch.einsum("pk,pik->pi", pa, wc[seg]) + bc[seg]
        if bnb:
            y2, prm, _ = keep
            pc = prm.double().cpu()[seg]
            yv = _patches(y2, rows, H, W, 1, 1, 1, 0)
            ref = torch.where((yv - pc[:, 0]) * pc[:, 2] + pc[:, 3] > 0, ref, torch.zeros_like(ref))
        _close(dx.reshape(M, Ci)[rows.to(dev)].double().cpu(), ref, "fold")
        return
    if res_mode == 3:  # C = (A B^T) * quickgelu'(X), column sums of C into the statistics
        a = _rnd(M, C, dev=dev, gen=gen)
        b = _rnd(Cout, C, dev=dev, gen=gen, scale=C ** -0.5)
        xg = _rnd(M, Cout, dev=dev, gen=gen)
        c = torch.empty(M, Cout, dtype=BF, device=dev)
        stats = torch.zeros(_hip.NSLOT, 2, Cout, device=dev)
        _hip.call("artsbir_gemm_nt_gate", M, Cout, C, a.data_ptr(), C, b.data_ptr(), c.data_ptr(), Cout,
                  xg.data_ptr(), stats.data_ptr(), st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel())
        ad, bd_, xv = a[rows.to(dev)].double().cpu(), b.double().cpu(), xg[rows.to(dev)].double().cpu()
        s = torch.sigmoid(1.702 * xv)
        ref = (ad @ bd_.T) * (s * (1 + 1.702 * xv * (1 - s)))
        _close(c[rows.to(dev)].double().cpu(), ref, "gate")
        return
    x = _rnd(N, H, W, C, dev=dev, gen=gen)
    w = _rnd(Cout, R, S, C, dev=dev, gen=gen, scale=(R * S * C) ** -0.5)
    y = torch.full((N, Ho, Wo, Cout), float("nan"), dtype=BF, device=dev)
    pa = _patches(x, rows, Ho, Wo, R, S, stride, pad)
    ref = pa @ w.reshape(Cout, -1).double().cpu().T
    pix = rows.to(dev)
    got = lambda: y.reshape(M, Cout)[pix].double().cpu()  # noqa: E731
    if bnb:  # fused BN-backward data gradient: key C = dy channels, Cout = dx channels
        kind, nt = bnb // 4, bnb % 4
        kind = 1 if kind == 1 else 3 if kind == 3 else 0
        d = _hip.conv_desc(BF, N, H, W, Cout, C, R, S, 1, R - 1 - pad)
        res = None
        if res_mode == 1:
            res = _rnd(N, H, W, Cout, dev=dev, gen=gen)
            ref = ref + _patches(res, rows, H, W, 1, 1, 1, 0)
        elif res_mode == 2:
            res = _rnd(N, H // 2, W // 2, Cout, dev=dev, gen=gen)
            n, r = rows // (H * W), rows % (H * W)
            ridx = (n * (H // 2) + (r // W) // 2) * (W // 2) + (r % W) // 2
            ref = ref + 0.25 * _patches(res, ridx, H // 2, W // 2, 1, 1, 1, 0)
        ys = [_rnd(N, H, W, Cout, dev=dev, gen=gen) for _ in range(nt)]
        prms = [_bn_params(nseg, Cout, dev, gen) for _ in range(nt)]
        slots = [torch.zeros(nseg, _hip.NSLOT, 2, Cout, device=dev) for _ in range(nt)]
        desc = _hip.BnBwdDesc()
        desc.dtype, desc.kind, desc.pool, desc.ntarget = _hip.DT_BF16, kind, 0, nt
        seg = rows // (M // nseg)
        if kind == 1:
            desc.mask_bn = prms[0].data_ptr()
            pc = prms[0].double().cpu()[seg]
            yv = _patches(ys[0], rows, H, W, 1, 1, 1, 0)
            keep = (yv - pc[:, 0]) * pc[:, 2] + pc[:, 3] > 0
        else:
            bits = torch.randint(0, 256, (M, Cout // 8), device=dev, generator=gen, dtype=torch.int32).to(torch.uint8)
            desc.mask = bits.data_ptr()
            bv = bits[pix].long().cpu()
            keep = ((bv[:, :, None] >> torch.arange(8)) & 1).reshape(len(rows), Cout) > 0
        for t in range(nt):
            desc.y[t], desc.mean[t], desc.istd[t] = ys[t].data_ptr(), prms[t].data_ptr(), prms[t][0, 1].data_ptr()
            desc.slots[t] = slots[t].data_ptr()
        desc.B, desc.H, desc.W, desc.C = N, H, W, Cout
        _hip.call("artsbir_conv2d_dgrad_bnb", d, x.data_ptr(), w.data_ptr(), y.data_ptr(),
                  res.data_ptr() if res is not None else None, res_mode, desc, nseg, 4 * Cout, st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel())
        _close(got(), torch.where(keep, ref, torch.zeros_like(ref)), f"dgrad_bnb k{kind}")
        return
    if res_mode in (1, 2) and not (flags & 6):  # residual data gradient
        d = _hip.conv_desc(BF, N, H, W, Cout, C, R, S, 1, R - 1 - pad)
        res = _rnd(*((N, H, W, Cout) if res_mode == 1 else (N, H // 2, W // 2, Cout)), dev=dev, gen=gen)
        if res_mode == 1:
            ref = ref + _patches(res, rows, H, W, 1, 1, 1, 0)
        else:
            n, r = rows // (H * W), rows % (H * W)
            ridx = (n * (H // 2) + (r // W) // 2) * (W // 2) + (r % W) // 2
            ref = ref + 0.25 * _patches(res, ridx, H // 2, W // 2, 1, 1, 1, 0)
        _hip.call("artsbir_conv2d_dgrad", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), res.data_ptr(), res_mode, st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel())
        _close(got(), ref, "dgrad res")
        return
    d = _hip.conv_desc(BF, N, H, W, C, Cout, R, S, stride, pad)
    if flags & 1:  # BN statistics per segment
        stats = torch.zeros(nseg, _hip.NSLOT, 2, Cout, device=dev)
        _hip.call("artsbir_conv2d_fwd_seg", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), nseg, stats.data_ptr(), st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel())
        _close(got(), ref, "fwd_seg")
        # the statistics: sum over the segment of the stored bf16 output, in f32
        s = stats.sum(1)
        yo = y.reshape(nseg, -1, Cout).float()
        assert torch.allclose(s[:, 0], yo.sum(1), rtol=2e-2, atol=2e-2 * (M // nseg) ** 0.5)
        return
    if flags & 6:  # bias (+ residual) (+ ReLU): the eval forward / linear heads
        bias = torch.randn(Cout, device=dev, generator=gen)
        res = _rnd(N, Ho, Wo, Cout, dev=dev, gen=gen) if res_mode == 1 else None
        relu = 1 if flags & 4 else 0
        _hip.call("artsbir_conv2d_fwd_act", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), bias.data_ptr(),
                  res.data_ptr() if res is not None else None, res_mode, relu, st)
        torch.cuda.synchronize()
        _check_name(cfg, _kernels.last_kernel())
        ref = ref + bias.double().cpu()
        if res is not None:
            ref = ref + _patches(res, rows, Ho, Wo, 1, 1, 1, 0)
        if relu:
            ref = ref.clamp_min(0)
        _close(got(), ref, "fwd_act")
        return
    _hip.call("artsbir_conv2d_fwd", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), Cout, 0, 0, None, None, None, 0,
              None, st)
    torch.cuda.synchronize()
    _check_name(cfg, _kernels.last_kernel())
    _close(got(), ref, "fwd")


def _wgrad_entry(vals, dev):
    M, H, W, C, Cout, R, S, stride, pad, dense, K, ldd, ldx, choice = vals
    cfg = str(choice)
    os.environ["ARTSBIR_WGRAD_CFG"] = cfg
    gen = torch.Generator(device=dev).manual_seed(M % 1000003 + 3 * C + Cout)
    gcpu = torch.Generator().manual_seed(Cout + C)
    st = _hip.stream()
    outs = []
    if dense == 2:  # gemm_tn2: dY in two parts along Cout (the fold's g^T x and x^T x)
        N1, N2 = ldd, Cout - ldd
        dy = _rnd(M, N1, dev=dev, gen=gen)
        dy2 = _rnd(M, N2, dev=dev, gen=gen)
        x = _rnd(M, K, dev=dev, gen=gen)
        dw, dw2 = torch.zeros(N1, K, device=dev), torch.zeros(N2, K, device=dev)
        _hip.call("artsbir_gemm_tn2", _hip.DT_BF16, M, N1, N2, K, dy.data_ptr(), N1, dy2.data_ptr(), N2, x.data_ptr(),
                  K, dw.data_ptr(), dw2.data_ptr(), st)
        outs = [(dw, dy, x), (dw2, dy2, x)]
    elif dense == 1 and H == 1 and W == 1:  # gemm_tn with a row stride (the attention-pool token rows)
        dy = _rnd(M, Cout, dev=dev, gen=gen)
        xb = _rnd((M - 1) * ldx + K, dev=dev, gen=gen)
        x = xb.as_strided((M, K), (ldx, 1))
        dw = torch.zeros(Cout, K, device=dev)
        _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, Cout, K, dy.data_ptr(), ldd, xb.data_ptr(), ldx, dw.data_ptr(),
                  st)
        outs = [(dw, dy, x)]
    else:
        Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        N = M // (Ho * Wo)
        xi = _rnd(N, H, W, C, dev=dev, gen=gen)
        dy = _rnd(N * Ho * Wo, Cout, dev=dev, gen=gen)
        dw = torch.zeros(Cout, R, S, C, device=dev)
        d = _hip.conv_desc(BF, N, H, W, C, Cout, R, S, stride, pad)
        _hip.call("artsbir_conv2d_wgrad", d, dy.data_ptr(), xi.data_ptr(), None, None, 0, dw.data_ptr(), st)
        xp = F.pad(xi, (0, 0, pad, pad, pad, pad))
        taps = []
        for dr in range(R):
            for ds in range(S):
                taps.append(xp[:, dr:dr + stride * (Ho - 1) + 1:stride, ds:ds + stride * (Wo - 1) + 1:stride, :]
                            .reshape(-1, C))
        outs = [(dw.reshape(Cout, R * S, C), dy, taps)]
    torch.cuda.synchronize()
    name = _kernels.last_kernel()
    assert re.match(_kernels.wgrad_pattern(cfg), name), (cfg, name)
    for dw, dy, x in outs:
        n = dw.shape[0]
        sel = torch.cat([torch.tensor([0, n - 1]), torch.randint(0, n, (14,), generator=gcpu)]).unique().to(dev)
        dys = dy[:, sel].float()
        if isinstance(x, list):
            ref = torch.stack([dys.T @ t.float() for t in x], 1)  # [sel][taps][C]
        else:
            ref = dys.T @ x.float()
        got = dw[sel]
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel < 2e-3, (cfg, name, rel)


@pytest.mark.parametrize("entry", ENTRIES, ids=IDS)
def test_tune_table_entry(entry, dev, forced):
    kind, vals = entry
    if kind == "c":
        _conv_entry(vals, dev)
    else:
        _wgrad_entry(vals, dev)
    torch.cuda.empty_cache()


def test_tune_table_covers_the_split_levels():
    """the weight-gradient split levels the table uses (14, 27-31) are among the
    entries above, so each is forced at a shape of its own"""
    used = {vals[-1] for kind, vals in ENTRIES if kind == "w"}
    assert {14, 27, 28, 29, 30, 31} <= used, used
