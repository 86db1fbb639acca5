"""Bottleneck and AttentionPool2d called on their own (the reference's submodule
forwards, models.py:191-236 and 239-272): forward (train and eval BatchNorm),
running statistics and the backward (input and parameter gradients) on the HIP
kernels against the float64 oracle modules (oracle/encoder.py) with the same
parameters, in f32 mode; bf16 mode against the same oracle with bf16-level bars."""
import copy

import pytest
import torch

from oracle import encoder as oenc

pytestmark = pytest.mark.gpu


def _pair(kind, seed):
    import models
    torch.manual_seed(seed)
    if kind[0] == "block":
        _, cin, planes, stride = kind
        mine, ref = models.Bottleneck(cin, planes, stride), oenc.Bottleneck(cin, planes, stride)
    else:
        _, sp, emb, heads, out = kind
        mine, ref = models.AttentionPool2d(sp, emb, heads, out), oenc.AttentionPool2d(sp, emb, heads, out)
    ref.load_state_dict(mine.state_dict())
    for m in ref.modules():  # non-trivial BN affine parameters
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    mine.load_state_dict(ref.state_dict())
    return mine, ref.double()


KINDS = [("block", 64, 16, 1), ("block", 64, 32, 2), ("block", 128, 32, 1), ("pool", 4, 512, 8, 64)]
IDS = ["block-proj", "block-stride2", "block-identity", "attnpool"]


@pytest.mark.parametrize("kind", KINDS, ids=IDS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_submodule_forward_backward_matches_oracle(kind, dtype, dev):
    mine, ref = _pair(kind, 3)
    mine = mine.to(dev)
    mine.compute_dtype = dtype
    if kind[0] == "block":
        x = torch.randn(6, kind[1], 16, 16, dtype=torch.float64)
    else:
        x = torch.randn(6, kind[2], kind[1], kind[1], dtype=torch.float64)
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    state0 = copy.deepcopy(ref.state_dict())
    for train in (True, False):
        mine.train(train)
        ref.train(train)
        xm = x.float().to(dev).requires_grad_(train)
        xr = x.clone().requires_grad_(train)
        out = mine(xm)
        want = ref(xr)
        assert out.shape == want.shape and out.dtype == torch.float32
        err = (out.double().cpu() - want.detach()).norm() / want.norm()
        assert err < tol, (train, err.item())
        if not train:
            continue
        w = torch.randn(want.shape, dtype=torch.float64)
        (out * w.float().to(dev)).sum().backward()
        (want * w).sum().backward()
        gx = (xm.grad.double().cpu() - xr.grad).norm() / xr.grad.norm()
        assert gx < tol * 5, gx.item()
        if dtype == torch.float32:
            floor = 1e-4 * max(p.grad.norm().item() for p in ref.parameters())
            for (k, pm), (_, pr) in zip(mine.named_parameters(), ref.named_parameters()):
                e = (pm.grad.double().cpu() - pr.grad).norm().item() / max(pr.grad.norm().item(), floor)
                assert e < tol * 5, (k, e)
        else:
            # bf16: per-parameter BN sums of bf16 gradients cancel (a bias gradient
            # can be ~1e-2 of its terms), so the bar is on the whole gradient vector
            # measured against what bf16 arithmetic itself does here: the oracle
            # under CPU bf16 autocast, the same bar as tests/test_c2_gpu.py
            gm = torch.cat([p.grad.double().cpu().flatten() for p in mine.parameters()])
            gr = torch.cat([p.grad.flatten() for p in ref.parameters()])
            auto = copy.deepcopy(ref).float()
            auto.zero_grad()
            auto.load_state_dict(state0)
            auto.train()
            with torch.autocast("cpu", dtype=torch.bfloat16):
                ya = auto(x.float())
            (ya.float() * w.float()).sum().backward()
            ga = torch.cat([p.grad.double().flatten() for p in auto.parameters()])
            e_mine = ((gm - gr).norm() / gr.norm()).item()
            e_auto = ((ga - gr).norm() / gr.norm()).item()
            assert e_mine < max(5e-2, 2 * e_auto), (e_mine, e_auto)
    # running statistics after the one train-mode call (bf16: statistics of bf16-rounded activations)
    rt, at = (1e-4, 1e-5) if dtype == torch.float32 else (3e-2, 1e-2)
    for (k, bm), (_, br) in zip(mine.named_buffers(), ref.named_buffers()):
        if bm.dtype.is_floating_point:
            assert torch.allclose(bm.double().cpu(), br, rtol=rt, atol=at), (k, (bm.double().cpu() - br).abs().max())


def test_submodule_no_grad_and_cpu_input(dev):
    import models
    blk = models.Bottleneck(64, 16).to(dev).eval()
    with torch.no_grad():
        y = blk(torch.randn(2, 64, 8, 8, device=dev))
    assert y.shape == (2, 64, 8, 8) and y.grad_fn is None
    with pytest.raises(RuntimeError):
        blk(torch.randn(2, 64, 8, 8))  # the module runs on the GPU only
