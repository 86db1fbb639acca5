"""Transformer block of models.py:382-417 (forward parity).

CPU: the oracle restatement against the PyTorch modules the reference's block
is made of (nn.MultiheadAttention, nn.LayerNorm in fp32, Linear) — the
reference's arithmetic lives in PyTorch, so this pins the restatement.
GPU: the HIP forward (artsbir_layernorm_fwd, gemm_nt, artsbir_mha_fwd,
artsbir_quickgelu) against the oracle, f32 within 2e-4 relative, bf16 within
3e-2."""
import pytest
import torch
from torch import nn

from oracle import encoder as oenc


def _torch_block(E, heads, seed):
    torch.manual_seed(seed)
    attn = nn.MultiheadAttention(E, heads)
    ln1, ln2 = nn.LayerNorm(E), nn.LayerNorm(E)
    fc, proj = nn.Linear(E, 4 * E), nn.Linear(4 * E, E)
    for m in (ln1, ln2):  # non-trivial affine
        nn.init.normal_(m.weight, 1.0, 0.1)
        nn.init.normal_(m.bias, 0.0, 0.1)
    sd = {"attn.in_proj_weight": attn.in_proj_weight, "attn.in_proj_bias": attn.in_proj_bias,
          "attn.out_proj.weight": attn.out_proj.weight, "attn.out_proj.bias": attn.out_proj.bias,
          "ln_1.weight": ln1.weight, "ln_1.bias": ln1.bias, "ln_2.weight": ln2.weight, "ln_2.bias": ln2.bias,
          "mlp.c_fc.weight": fc.weight, "mlp.c_fc.bias": fc.bias,
          "mlp.c_proj.weight": proj.weight, "mlp.c_proj.bias": proj.bias}
    sd = {k: v.detach() for k, v in sd.items()}

    def run(x, mask=None):
        h = ln1(x.float()).to(x.dtype)
        x = x + attn(h, h, h, need_weights=False, attn_mask=mask)[0]
        h = ln2(x.float()).to(x.dtype)
        f = fc(h)
        return x + proj(f * torch.sigmoid(1.702 * f))
    return sd, run


@pytest.mark.parametrize("masked", [False, True])
def test_oracle_block_matches_torch_modules(masked):
    E, heads, L, N = 128, 2, 9, 3
    sd, run = _torch_block(E, heads, 5)
    x = torch.randn(L, N, E, generator=torch.Generator().manual_seed(6))
    mask = torch.triu(torch.full((L, L), float("-inf")), 1) if masked else None
    with torch.no_grad():
        ref = run(x, mask)
    got = oenc.residual_attention_block(x, sd, heads, mask)
    assert torch.allclose(got, ref, atol=2e-5, rtol=1e-5), (got - ref).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("L,N,E,heads,masked", [(9, 3, 128, 2, False), (197, 2, 768, 12, False),
                                                 (17, 4, 256, 4, True)])
def test_hip_block_matches_oracle(L, N, E, heads, masked, dtype, tol, dev):
    import models
    torch.manual_seed(11)
    mask = torch.triu(torch.full((L, L), float("-inf")), 1) if masked else None
    blk = models.ResidualAttentionBlock(E, heads, attn_mask=mask)
    for m in (blk.ln_1, blk.ln_2):
        nn.init.normal_(m.weight, 1.0, 0.1)
        nn.init.normal_(m.bias, 0.0, 0.1)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    x = torch.randn(L, N, E, generator=torch.Generator().manual_seed(12))
    if dtype == torch.bfloat16:
        x = x.bfloat16().float()
    ref = oenc.residual_attention_block(x.double(), {k: v.double() for k, v in sd.items()}, heads,
                                        mask.double() if mask is not None else None)
    blk = blk.to(dev)
    got = blk(x.to(dev, dtype)).float().cpu()
    err = (got.double() - ref).norm() / ref.norm()
    assert err < tol, float(err)


@pytest.mark.gpu
def test_hip_block_backward_refuses(dev):
    import models
    blk = models.ResidualAttentionBlock(128, 2).to(dev)
    x = torch.randn(5, 2, 128, device=dev, requires_grad=True)
    y = blk(x)
    with pytest.raises(NotImplementedError):
        y.sum().backward()
