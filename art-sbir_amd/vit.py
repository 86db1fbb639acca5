"""Transformer pieces of /root/reference/models.py:382-417 and the ViT-B/16
encoder of configuration C5, forward AND backward on
libartsbir_hip.

  LayerNorm               models.py:382-388 (fp32 arithmetic whatever the storage dtype)
  QuickGELU               models.py:391-393
  ResidualAttentionBlock  models.py:396-417 (pre-LN block, nn.MultiheadAttention
                          seq-first, MLP 4x with QuickGELU) — same submodules and
                          state-dict keys as the reference
  Transformer             CLIP's stack of ResidualAttentionBlocks (key "resblocks.<i>")
  VisionTransformer       CLIP's ViT image encoder (conv1 patch embedding, class
                          embedding, positional embedding, ln_pre, transformer,
                          ln_post on the class token, proj): the reference ships
                          only the blocks; the keys follow CLIP's model so
                          a CLIP ViT-B/16 state dict loads as is.

Each block is ONE autograd node (_BlockFunction): its forward saves what the
backward needs (the attention's per-row log-sum-exp instead of the probability
matrix) and its backward runs the library's kernels: MFMA GEMMs for the five
projections (data gradients through transposed weights, weight gradients by
artsbir_gemm_tn, bias gradients by artsbir_colsum), artsbir_mha_bwd,
artsbir_quickgelu_bwd, artsbir_layernorm_bwd (residual branch gradient added in
the same pass).  The residual stream of the forward is summed in f32.

compute dtype (``compute_dtype``): torch.float32 (parity), torch.bfloat16, or
"fp8": the projection GEMMs of the forward run on fp8 e4m3 operands with
per-tensor scales (artsbir_gemm_nt_fp8, MX-scaled MFMA) and bf16 elsewhere;
the backward stays bf16.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import torch
from torch import nn

import _hip
from _hip import call


def _dt(x: torch.Tensor) -> int:
    if not x.is_cuda or x.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("transformer: CUDA (HIP) f32/bf16 tensors only; there is no CPU path")
    return _hip.DT_BF16 if x.dtype == torch.bfloat16 else _hip.DT_F32


def _st() -> int:
    return torch.cuda.current_stream().cuda_stream


def _as(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """f32 parameter in the compute dtype (artsbir_cast)"""
    w = w.detach().float().contiguous()
    if dtype == torch.float32:
        return w
    out = torch.empty(w.shape, dtype=dtype, device=w.device)
    call("artsbir_cast", _hip.DT_F32, w.data_ptr(), _hip.DT_BF16, out.data_ptr(), w.numel(), _st())
    return out


def _t(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """2-D parameter [R][C] transposed to [C][R] in the compute dtype (artsbir_pack_weight, mode 1)"""
    w = w.detach().float().contiguous()
    R, C = w.shape
    out = torch.empty(C, R, dtype=dtype, device=w.device)
    call("artsbir_pack_weight", _hip.dtype_code(dtype), w.data_ptr(), R, C, 1, 1, C, 1, R, out.data_ptr(), _st())
    return out


def _cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    call("artsbir_cast", _dt(x), x.data_ptr(), _dt(out), out.data_ptr(), x.numel(), _st())
    return out


def _gemm(a: torch.Tensor, b_nk: torch.Tensor, M: int, N: int, K: int, bias=None, out=None, out_f32=False):
    """C[M][N] = A[M][K] @ B[N][K]^T (+ bias); with `out` (f32) given, accumulated onto it"""
    acc = out is not None
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32 if out_f32 else a.dtype, device=a.device)
    call("artsbir_gemm_nt", _dt(a), M, N, K, a.data_ptr(), K, b_nk.data_ptr(), out.data_ptr(), N,
         1 if (acc or out.dtype == torch.float32) else 0, 1 if acc else 0,
         bias.data_ptr() if bias is not None else None, None, _st(), kernel="auto", flops=2.0 * M * N * K,
         nbytes=float(a.element_size() * (M * K + N * K) + out.element_size() * M * N * (2 if acc else 1)),
         tag=f"vit gemm_nt {M}x{N}x{K}")
    return out


def _wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor):
    """dw[N][K] += sum_m dy[m][n] x[m][k]"""
    M, N = dy.shape
    K = x.shape[1]
    call("artsbir_gemm_tn", _dt(dy), M, N, K, dy.data_ptr(), N, x.data_ptr(), K, dw.data_ptr(), _st(),
         kernel="auto", flops=2.0 * M * N * K, nbytes=float(dy.element_size() * (M * N + M * K) + 8 * N * K),
         tag=f"vit gemm_tn {M}x{N}x{K}")


def _colsum(x: torch.Tensor, out: torch.Tensor):
    call("artsbir_colsum", _dt(x), x.data_ptr(), x.shape[0], x.shape[1], x.shape[1], out.data_ptr(), _st())


PMAX = 4096  # partial maxima a fused-amax producer folds into (csrc/vit.hip vt_block_amax)


def _pmax(dev) -> torch.Tensor:
    return torch.zeros(PMAX, dtype=torch.int32, device=dev)


def _ln(x2: torch.Tensor, w, b, eps, pmax=None) -> torch.Tensor:
    """LayerNorm forward; with pmax (fp8 mode) its max |y| is folded into pmax on the way"""
    y = torch.empty_like(x2)
    wg, bg = w.detach().float().contiguous(), b.detach().float().contiguous()
    if pmax is None:
        call("artsbir_layernorm_fwd", _dt(x2), x2.data_ptr(), wg.data_ptr(), bg.data_ptr(), x2.shape[0], x2.shape[1],
             float(eps), y.data_ptr(), _st())
    else:
        call("artsbir_layernorm_fwd_pmax", _dt(x2), x2.data_ptr(), wg.data_ptr(), bg.data_ptr(), x2.shape[0],
             x2.shape[1], float(eps), y.data_ptr(), pmax.data_ptr(), _st())
    return y


def _ln_bwd(x2, w, dy2, eps, dres, dw, db, dres_sum=None, dx_sum=None) -> torch.Tensor:
    """LayerNorm backward (+ residual gradient); with dres_sum / dx_sum the column
    sums of dres and dx (bias gradients of the projections around it) in the same pass"""
    dx = torch.empty_like(x2)
    wg = w.detach().float().contiguous()
    if dres_sum is None and dx_sum is None:
        call("artsbir_layernorm_bwd", _dt(x2), x2.data_ptr(), wg.data_ptr(), dy2.data_ptr(), x2.shape[0],
             x2.shape[1], float(eps), dres.data_ptr() if dres is not None else None, dx.data_ptr(), dw.data_ptr(),
             db.data_ptr(), _st())
    else:
        call("artsbir_layernorm_bwd_sums", _dt(x2), x2.data_ptr(), wg.data_ptr(), dy2.data_ptr(), x2.shape[0],
             x2.shape[1], float(eps), dres.data_ptr() if dres is not None else None, dx.data_ptr(), dw.data_ptr(),
             db.data_ptr(), dres_sum.data_ptr() if dres_sum is not None else None,
             dx_sum.data_ptr() if dx_sum is not None else None, _st())
    return dx


# ------------------------------------------------------------ fp8 projections
FP8_MAX = 448.0  # e4m3fn


def _fp8(x: torch.Tensor, pmax=None):
    """per-tensor e4m3 quantisation on the device: (uint8 codes, f32 scale tensor [1]);
    pmax: the partial maxima x's producer folded (no amax pass over x)"""
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    sc = torch.empty(1, dtype=torch.float32, device=x.device)
    if pmax is None:
        call("artsbir_quantize_fp8", _dt(x), x.data_ptr(), x.numel(), q.data_ptr(), sc.data_ptr(), _st())
    else:
        call("artsbir_quantize_fp8_pmax", _dt(x), x.data_ptr(), x.numel(), pmax.data_ptr(), pmax.numel(),
             q.data_ptr(), sc.data_ptr(), _st(), kernel="fp8_quant_kernel",
             nbytes=float(x.numel() * (x.element_size() + 1)), tag=f"vit quantize {x.numel()}")
    return q, sc


def _gemm_fp8(a: torch.Tensor, w: torch.Tensor, bias, out=None, out_dtype=torch.bfloat16, a_pmax=None,
              accumulate=None, res=None, out2=None, skip_c=False):
    """C = A @ W^T (+ bias) (+ C if accumulate) (+ res) with both operands quantised
    to e4m3 per tensor; out2: a bf16 copy of the result; skip_c: C not written"""
    M, K = a.shape
    N = w.shape[0]
    qa, sa = _fp8(a, a_pmax)
    qw, sw = _fp8(_as(w, torch.bfloat16))
    acc = (out is not None) if accumulate is None else accumulate
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    b = bias.detach().float().contiguous() if bias is not None else None
    es = out.element_size()
    nb = M * K + N * K + M * N * ((0 if skip_c else es) + (es if acc else 0) + (2 if res is not None else 0)
                                  + (2 if out2 is not None else 0))
    call("artsbir_gemm_nt_fp8_ex", M, N, K, qa.data_ptr(), qw.data_ptr(), sa.data_ptr(), sw.data_ptr(),
         b.data_ptr() if b is not None else None, out.data_ptr(), _hip.dtype_code(out.dtype), 1 if acc else 0,
         res.data_ptr() if res is not None else None, out2.data_ptr() if out2 is not None else None,
         1 if skip_c else 0, _st(), kernel="auto", flops=2.0 * M * N * K, nbytes=float(nb),
         tag=f"vit gemm_fp8 {M}x{N}x{K}")
    return out


def _gemm_fp8_gelu(a: torch.Tensor, w: torch.Tensor, bias, a_pmax, g_pmax):
    """f = A @ W^T + bias and g = quickgelu(f), both bf16, from one fp8 GEMM whose
    epilogue also folds max |g| into g_pmax (g's quantiser then skips the amax pass)"""
    M, K = a.shape
    N = w.shape[0]
    qa, sa = _fp8(a, a_pmax)
    qw, sw = _fp8(_as(w, torch.bfloat16))
    f = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    g = torch.empty_like(f)
    b = bias.detach().float().contiguous() if bias is not None else None
    call("artsbir_gemm_nt_fp8_gelu", M, N, K, qa.data_ptr(), qw.data_ptr(), sa.data_ptr(), sw.data_ptr(),
         b.data_ptr() if b is not None else None, f.data_ptr(), g.data_ptr(), g_pmax.data_ptr(), _st(),
         kernel="auto", flops=2.0 * M * N * K, nbytes=float(M * K + N * K + 4 * M * N),
         tag=f"vit gemm_fp8_gelu {M}x{N}x{K}")
    return f, g


# ------------------------------------------------------------------ modules
class _LNFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x2 = x.contiguous().view(-1, x.shape[-1])
        ctx.save_for_backward(x2, weight)
        ctx.eps, ctx.shape = eps, x.shape
        return _ln(x2, weight, bias, eps).view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dw = torch.zeros(weight.shape, dtype=torch.float32, device=x2.device)
        db = torch.zeros_like(dw)
        dy2 = dy.contiguous().view(-1, x2.shape[1]).to(x2.dtype)
        dx = _ln_bwd(x2, weight, dy2, ctx.eps, None, dw, db)
        return dx.view(ctx.shape), dw, db, None


class LayerNorm(nn.LayerNorm):
    """fp32-computing LayerNorm (models.py:382-388) -> artsbir_layernorm_fwd / _bwd"""

    def forward(self, x: torch.Tensor):
        _dt(x)
        return _LNFunction.apply(x, self.weight, self.bias, self.eps)


class _GELUFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        call("artsbir_quickgelu", _dt(x), x.data_ptr(), x.numel(), y.data_ptr(), _st())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        dx = torch.empty_like(x)
        call("artsbir_quickgelu_bwd", _dt(x), x.data_ptr(), dy.data_ptr(), x.numel(), dx.data_ptr(), _st())
        return dx


class QuickGELU(nn.Module):
    """x * sigmoid(1.702 x) (models.py:391-393) -> artsbir_quickgelu / _bwd"""

    def forward(self, x: torch.Tensor):
        return _GELUFunction.apply(x)


def _block_params(blk):
    return (blk.attn.in_proj_weight, blk.attn.in_proj_bias, blk.attn.out_proj.weight, blk.attn.out_proj.bias,
            blk.ln_1.weight, blk.ln_1.bias, blk.mlp.c_fc.weight, blk.mlp.c_fc.bias, blk.mlp.c_proj.weight,
            blk.mlp.c_proj.bias, blk.ln_2.weight, blk.ln_2.bias)


class _BlockFunction(torch.autograd.Function):
    """one ResidualAttentionBlock: x [L, N, E] -> x + attn(ln_1 x) + mlp(ln_2 .)"""

    @staticmethod
    def forward(ctx, x, blk, fp8, *params):
        (w_in, b_in, w_o, b_o, g1, be1, w_fc, b_fc, w_pr, b_pr, g2, be2) = params
        L, N, E = x.shape
        heads = blk.attn.num_heads
        if E != heads * 64:
            raise RuntimeError(f"transformer block: head_dim must be 64 (E={E}, heads={heads})")
        T = x.dtype
        M = L * N
        x2 = x.contiguous().view(M, E)
        eps1, eps2 = blk.ln_1.eps, blk.ln_2.eps
        # fp8: every quantised activation's producer folds its amax on the way (pm*)
        pm = [_pmax(x.device) for _ in range(4)] if fp8 else [None] * 4
        h = _ln(x2, g1, be1, eps1, pm[0])
        bi = b_in.detach().float().contiguous()
        qkv = (_gemm_fp8(h, w_in, b_in, out_dtype=T, a_pmax=pm[0]) if fp8
               else _gemm(h, _as(w_in, T), M, 3 * E, E, bias=bi))
        att = torch.empty(M, E, dtype=T, device=x.device)
        lse = torch.empty(M * heads, dtype=torch.float32, device=x.device)
        mask = blk._mask(x)
        if fp8:
            call("artsbir_mha_fwd_lse_pmax", _dt(x), qkv.data_ptr(), L, N, heads,
                 mask.data_ptr() if mask is not None else None, att.data_ptr(), lse.data_ptr(), pm[1].data_ptr(),
                 _st(), kernel="attn_fwd_kernel", flops=4.0 * N * heads * L * L * 64,
                 nbytes=float(qkv.element_size() * M * 4 * E), tag=f"vit attn fwd L{L} N{N}")
        else:
            call("artsbir_mha_fwd_lse", _dt(x), qkv.data_ptr(), L, N, heads,
                 mask.data_ptr() if mask is not None else None, att.data_ptr(), lse.data_ptr(), _st())
        if fp8:  # x1 = x + out_proj(att) (f32 residual stream) and its bf16 copy, in the GEMM epilogue
            x1 = torch.empty(M, E, dtype=torch.float32, device=x.device)
            x1t = torch.empty(M, E, dtype=T, device=x.device)
            _gemm_fp8(att, w_o, b_o, out=x1, a_pmax=pm[1], accumulate=False, res=x2, out2=x1t)
        else:
            x1 = x2.float().clone() if T == torch.float32 else _cast(x2, torch.float32)  # the f32 residual stream
            _gemm(att, _as(w_o, T), M, E, E, bias=b_o.detach().float().contiguous(), out=x1)
            x1t = x1.clone() if T == torch.float32 else _cast(x1, T)  # LN2's input (x1 goes on accumulating)
        h2 = _ln(x1t, g2, be2, eps2, pm[2])
        if fp8 and T == torch.bfloat16:  # c_fc and QuickGELU in one GEMM epilogue
            f, a = _gemm_fp8_gelu(h2, w_fc, b_fc, pm[2], pm[3])
        else:
            if fp8:
                f = _gemm_fp8(h2, w_fc, b_fc, out_dtype=T, a_pmax=pm[2])
            else:
                f = _gemm(h2, _as(w_fc, T), M, 4 * E, E, bias=b_fc.detach().float().contiguous())
            a = torch.empty_like(f)
            if fp8:
                call("artsbir_quickgelu_pmax", _dt(f), f.data_ptr(), f.numel(), a.data_ptr(), pm[3].data_ptr(),
                     _st())
            else:
                call("artsbir_quickgelu", _dt(f), f.data_ptr(), f.numel(), a.data_ptr(), _st())
        if fp8:  # y = x1 + c_proj(a), written once in bf16 by the GEMM epilogue
            y = torch.empty(M, E, dtype=T, device=x.device)
            _gemm_fp8(a, w_pr, b_pr, out=x1, a_pmax=pm[3], accumulate=True, out2=y, skip_c=True)
        else:
            _gemm(a, _as(w_pr, T), M, E, 4 * E, bias=b_pr.detach().float().contiguous(), out=x1)
            y = x1 if T == torch.float32 else _cast(x1, T)
        ctx.save_for_backward(x2, h, qkv, att, lse, x1t, h2, f, a)
        ctx.blk, ctx.mask, ctx.dims = blk, mask, (L, N, E, heads)
        return y.view(L, N, E)

    @staticmethod
    def backward(ctx, dy):
        x2, h, qkv, att, lse, x1t, h2, f, a = ctx.saved_tensors
        blk = ctx.blk
        L, N, E, heads = ctx.dims
        M = L * N
        T = x2.dtype
        dev = x2.device
        (w_in, b_in, w_o, b_o, g1, be1, w_fc, b_fc, w_pr, b_pr, g2, be2) = _block_params(blk)
        # the twelve parameter gradients as views of one zero-filled buffer (one fill)
        ps = (w_in, b_in, w_o, b_o, g1, be1, w_fc, b_fc, w_pr, b_pr, g2, be2)
        flat = torch.zeros(sum(p.numel() for p in ps), dtype=torch.float32, device=dev)
        views, o = [], 0
        for p in ps:
            views.append(flat[o:o + p.numel()].view(p.shape))
            o += p.numel()
        dw_in, db_in, dw_o, db_o, dg1, dbe1, dw_fc, db_fc, dw_pr, db_pr, dg2, dbe2 = views
        dy2 = dy.contiguous().view(M, E).to(T)
        # mlp: y = x1 + c_proj(gelu(c_fc(ln_2(x1))))
        _wgrad(dy2, a, dw_pr)
        df = torch.empty_like(f)
        if T == torch.bfloat16:
            # c_proj input gradient gated by QuickGELU's derivative in the GEMM epilogue,
            # the c_fc bias gradient as its column sums (per-slot partials, then summed)
            slots = torch.zeros(_hip.NSLOT, 2, 4 * E, dtype=torch.float32, device=dev)
            call("artsbir_gemm_nt_gate", M, 4 * E, E, dy2.data_ptr(), E, _t(w_pr, T).data_ptr(), df.data_ptr(),
                 4 * E, f.data_ptr(), slots.data_ptr(), _st(), kernel="auto", flops=2.0 * M * 4 * E * E,
                 nbytes=float(2 * (M * E + 4 * E * E + 2 * M * 4 * E)), tag=f"vit gemm_gate {M}x{4 * E}x{E}")
            call("artsbir_colsum", _hip.DT_F32, slots.data_ptr(), _hip.NSLOT, 8 * E, 4 * E, db_fc.data_ptr(), _st())
        else:
            da = _gemm(dy2, _t(w_pr, T), M, 4 * E, E)
            # QuickGELU backward with the c_fc bias gradient (column sums of df) in the same pass
            call("artsbir_quickgelu_bwd_sum", _dt(f), f.data_ptr(), da.data_ptr(), M, 4 * E, df.data_ptr(),
                 db_fc.data_ptr(), _st())
        _wgrad(df, h2, dw_fc)
        dh2 = _gemm(df, _t(w_fc, T), M, E, 4 * E)
        # LayerNorm-2 backward + the residual gradient dy2; its pass also sums the
        # c_proj bias gradient (columns of dy2) and the out_proj one (columns of dx1)
        dx1 = _ln_bwd(x1t, g2, dh2, blk.ln_2.eps, dy2, dg2, dbe2, dres_sum=db_pr, dx_sum=db_o)
        # attention: x1 = x + out_proj(mha(in_proj(ln_1(x))))
        _wgrad(dx1, att, dw_o)
        datt = _gemm(dx1, _t(w_o, T), M, E, E)
        dqkv = torch.empty_like(qkv)
        dsc = torch.empty(M * heads, dtype=torch.float32, device=dev)
        mask = ctx.mask
        call("artsbir_mha_bwd", _dt(qkv), qkv.data_ptr(), att.data_ptr(), datt.data_ptr(), lse.data_ptr(), L, N,
             heads, mask.data_ptr() if mask is not None else None, dqkv.data_ptr(), dsc.data_ptr(), _st(),
             kernel="attn_bwd_kernels", flops=10.0 * N * heads * L * L * 64,
             nbytes=float(qkv.element_size() * M * 8 * E), tag=f"vit attn bwd L{L} N{N}")
        _wgrad(dqkv, h, dw_in)
        _colsum(dqkv, db_in)
        dh = _gemm(dqkv, _t(w_in, T), M, E, 3 * E)
        dx = _ln_bwd(x2, g1, dh, blk.ln_1.eps, dx1, dg1, dbe1)
        return (dx.view(L, N, E), None, None, dw_in, db_in, dw_o, db_o, dg1, dbe1, dw_fc, db_fc, dw_pr, db_pr,
                dg2, dbe2)


class ResidualAttentionBlock(nn.Module):
    """models.py:396-417 on libartsbir_hip, forward and backward (one autograd
    node).  Sequence-first x [L, N, E] as nn.MultiheadAttention; head_dim 64."""

    def __init__(self, d_model: int, n_head: int, attn_mask: torch.Tensor = None):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 4)),
            ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 4, d_model))]))
        self.ln_2 = LayerNorm(d_model)
        self.attn_mask = attn_mask
        self.fp8 = False

    def _mask(self, x):
        if self.attn_mask is None:
            return None
        m = self.attn_mask.to(device=x.device)
        if m.dtype == torch.bool:  # True = not allowed (nn.MultiheadAttention)
            m = torch.zeros(m.shape, device=x.device).masked_fill(m, float("-inf"))
        return m.to(x.dtype).float().contiguous()  # the reference casts the mask to x.dtype

    def forward(self, x):
        _dt(x)
        return _BlockFunction.apply(x, self, self.fp8, *_block_params(self))


class Transformer(nn.Module):
    """CLIP's Transformer: resblocks 0 .. layers-1"""

    def __init__(self, width: int, layers: int, heads: int, attn_mask: torch.Tensor = None):
        super().__init__()
        self.width, self.layers = width, layers
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, attn_mask) for _ in range(layers)])

    def forward(self, x):
        return self.resblocks(x)


class _PatchFunction(torch.autograd.Function):
    """conv1 (patch x patch, stride patch, no bias) as patchify + GEMM: [B,3,R,R] -> [B*P, E]"""

    @staticmethod
    def forward(ctx, img, weight, dtype, patch, more=()):
        """img, then any further image batches of the same shape (the other
        branches of forward_branches): their patch rows follow in one buffer,
        so the branches are never concatenated as images"""
        imgs = (img,) + tuple(more)
        Bi, _, R, _ = img.shape
        B = Bi * len(imgs)
        E = weight.shape[0]
        K = 3 * patch * patch
        P = (R // patch) ** 2
        rows = torch.empty(B * P, K, dtype=dtype, device=img.device)
        for i, im in enumerate(imgs):
            if im.shape != img.shape:
                raise ValueError(f"branch {i}: image batch {tuple(im.shape)} != {tuple(img.shape)}")
            call("artsbir_vit_patchify", _hip.dtype_code(dtype), im.contiguous().float().data_ptr(), Bi, R, patch,
                 rows[i * Bi * P:].data_ptr(), _st())
        out = _gemm(rows, _as(weight.view(E, K), dtype), B * P, E, K)
        ctx.save_for_backward(rows)
        ctx.wshape = weight.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        rows, = ctx.saved_tensors
        dw = torch.zeros(ctx.wshape, dtype=torch.float32, device=rows.device)
        _wgrad(dout.contiguous().to(rows.dtype), rows, dw.view(ctx.wshape[0], -1))
        return None, dw, None, None, None


class _TokensFunction(torch.autograd.Function):
    """[B*P, E] patch embeddings -> tokens [P+1, B, E]: class embedding first, + positional embedding"""

    @staticmethod
    def forward(ctx, patches, cls, pos, B):
        P = patches.shape[0] // B
        E = patches.shape[1]
        out = torch.empty(P + 1, B, E, dtype=patches.dtype, device=patches.device)
        call("artsbir_vit_tokens", _dt(patches), patches.data_ptr(), cls.detach().float().contiguous().data_ptr(),
             pos.detach().float().contiguous().data_ptr(), B, P, E, out.data_ptr(), _st())
        ctx.dims, ctx.dtype = (B, P, E), patches.dtype
        return out

    @staticmethod
    def backward(ctx, dtok):
        B, P, E = ctx.dims
        dtok = dtok.contiguous().to(ctx.dtype)
        dpatch = torch.empty(B * P, E, dtype=ctx.dtype, device=dtok.device)
        dcls = torch.zeros(E, dtype=torch.float32, device=dtok.device)
        dpos = torch.zeros(P + 1, E, dtype=torch.float32, device=dtok.device)
        call("artsbir_vit_tokens_bwd", _dt(dtok), dtok.data_ptr(), B, P, E, dpatch.data_ptr(), dcls.data_ptr(),
             dpos.data_ptr(), _st())
        return dpatch, dcls, dpos, None


class _ClassTokenFunction(torch.autograd.Function):
    """x[0] of the sequence-first tokens (rows 0 .. B-1, contiguous)"""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.contiguous()[0].clone()

    @staticmethod
    def backward(ctx, g):
        dx = torch.zeros(ctx.shape, dtype=g.dtype, device=g.device)
        dx[0].copy_(g)
        return dx


class _ProjFunction(torch.autograd.Function):
    """x [B, E] @ proj [E, D] -> f32 [B, D]"""

    @staticmethod
    def forward(ctx, x, proj):
        B, E = x.shape
        D = proj.shape[1]
        out = _gemm(x.contiguous(), _t(proj, x.dtype), B, D, E, out_f32=True)
        ctx.save_for_backward(x, proj)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, proj = ctx.saved_tensors
        B, E = x.shape
        D = proj.shape[1]
        g = dout.contiguous().to(x.dtype)
        dx = _gemm(g, _as(proj, x.dtype), B, E, D)
        dproj = torch.zeros(E, D, dtype=torch.float32, device=x.device)
        _wgrad(x.contiguous(), g, dproj)
        return dx, dproj


class VisionTransformer(nn.Module):
    """CLIP's ViT image encoder (ViT-B/16: input_resolution 224, patch_size 16,
    width 768, layers 12, heads 12): [B, 3, R, R] -> [B, output_dim] f32"""

    def __init__(self, input_resolution: int = 224, patch_size: int = 16, width: int = 768, layers: int = 12,
                 heads: int = 12, output_dim: int = 768):
        super().__init__()
        self.input_resolution, self.patch_size, self.output_dim = input_resolution, patch_size, output_dim
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn((input_resolution // patch_size) ** 2 + 1,
                                                                     width))
        self.ln_pre = LayerNorm(width)
        self.transformer = Transformer(width, layers, heads)
        self.ln_post = LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))
        self.compute_dtype = torch.float32
        self.trained_layers = []
        import models  # the encoder's image transform (models.py:289-295); imported late (models imports vit)
        self.transform = models.ClipTransform(input_resolution)

    def freeze_layers(self):
        self.trained_layers.append('all')

    def forward(self, x, more=()):
        fp8 = self.compute_dtype == "fp8"
        dtype = torch.bfloat16 if fp8 else self.compute_dtype
        for blk in self.transformer.resblocks:
            blk.fp8 = fp8
        B = x.shape[0] * (1 + len(more))
        t = _PatchFunction.apply(x, self.conv1.weight, dtype, self.patch_size, tuple(more))
        t = _TokensFunction.apply(t, self.class_embedding, self.positional_embedding, B)
        t = self.ln_pre(t)
        t = self.transformer(t)
        c = self.ln_post(_ClassTokenFunction.apply(t))
        return _ProjFunction.apply(c, self.proj)

    def forward_branches(self, xs):
        """the three branch calls of train.py:28-30 (no BatchNorm here: one batched call is exact)"""
        xs = list(xs)
        if all(x.shape == xs[0].shape for x in xs):
            out = self.forward(xs[0], tuple(xs[1:]))
        else:
            out = self.forward(torch.cat(xs))
        return list(out.chunk(len(xs)))
