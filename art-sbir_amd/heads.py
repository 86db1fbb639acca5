"""Classification heads of ModifiedResNet_with_classification (models.py:363-379).

``classifier`` / ``classifier2`` are nn.Linear(output_dim, num_classes) on the
f32 embedding; forward and backward run on the small f32 kernels of heads.hip
(a [B, D] x [C, D]^T product with C <= a few hundred classes).
"""
from __future__ import annotations

import torch

import _hip
from _hip import call, ptr


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        if not x.is_cuda:
            raise RuntimeError("classification heads on libartsbir_hip need CUDA tensors")
        xf = x.contiguous().float()
        w = weight.detach().contiguous().float()
        B, D = xf.shape
        C = w.shape[0]
        y = torch.empty(B, C, dtype=torch.float32, device=x.device)
        call("artsbir_linear_fwd", ptr(xf), ptr(w), ptr(bias.detach()) if bias is not None else None, B, D, C, ptr(y),
             _hip.stream())
        ctx.save_for_backward(xf, w)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xf, w = ctx.saved_tensors
        B, D = xf.shape
        C = w.shape[0]
        dy = dy.contiguous().float()
        dx = torch.empty_like(xf) if ctx.needs_input_grad[0] else None
        dw = torch.zeros_like(w) if ctx.needs_input_grad[1] else None
        db = torch.zeros(C, dtype=torch.float32, device=dy.device) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        call("artsbir_linear_bwd", ptr(dy), ptr(xf), ptr(w), B, D, C, ptr(dx), ptr(dw), ptr(db), _hip.stream())
        return dx, dw, db


def linear(x, weight, bias):
    return _LinearFn.apply(x, weight, bias)
