"""Triplet-margin loss on libartsbir_hip.

Replaces nn.TripletMarginLoss(margin=utils.MARGIN) (train.py:169): p=2,
eps=1e-6 added to the difference (torch.pairwise_distance), swap=False,
reduction='mean', clamp_min(margin + d(a,p) - d(a,n), 0).
"""
from __future__ import annotations

import torch
from torch import nn

import _hip
from _hip import call, ptr


class _TripletFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, p, n, margin, eps):
        if not a.is_cuda:
            raise RuntimeError("TripletMarginLoss on libartsbir_hip needs CUDA tensors")
        a, p, n = (t.contiguous().float() for t in (a, p, n))
        B, D = a.shape
        dist = torch.empty(2 * B, dtype=torch.float32, device=a.device)
        loss = torch.empty((), dtype=torch.float32, device=a.device)
        call("artsbir_triplet_fwd", ptr(a), ptr(p), ptr(n), B, D, margin, eps, ptr(dist), ptr(loss), _hip.stream())
        ctx.save_for_backward(a, p, n, dist)
        ctx.margin, ctx.eps = margin, eps
        return loss

    @staticmethod
    def backward(ctx, gout):
        a, p, n, dist = ctx.saved_tensors
        B, D = a.shape
        gout = gout.contiguous().float()
        da, dp, dn = (torch.empty_like(a) for _ in range(3))
        call("artsbir_triplet_bwd", ptr(a), ptr(p), ptr(n), B, D, ctx.margin, ctx.eps, ptr(dist), ptr(gout),
             ptr(da), ptr(dp), ptr(dn), _hip.stream())
        return da, dp, dn, None, None


class TripletMarginLoss(nn.Module):
    """Drop-in for nn.TripletMarginLoss(margin) with p=2, eps=1e-6, swap=False, mean."""

    def __init__(self, margin: float = 1.0, p: float = 2.0, eps: float = 1e-6, swap: bool = False,
                 reduction: str = "mean"):
        super().__init__()
        if p != 2.0 or swap or reduction != "mean":
            raise NotImplementedError("only p=2, swap=False, reduction='mean' (the reference's configuration)")
        self.margin, self.p, self.eps, self.swap, self.reduction = margin, p, eps, swap, reduction

    def forward(self, anchor, positive, negative):
        return _TripletFn.apply(anchor, positive, negative, float(self.margin), float(self.eps))
