"""Losses and distances of the training step on libartsbir_hip.

  TripletMarginLoss            nn.TripletMarginLoss(margin=utils.MARGIN) (train.py:169): p=2,
                               eps=1e-6 added to the difference (torch.pairwise_distance),
                               swap=False, mean of clamp_min(margin + d(a,p) - d(a,n), 0)
  TripletMarginWithDistanceLoss  nn.TripletMarginWithDistanceLoss (train.py:175, utils.py:56,69)
                               for the two distance functions of the reference:
                               utils.euclidean_distance and utils.cosine_distance
  CrossEntropyLoss             nn.CrossEntropyLoss() (utils.py:57,70), mean, ignore_index=-100
  cosine_distance              1 - CosineSimilarity(dim=1, eps=1e-8)  (utils.py:31-40)
All run on the GPU kernels with explicit backward kernels.
"""
from __future__ import annotations

import torch
from torch import nn

import _hip
from _hip import call, ptr


def _s():
    return _hip.stream()


def _cuda(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("libartsbir_hip losses need CUDA tensors")


class _TripletFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, p, n, margin, eps):
        _cuda(a, p, n)
        a, p, n = (t.contiguous().float() for t in (a, p, n))
        B, D = a.shape
        dist = torch.empty(2 * B, dtype=torch.float32, device=a.device)
        loss = torch.empty((), dtype=torch.float32, device=a.device)
        call("artsbir_triplet_fwd", ptr(a), ptr(p), ptr(n), B, D, margin, eps, ptr(dist), ptr(loss), _s())
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
             ptr(da), ptr(dp), ptr(dn), _s())
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


# ------------------------------------------------------------ distances
class _PairwiseL2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x1, x2, eps):
        _cuda(x1, x2)
        a = x1.contiguous().float().reshape(-1, x1.shape[-1])
        b = x2.contiguous().float().reshape(-1, x2.shape[-1])
        n = max(a.shape[0], b.shape[0])
        out = torch.empty(n, dtype=torch.float32, device=a.device)
        call("artsbir_pairwise_l2", ptr(a), a.shape[0], ptr(b), b.shape[0], a.shape[1], eps, ptr(out), _s())
        ctx.save_for_backward(a, b, out)
        ctx.eps, ctx.shapes = eps, (x1.shape, x2.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b, out = ctx.saved_tensors
        g = g.contiguous().float()
        d1 = torch.zeros_like(a) if ctx.needs_input_grad[0] else None
        d2 = torch.zeros_like(b) if ctx.needs_input_grad[1] else None
        call("artsbir_pairwise_l2_bwd", ptr(a), a.shape[0], ptr(b), b.shape[0], a.shape[1], ctx.eps, ptr(out), ptr(g),
             ptr(d1), ptr(d2), _s())
        return (d1.view(ctx.shapes[0]) if d1 is not None else None,
                d2.view(ctx.shapes[1]) if d2 is not None else None, None)


def pairwise_l2_autograd(x1, x2, eps=1e-6):
    return _PairwiseL2Fn.apply(x1, x2, float(eps))


class _CosineFn(torch.autograd.Function):
    """cos = (x1/max|x1|,eps) . (x2/max|x2|,eps); returns 1 - cos (the reference's CosineLoss)."""

    @staticmethod
    def forward(ctx, x1, x2, eps):
        _cuda(x1, x2)
        a = x1.contiguous().float()
        b = x2.contiguous().float()
        n = max(a.shape[0], b.shape[0])
        cosv = torch.empty(n, dtype=torch.float32, device=a.device)
        norms = torch.empty(2 * n, dtype=torch.float32, device=a.device)
        call("artsbir_cosine_fwd", ptr(a), a.shape[0], ptr(b), b.shape[0], a.shape[1], eps, ptr(cosv), ptr(norms),
             _s())
        ctx.save_for_backward(a, b, cosv, norms)
        return 1.0 - cosv

    @staticmethod
    def backward(ctx, g):
        a, b, cosv, norms = ctx.saved_tensors
        gcos = (-g).contiguous().float()
        d1 = torch.zeros_like(a) if ctx.needs_input_grad[0] else None
        d2 = torch.zeros_like(b) if ctx.needs_input_grad[1] else None
        call("artsbir_cosine_bwd", ptr(a), a.shape[0], ptr(b), b.shape[0], a.shape[1], ptr(cosv), ptr(norms),
             ptr(gcos), ptr(d1), ptr(d2), _s())
        return d1, d2, None


def cosine_distance(x1, x2, eps=1e-8):
    return _CosineFn.apply(x1, x2, float(eps))


class _HingeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dp, dn, margin):
        dp, dn = dp.contiguous().float(), dn.contiguous().float()
        loss = torch.empty((), dtype=torch.float32, device=dp.device)
        call("artsbir_hinge_fwd", ptr(dp), ptr(dn), dp.numel(), margin, ptr(loss), _s())
        ctx.save_for_backward(dp, dn)
        ctx.margin = margin
        return loss

    @staticmethod
    def backward(ctx, g):
        dp, dn = ctx.saved_tensors
        gdp, gdn = torch.empty_like(dp), torch.empty_like(dn)
        call("artsbir_hinge_bwd", ptr(dp), ptr(dn), dp.numel(), ctx.margin, ptr(g.contiguous().float()), ptr(gdp),
             ptr(gdn), _s())
        return gdp, gdn, None


class TripletMarginWithDistanceLoss(nn.Module):
    """mean(clamp_min(margin + d(a,p) - d(a,n), 0)), swap=False, for d in
    {utils.euclidean_distance (fused triplet kernel), utils.cosine_distance}."""

    def __init__(self, distance_function=None, margin: float = 1.0, swap: bool = False, reduction: str = "mean"):
        super().__init__()
        if swap or reduction != "mean":
            raise NotImplementedError("only swap=False, reduction='mean' (the reference's configuration)")
        self.distance_function = distance_function
        self.margin, self.swap, self.reduction = margin, swap, reduction

    def forward(self, anchor, positive, negative):
        f = self.distance_function
        if f is None or getattr(f, "p", None) == 2.0:  # euclidean (PairwiseDistance) -> fused kernel
            return _TripletFn.apply(anchor, positive, negative, float(self.margin), float(getattr(f, "eps", 1e-6)))
        dp = f(anchor, positive)
        dn = f(anchor, negative)
        return _HingeFn.apply(dp, dn, float(self.margin))


# ------------------------------------------------------------ cross entropy
class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        _cuda(logits, labels)
        x = logits.contiguous().float()
        lab = labels.contiguous().to(torch.int64)
        B, C = x.shape
        prob = torch.empty_like(x)
        loss2 = torch.empty(2, dtype=torch.float32, device=x.device)
        call("artsbir_cross_entropy_fwd", ptr(x), ptr(lab), B, C, ignore_index, ptr(prob), ptr(loss2), _s())
        ctx.save_for_backward(prob, lab, loss2)
        ctx.ignore_index = ignore_index
        return loss2[0].clone()

    @staticmethod
    def backward(ctx, g):
        prob, lab, loss2 = ctx.saved_tensors
        B, C = prob.shape
        d = torch.empty_like(prob)
        call("artsbir_cross_entropy_bwd", ptr(prob), ptr(lab), B, C, ctx.ignore_index, ptr(g.contiguous().float()),
             ptr(loss2), ptr(d), _s())
        return d, None, None


class CrossEntropyLoss(nn.Module):
    def __init__(self, ignore_index: int = -100, reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("only reduction='mean' (the reference's configuration)")
        self.ignore_index, self.reduction = ignore_index, reduction

    def forward(self, logits, labels):
        return _CEFn.apply(logits, labels, int(self.ignore_index))
