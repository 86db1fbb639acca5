"""Adam on libartsbir_hip: one kernel launch updates every parameter tensor.

Drop-in for torch.optim.Adam(params, lr, weight_decay) as used at train.py:158:
coupled L2 (grad += weight_decay*param), betas (0.9, 0.999), eps 1e-8, no
amsgrad, bias corrections 1-beta^step; same per-parameter state keys
(``step``, ``exp_avg``, ``exp_avg_sq``) so optimizer state_dicts interchange.
"""
from __future__ import annotations

import ctypes

import torch

import _hip
import engine as _engine
from _hip import call

CHUNK = 4096


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference (train.py:158)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self._tables = {}

    def _table(self, group, plist):
        key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                     self.state[p]["exp_avg_sq"].data_ptr()) for p in plist)
        hit = self._tables.get(id(group))
        if hit is not None and hit[0] == key:
            return hit[1]
        recs = (_hip.AdamTensor * len(plist))()
        numels = (ctypes.c_longlong * len(plist))()
        for i, p in enumerate(plist):
            st = self.state[p]
            recs[i] = _hip.AdamTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                      st["exp_avg_sq"].data_ptr(), p.numel())
            numels[i] = p.numel()
        lib = _hip.lib()
        nblocks = lib.artsbir_adam_table_blocks(numels, len(plist), CHUNK)
        host_table = (ctypes.c_longlong * nblocks)()
        lib.artsbir_adam_fill_table(numels, len(plist), CHUNK, host_table)
        dev = plist[0].device
        rec_t = torch.frombuffer(bytearray(recs), dtype=torch.uint8).to(dev)
        tab_t = torch.frombuffer(bytearray(host_table), dtype=torch.int64).to(dev)
        entry = (rec_t, tab_t, nblocks)
        self._tables[id(group)] = (key, entry)
        return entry

    @torch.no_grad()
    def zero_grad(self, set_to_none: bool = True):
        """torch semantics; with set_to_none=False and every gradient a view of
        one flat buffer (the engine's GradBuffer) that holds nothing else, the
        buffer is cleared by ONE fill instead of one launch per parameter"""
        grads = [p.grad for g in self.param_groups for p in g["params"] if p.grad is not None]
        if set_to_none or not grads:
            return super().zero_grad(set_to_none=set_to_none)
        base = grads[0]._base
        if (base is not None and base.is_contiguous() and all(g._base is base for g in grads)
                and sum(g.numel() for g in grads) == base.numel()):
            base.zero_()
            return None
        return super().zero_grad(set_to_none=False)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
            for p in plist:
                if not p.is_cuda:
                    raise RuntimeError("Adam on libartsbir_hip needs CUDA parameters")
                if p.grad.is_sparse:
                    raise RuntimeError("sparse gradients are not supported")
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    p.grad = p.grad.float().contiguous()
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
            step = int(self.state[plist[0]]["step"].item())
            if any(int(self.state[p]["step"].item()) != step for p in plist):
                raise RuntimeError("parameters of one group are at different Adam steps")
            recs, table, nblocks = self._table(group, plist)
            b1, b2 = group["betas"]
            call("artsbir_adam_step", recs.data_ptr(), table.data_ptr(), nblocks, CHUNK, float(group["lr"]),
                 float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), step, _hip.stream())
        _engine.bump_weights_generation()
        return loss
