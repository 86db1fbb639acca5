#!/usr/bin/env python3
"""Times the ViT-B/16 attention core at the C5 bench shape (L = 197 tokens,
N = 1536 sequences = 512 triplets x 3, 12 heads of 64; bf16): artsbir_mha_fwd_lse
and artsbir_mha_bwd, one JSON line.  ARTSBIR_ATTN_BWD2=1 selects the two-kernel
backward (read once per process).  --dump PATH saves dqkv of the first backward
so that two runs (one per form) can be compared bit for bit with --compare."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=197)
    ap.add_argument("--N", type=int, default=1536)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dump", default=None)
    ap.add_argument("--compare", nargs=2, default=None)
    a = ap.parse_args()
    if a.compare:
        x, y = (torch.load(p, weights_only=True) for p in a.compare)
        print(json.dumps({"bit_identical": bool(torch.equal(x, y)),
                          "max_abs_diff": float((x.float() - y.float()).abs().max())}))
        return
    dev = torch.device("cuda:0")
    L, N, H = a.L, a.N, a.heads
    E = 64 * H
    g = torch.Generator(device=dev).manual_seed(3)
    qkv = torch.randn(L * N, 3 * E, device=dev, generator=g).bfloat16()
    dout = torch.randn(L * N, E, device=dev, generator=g).bfloat16()
    out = torch.empty(L * N, E, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(L * N * H, device=dev)
    dq = torch.empty_like(qkv)
    dsc = torch.empty(L * N * H, device=dev)
    st = _hip.stream()

    def fwd():
        _hip.call("artsbir_mha_fwd_lse", _hip.DT_BF16, qkv.data_ptr(), L, N, H, None, out.data_ptr(), lse.data_ptr(),
                  st)

    def bwd():
        _hip.call("artsbir_mha_bwd", _hip.DT_BF16, qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), L,
                  N, H, None, dq.data_ptr(), dsc.data_ptr(), st)

    fwd()
    bwd()
    torch.cuda.synchronize()
    if a.dump:
        torch.save(dq.cpu(), a.dump)
    res = {}
    for name, fn, fl in (("fwd", fwd, 4.0), ("bwd", bwd, 10.0)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        res[name + "_ms"] = round(ms, 4)
        res[name + "_tflops"] = round(fl * N * H * L * L * 64 / ms / 1e9, 1)
    res.update({"L": L, "N": N, "heads": H, "bwd_form": "two-kernel" if os.environ.get("ARTSBIR_ATTN_BWD2") == "1"
                else "fused"})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
