"""Times the four fp8 projection GEMMs of the C5 ViT block forward at the
bench's token count (artsbir_gemm_nt_fp8_ex), one line per shape.
ARTSBIR_FP8_CFG / ARTSBIR_FP8_NOSTORE select the kernel variant (read once
per process)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=302592)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, E = a.tokens, 768
    torch.manual_seed(0)
    shapes = [("qkv", 2304, 768, torch.bfloat16, {}),
              ("out_proj", 768, 768, torch.float32, {"res": True, "out2": True}),
              ("c_fc", 3072, 768, torch.bfloat16, {}),
              ("c_proj", 768, 3072, torch.float32, {"acc": True, "out2": True, "skip": True})]
    tot = 0.0
    for name, N, K, odt, f in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device=dev)
        out = torch.randn(M, N, device=dev, dtype=odt)
        res = torch.randn(M, N, device=dev, dtype=torch.bfloat16) if f.get("res") else None
        out2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if f.get("out2") else None
        qa, sa = vit._fp8(x)
        qw, sw = vit._fp8(w)
        bb = b.float().contiguous()
        st = torch.cuda.current_stream().cuda_stream

        def run():
            vit.call("artsbir_gemm_nt_fp8_ex", M, N, K, qa.data_ptr(), qw.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                     bb.data_ptr(), out.data_ptr(), vit._hip.dtype_code(odt), 1 if f.get("acc") else 0,
                     res.data_ptr() if res is not None else None, out2.data_ptr() if out2 is not None else None,
                     1 if f.get("skip") else 0, st)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tot += ms
        tf = 2.0 * M * N * K / ms / 1e9
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "ms": round(ms, 4), "TFLOPs": round(tf, 1),
                          "cfg": os.environ.get("ARTSBIR_FP8_CFG", "0"),
                          "nostore": os.environ.get("ARTSBIR_FP8_NOSTORE", "0")}), flush=True)
        del x, w, out, res, out2, qa, qw
    print(json.dumps({"total_ms": round(tot, 3)}), flush=True)


if __name__ == "__main__":
    main()
