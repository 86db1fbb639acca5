#!/usr/bin/env python3
"""The fp8 quantiser's pass (artsbir_quantize_fp8_pmax: partial-max reduce +
quantisation) on the C5 activation sizes: the c_fc output (302592 x 3072) and a
768-wide one (302592 x 768), HIP events on the current stream, best of rounds,
with the codes checked equal across runs of the same input."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    st = _hip.stream()
    for rows, cols in ((302592, 3072), (302592, 768)):
        x = (torch.randn(rows, cols, device=dev, generator=g) * 2).bfloat16()
        n = x.numel()
        q = torch.empty(n, dtype=torch.uint8, device=dev)
        sc = torch.empty(1, device=dev)
        amax = float(x.float().abs().max())
        pm = torch.full((4096,), 0, dtype=torch.int32, device=dev)
        pm[0] = torch.tensor([amax], dtype=torch.float32).view(torch.int32)[0]

        def run():
            _hip.call("artsbir_quantize_fp8_pmax", _hip.DT_BF16, x.data_ptr(), n, pm.data_ptr(), 4096, q.data_ptr(),
                      sc.data_ptr(), st)
        run()
        torch.cuda.synchronize()
        ref = q.clone()
        best = 1e30
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 10)
        same = bool(torch.equal(q, ref))
        print(json.dumps({"shape": [rows, cols], "ms": round(best, 4), "GBps": round(3.0 * n / best / 1e6, 1),
                          "codes_stable": same, "lib": os.environ.get("ARTSBIR_LIB", "production")}), flush=True)
        del x, q


if __name__ == "__main__":
    main()
