#!/usr/bin/env python3
"""Retrieval leg of bench.py alone (1M x 512 gallery, 10k queries, top-10 + rank),
once per scan kernel: `python tools/retr_bench.py [v1|auto ...]`."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import knn  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    orig = knn.knn
    for scan in (sys.argv[1:] or ["auto", "v1"]):
        sc = scan.split("+")[0].split("-")[0]  # e.g. auto, v1, auto-noshare, auto+prepass
        knn.knn = (lambda *a, _s=sc, _p=(8192 if "+prepass" in scan else 0), _b=("-noshare" not in scan), **kw:
                   orig(*a, scan=_s, prepass_rows=_p, share_bound=_b, **kw))
        r = bench.retrieval_leg(dev, 0, 1)
        r["scan"] = scan
        print(json.dumps(r), flush=True)
