#!/usr/bin/env python3
"""Retrieval leg of bench.py alone (1M x 512 gallery, 10k queries, top-10 + rank),
once per gallery chunk size: `python tools/retr_bench.py [tiles_per_chunk ...]`
(0 = the library's default)."""
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
    for tpc in (sys.argv[1:] or ["0"]):
        knn.knn = (lambda *a, _t=int(tpc), **kw: orig(*a, tiles_per_chunk=_t, **kw))
        r = bench.retrieval_leg(dev, 0, 1)
        r["tiles_per_chunk"] = int(tpc)
        print(json.dumps(r), flush=True)
