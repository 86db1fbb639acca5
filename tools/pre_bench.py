#!/usr/bin/env python3
"""bench.py's GPU input-transform leg alone (optionally with its CPU baseline)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    out = bench.preprocess_leg(dev, 0, 1)
    if "--cpu" in sys.argv:
        out["cpu_baseline"] = bench.cpu_preprocess_baseline()
    print(json.dumps(out))
