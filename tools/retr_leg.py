#!/usr/bin/env python3
"""bench.py's C4 retrieval leg alone (noise 0.5 and 3.0): QPS, scan kernel time, mAP@10."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    import ctypes
    import _hip
    dev = torch.device("cuda:0")
    st = (ctypes.c_ulonglong * 4)()
    for noise in (0.5, 3.0):
        _hip.lib().artsbir_knn_stat_read(st, 1)
        r = bench.retrieval_leg(dev, 0, 1, reps=3, noise=noise)
        _hip.lib().artsbir_knn_stat_read(st, 1)
        print(json.dumps({"noise": noise, "qps": r["value"], "ms": r["ms"], "map@10": r["map@10"],
                          "scan_us": r["roofline"]["avg_launch_us"], "scan_frac": r["roofline"]["frac"],
                          "kb": os.environ.get("ARTSBIR_KNN_KB", "1"),
                          "wave_tiles": st[0], "entries": st[1], "insertions": st[2], "merge_live_per_query": round(st[3] / (4 * 10_000), 2),
                          "entry_frac": round(st[1] / max(st[0], 1), 4)}), flush=True)
