"""The retrieval order the HIP path reproduces (float64 distances, ties by the lower
gallery index: oracle/retrieval.py) against the reference's own float32
arithmetic (nn.PairwiseDistance + torch.topk on the CPU, inference.py:43-66,
utils.py:42): how many top-10 lists and ranks differ, and whether every
difference is an fp32 tie (equal float32 distances, or within 4 ulp).

Committed counts: tests/golden/fp32_order.json, written by
`python tests/test_fp32_order.py --write`.  Two workloads: the committed golden
fixture (tests/golden/retrieval.npz: 4096 x 64 with exact duplicate rows) and
64 queries of C4's 1M x 512 gallery at noise 3.0 (the sample
tests/test_retrieval_gpu.py checks the kernel on)."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import retrieval as oret  # noqa: E402

ULP_TIE = 4  # float32 ulps at the distance's magnitude that count as a near-tie


def _near(a, b):
    a32, b32 = np.float32(a), np.float32(b)
    return abs(float(a32) - float(b32)) <= ULP_TIE * float(np.spacing(np.float32(max(abs(a32), abs(b32)))))


def compare(name, g, qs, pos, k, f64_idx, f64_rank):
    """fp32 reference order vs the float64 order on one workload -> summary dict"""
    i32, _, r32, d32 = oret.fp32_reference_order(qs, g, pos, k)
    lists, ranks, exact, near, unexplained = 0, 0, 0, 0, []
    for q in range(len(qs)):
        d = d32[q]
        if not np.array_equal(i32[q], f64_idx[q]):
            lists += 1
            for a, b in zip(f64_idx[q], i32[q]):
                if a == b:
                    continue
                if d[a] == d[b]:
                    exact += 1
                elif _near(d[a], d[b]):
                    near += 1
                else:
                    unexplained.append([q, int(a), int(b)])
        p = int(pos[q])
        if p >= 0 and int(r32[q]) != int(f64_rank[q]):
            ranks += 1
            # every item the two orders place on different sides of the positive is an fp32 (near-)tie with it
            lo, hi = sorted((int(r32[q]), int(f64_rank[q])))
            order32 = np.argsort(d, kind="stable")
            for j in order32[lo:hi + 1]:
                if j != p and not (d[j] == d[p] or _near(d[j], d[p])):
                    unexplained.append([q, p, int(j)])
    return {"workload": name, "queries": int(len(qs)), "k": k, "topk_lists_differ": lists,
            "ranks_differ": ranks, "exact_fp32_ties": exact, "near_ties_le_4ulp": near,
            "unexplained": unexplained}


def golden_workload():
    import make_golden
    g, qs, pos = make_golden.golden_gallery()
    gold = np.load(os.path.join(HERE, "golden", "retrieval.npz"), allow_pickle=False)
    ranks = np.where(pos >= 0, gold["ranks"], -1)
    return compare("golden retrieval.npz 4096x64", g, qs, pos, 10, gold["topk_idx"], ranks)


def c4_workload():
    N, D, Q, k = 1_000_000, 512, 64, 10
    g, qs, pos = oret.synthetic_gallery(N, D, Q, noise=3.0)
    ri, _, rr = oret.topk_rank_large(qs, g, pos, k, "euclidean")
    return compare("C4 1Mx512 noise 3.0, 64 queries", g, qs, pos, k, ri, rr)


def _committed():
    with open(os.path.join(HERE, "golden", "fp32_order.json")) as f:
        return {w["workload"]: w for w in json.load(f)}


def _check(res):
    want = _committed()[res["workload"]]
    assert res == want, (res, want)
    assert not res["unexplained"], res["unexplained"]


def test_golden_fixture_fp32_order():
    _check(golden_workload())


@pytest.mark.slow
def test_c4_sample_fp32_order():
    _check(c4_workload())


if __name__ == "__main__":
    if "--write" in sys.argv:
        out = [golden_workload(), c4_workload()]
        with open(os.path.join(HERE, "golden", "fp32_order.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))
