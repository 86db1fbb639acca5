#!/usr/bin/env python3
"""Headline benchmark: the triplet training step of train.py on MI355X.

One step = the reference's train.py:59-70 iteration on a synthetic minibatch
of B triplets per GPU (3 separate encoder forwards for sketch / positive /
negative, nn.TripletMarginLoss(0.2), backward, Adam(lr 1e-5, wd 0.002)), with
ModifiedResNet((3,4,6,3), output_dim=512) at 224x224 in bf16 (BASELINE.json
configs[1]; configs[2] at --gpus 8).  Data-parallel over RCCL when launched
with torch.distributed.run.  Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LAYERS, OUT_DIM, RES, WIDTH, HEADS = (3, 4, 6, 3), 512, 224, 64, 32
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}  # MI355X dense (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md; ~6.3 TB/s measured copy)
# per-launch HBM bytes of each kernel from the committed rocprofv3 PMC passes
# (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; profiles/summarize_pmc.py)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r1_pmc_traffic.json")


def pmc_traffic(kernel):
    try:
        with open(PMC_TRAFFIC) as f:
            k = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None else round(k["hbm_bytes_per_launch"])


def encoder_flops_per_image(layers=LAYERS, out_dim=OUT_DIM, res=RES, width=WIDTH):
    """Algorithmic forward FLOPs of one image (2 x MACs of every conv/linear +
    the attention core), from the models.py:275-360 geometry."""
    f = 0.0
    h = res // 2
    half = width // 2
    f += 2 * h * h * half * 3 * 9 + 2 * h * h * half * half * 9 + 2 * h * h * width * half * 9
    h //= 2
    cin = width
    for i, n in enumerate(layers):
        planes = width * (1 << i)
        for j in range(n):
            s = 2 if (i > 0 and j == 0) else 1
            ho = h // s
            f += 2 * h * h * planes * cin                # conv1 1x1
            f += 2 * h * h * planes * planes * 9         # conv2 3x3
            f += 2 * ho * ho * planes * 4 * planes       # conv3 1x1
            if s > 1 or cin != 4 * planes:
                f += 2 * ho * ho * 4 * planes * cin      # downsample 1x1
            cin, h = 4 * planes, ho
    C = width * 32
    T = h * h + 1
    f += 2 * T * C * 2 * C + 2 * C * C + 2 * C * out_dim  # k|v, q, c_proj
    f += 2 * 2 * T * C                                    # q.k and p.v
    return f


def train_flops_per_triplet():
    """fwd + data-grad + weight-grad ~= 3x forward for every image of the triplet
    (the stem conv1 has no data gradient: x does not require grad)."""
    stem1 = 2 * (RES // 2) ** 2 * (WIDTH // 2) * 3 * 9
    return 3 * (3 * encoder_flops_per_image() - stem1)


def cpu_baseline(batch=32, steps=3):
    """The oracle (torch CPU fp32 restatement of the reference path) on the host
    cores: same model/config, a bounded sample of `batch` triplets per step."""
    from oracle import encoder as oenc, steps as osteps
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    torch.set_num_threads(cores)
    m = osteps.build(LAYERS, OUT_DIM, HEADS, RES, WIDTH)
    opt = osteps.make_optimizer(m)
    loss = osteps.make_loss(0.2)
    el = list(oenc.synthetic_triplet(batch, RES))
    osteps.train_step(m, opt, loss, el)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        osteps.train_step(m, opt, loss, el)
    dt = time.perf_counter() - t0
    return {"value": round(3 * batch * steps / dt, 3), "unit": "triplet-images/s", "cores": cores, "kind": "port",
            "sample": f"oracle/steps.py train_step, ModifiedResNet((3,4,6,3),512) fp32 224^2, {steps} timed steps x "
                      f"{batch} triplets after 1 warm-up, torch CPU {torch.__version__} on {platform.processor() or 'x86_64'}"}


def retrieval_leg(dev, rank, world, N=1_000_000, D=512, Q=10_000, k=10, reps=3):
    """BASELINE metric, second half: gallery kNN QPS at 1M x 512.
    Synthetic gallery G ~ N(0,1); query i = G[(i*7919) mod N] + 0.5 N(0,1), so each
    query has one planted positive.  Timed: knn.knn (or knn_sharded over the
    ranks: gallery rows split, one all_gather + all_reduce) producing the exact
    top-10 and the rank of the positive for all Q queries; inputs resident in HBM."""
    import knn
    g = torch.Generator(device=dev).manual_seed(7)
    lo, hi = rank * N // world, (rank + 1) * N // world
    gal = torch.randn(N, D, device=dev, generator=g)  # same full gallery on every rank (seeded)
    pos = (torch.arange(Q, device=dev, dtype=torch.int64) * 7919) % N
    qs = gal[pos] + 0.5 * torch.randn(Q, D, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
    shard = gal[lo:hi].contiguous()
    del gal

    def run():
        if world > 1:
            return knn.knn_sharded(qs, shard, lo, k, pos)
        idx, dd, r, _ = knn.knn(qs, shard, k, pos)
        return idx, dd, r

    run()  # warm-up
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    prof = []
    import _hip
    _hip.PROFILE = prof
    t0 = time.perf_counter()
    for _ in range(reps):
        idx, dd, r = run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    _hip.PROFILE = None
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    scan_kernel = "knn_scan_v2_kernel" if any(kn == "knn_scan_v2_kernel" for kn, *_ in prof) else "knn_scan_kernel"
    scan = [(fl, e0.elapsed_time(e1) / 1e3) for kn, fl, _, e0, e1, *_ in prof if kn == scan_kernel]
    scan_s = sum(s for _, s in scan) / len(scan)
    scan_fl = sum(f for f, _ in scan) / len(scan)
    rk = r.double() + 1
    map10 = float(torch.where(rk <= k, 1.0 / rk, torch.zeros_like(rk)).mean())
    return {"metric": "gallery kNN QPS @1M x 512 (exact top-10 + rank of positive)", "value": round(Q / el, 1),
            "unit": "queries/s", "ms": round(el * 1e3, 3), "N": N, "D": D, "Q": Q, "k": k, "n_gpus": world,
            "scaling": "strong", "compute": "bf16 MFMA scan + exact f64 rerank", "map@10": round(map10, 6),
            "mrr": round(float((1.0 / rk).mean()), 6),
            "roofline": {"bound": "mfma", "kernel": scan_kernel, "achieved": round(scan_fl / scan_s / 1e12, 2),
                         "peak": MFMA_PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                         "frac": round(scan_fl / scan_s / 1e12 / MFMA_PEAK_TFLOPS["bf16"], 4),
                         "avg_launch_us": round(scan_s * 1e6, 2), "avg_launch_flops": scan_fl,
                         "traffic": pmc_traffic(scan_kernel)}}


def cpu_retrieval_baseline(N=1_000_000, D=512, nq=8):
    """reference-style per-query loop (inference.py:30-57: PairwiseDistance over the
    whole gallery + full sort + position of the positive) via the oracle's float64
    restatement on the host cores, on nq queries of the C4 workload, as queries/s."""
    import numpy as np
    from oracle import retrieval as oret
    g, qs, pos = oret.synthetic_gallery(N, D, nq)
    t0 = time.perf_counter()
    for i in range(nq):
        d = oret.l2_distances(qs[i], g)
        o = oret.order(d)
        int(np.nonzero(o == pos[i])[0][0])
    dt = time.perf_counter() - t0
    return {"value": round(nq / dt, 3), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{nq} queries x full {N}x{D} gallery, oracle/retrieval.py float64 distances + stable argsort "
                      "(numpy, single-threaded), per-query like the reference"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=384, help="triplets per GPU per step")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the live per-launch event timing")
    ap.add_argument("--no-retrieval", action="store_true", help="skip the 1M x 512 kNN leg")
    ap.add_argument("--unbatched", dest="batched", action="store_false",
                    help="three separate encoder calls per step instead of forward_branches")
    args = ap.parse_args()

    import _hip
    import ddp
    import losses
    import models
    import optim

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    torch.manual_seed(1234)
    model = models.ModifiedResNet(LAYERS, OUT_DIM, heads=HEADS, input_resolution=RES, width=WIDTH).to(dev)
    model.compute_dtype = dtype
    model.train()
    ddp.broadcast_parameters(model)
    opt = optim.Adam(model.parameters(), lr=1e-5, weight_decay=0.002)
    loss_fn = losses.TripletMarginLoss(margin=0.2)

    # synthetic normalised 224x224 triplets, resident in HBM before timing
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    B = args.batch
    sketch = (torch.rand(B, 1, RES, RES, device=dev, generator=g) >= 0.1).float().expand(B, 3, RES, RES)
    pos = torch.rand(B, 3, RES, RES, device=dev, generator=g)
    neg = torch.rand(B, 3, RES, RES, device=dev, generator=g)
    mean = torch.tensor(models.CLIP_MEAN, device=dev)[None, :, None, None]
    std = torch.tensor(models.CLIP_STD, device=dev)[None, :, None, None]
    batch = [((t - mean) / std).contiguous() for t in (sketch, pos, neg)]

    def step():
        # the three branch forwards of train.py:28-30 (per-branch BN statistics),
        # each GEMM launched once over the 3 x B images
        outs = model.forward_branches(batch) if args.batched else [model(x) for x in batch]
        loss = loss_fn(*outs)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        ddp.allreduce_gradients(model)
        opt.step()
        return loss

    # the step runs on a high-priority stream: the dispatcher then serves the
    # HBM-bound data-gradient / BatchNorm chain first and the weight gradients
    # of the side stream (engine.py) fill in (ARTSBIR_STEP_PRIO=0: torch's stream)
    prio = int(os.environ.get("ARTSBIR_STEP_PRIO", "-1"))
    if prio:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=prio))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        ddp.broadcast_buffers(model)
        dist.barrier()
    torch.cuda.synchronize()
    prof = [] if not args.no_profile else None
    _hip.PROFILE = prof
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _hip.PROFILE = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last_loss = float(loss.item())

    if rank == 0:
        images = 3 * B * world * args.steps
        value = images / elapsed
        roof = None
        if prof:
            # per kernel: algorithmic FLOPs and bytes (declared by the engine per
            # launch) over the HIP-event time of its launches; the dominant kernel
            # (most time) is priced against the roof its arithmetic intensity hits
            agg = {}
            for kname, fl, nb, e0, e1, *_ in prof:
                a = agg.setdefault(kname, [0.0, 0.0, 0, 0.0])
                a[0] += fl
                a[1] += e0.elapsed_time(e1) / 1e3
                a[2] += 1
                a[3] += nb
            dom = max(agg, key=lambda k: agg[k][1])
            fl, secs, cnt, nb = agg[dom]
            peak_fl = MFMA_PEAK_TFLOPS[args.dtype]
            ridge = peak_fl * 1e12 / (HBM_PEAK_GBS * 1e9)
            if nb > 0 and fl / nb < ridge:
                achieved = nb / secs / 1e9
                roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4)}
            else:
                achieved = fl / secs / 1e12
                roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak_fl, "unit": "TFLOP/s",
                        "frac": round(achieved / peak_fl, 4)}
            roof.update({"traffic": pmc_traffic(dom), "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT),
                         "kernel": dom, "launches": cnt, "avg_launch_us": round(secs / cnt * 1e6, 2),
                         "avg_launch_flops": fl / cnt, "avg_launch_bytes": nb / cnt,
                         "intensity_flop_per_byte": round(fl / nb, 1) if nb else None,
                         "per_kernel": {k: {"launches": v[2], "avg_us": round(v[1] / v[2] * 1e6, 2),
                                            "tflops": round(v[0] / v[1] / 1e12, 1),
                                            "gbs": round(v[3] / v[1] / 1e9, 1), "share_s": round(v[1], 4)}
                                        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])}})
        step_flops = train_flops_per_triplet() * B
        line = {
            "metric": "triplet-images/sec embedded @224² bf16, 1→8 GPU; gallery kNN QPS @1M×512",
            "value": round(value, 2), "unit": "triplet-images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": "triplet training step (train.py:59-70): 3x encoder fwd + TripletMarginLoss "
                                   "+ backward + Adam", "model": "ModifiedResNet((3,4,6,3), output_dim=512)",
                       "global_batch": B * world, "triplets_per_gpu": B, "seq_len": None, "resolution": RES,
                       "parallelism": f"dp{world}"},
            "triplets_per_s": round(value / 3, 2),
            "step_tflops": round(step_flops * world / (elapsed / args.steps) / 1e12, 2),
            "loss": last_loss,
            "roofline": roof,
        }
    ret = None if args.no_retrieval else retrieval_leg(dev, rank, world)
    if rank == 0:
        if ret is not None:
            line["retrieval"] = ret
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
            if ret is not None:
                ret["cpu_baseline"] = cpu_retrieval_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
