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
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0}  # MI355X dense (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md; ~6.3 TB/s measured copy)
# per-launch HBM bytes of each kernel from the committed rocprofv3 PMC passes
# (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; profiles/summarize_pmc.py)
# One file per leg: a kernel name pools different launch shapes in each leg
# (training step + retrieval scan, eval-BN embed pass, C5 ViT step), so a leg's
# roofline only takes traffic measured on that leg's own launches.
# the autotuner's choices for every shape of every leg on MI355X (a find-db:
# `bench.py --tune-cache none --tune-save FILE` regenerates it); the PMC traffic
# files below were measured with it loaded, so a kernel name stands for the
# same launches in both
TUNE_CACHE = os.path.join(ROOT, "profiles", "tune_r6.txt")
PMC_TRAFFIC = os.environ.get("ARTSBIR_PMC_TRAFFIC", os.path.join(ROOT, "profiles", "r6_pmc_traffic.json"))
PMC_TRAFFIC_EMBED = os.environ.get("ARTSBIR_PMC_TRAFFIC_EMBED",
                                   os.path.join(ROOT, "profiles", "r6_embed_pmc_traffic.json"))
PMC_TRAFFIC_C5 = os.environ.get("ARTSBIR_PMC_TRAFFIC_C5", os.path.join(ROOT, "profiles", "r6_c5_pmc_traffic.json"))


def pmc_traffic(kernel, path=None):
    try:
        with open(path or PMC_TRAFFIC) as f:
            ks = json.load(f)["kernels"]
        # the traffic files key the tiled GEMM kernels by the same names the
        # library records (profiles/summarize_pmc.py); other kernels by bare name
        k = ks.get(kernel) or ks.get(kernel.split("<")[0])
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None else round(k["hbm_bytes_per_launch"])


def pmc_traffic_by_size(kernel, path=None):
    """the same kernel's bytes with the reads counted by request size (None
    when the traffic file has no request-size pass)"""
    try:
        with open(path or PMC_TRAFFIC) as f:
            ks = json.load(f)["kernels"]
        k = ks.get(kernel) or ks.get(kernel.split("<")[0])
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None or "hbm_bytes_by_size_per_launch" not in k else round(k["hbm_bytes_by_size_per_launch"])


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


def cpu_model():
    """the host CPU's model string (stated with every CPU baseline)"""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def roofline(prof, peak_of, traffic_file=None):
    """Roofline of the dominant kernel from a live per-launch profile (_hip.PROFILE
    entries: kernel, algorithmic FLOPs, algorithmic bytes, HIP start / end events
    on the launch's stream).  Launches are pooled by kernel name; the dominant
    kernel has the largest summed time; its bound follows its arithmetic
    intensity against the ridge peak / HBM.  peak_of(kernel) -> the dense MFMA
    TFLOP/s of that kernel's operand type.  Each launch is also priced at its own
    roofline time max(bytes / HBM peak, FLOPs / MFMA peak): a kernel name pools
    MFMA-bound and HBM-bound shapes, whose pooled GB/s or TFLOP/s alone
    understates both; sum(roofline time) / sum(time) does not."""
    main_sid = torch.cuda.current_stream().cuda_stream
    agg = {}
    for kname, fl, nb, e0, e1, *_ in prof:
        a = agg.setdefault(kname, [0.0, 0.0, 0, 0.0, 0.0])
        a[0] += fl
        a[1] += e0.elapsed_time(e1) / 1e3
        a[2] += 1
        a[3] += nb
        a[4] += max(nb / (HBM_PEAK_GBS * 1e9), fl / (peak_of(kname) * 1e12))
    # per family (by the launch's tag) and per stream: kernel time per step would
    # otherwise hinge on which tile variant of a family happens to be the largest
    fam, streams = {}, {}
    for kname, fl, nb, e0, e1, *rest in prof:
        tag = rest[0] if rest else None
        f = launch_family(kname, tag)
        ms = e0.elapsed_time(e1)
        v = fam.setdefault(f, [0.0, 0, 0.0, 0.0])
        v[0] += ms
        v[1] += 1
        v[2] += fl
        v[3] += nb
        if len(rest) > 1:
            streams[rest[1]] = streams.get(rest[1], 0.0) + ms
    dom = max(agg, key=lambda k: agg[k][1])
    fl, secs, cnt, nb, rt = agg[dom]
    peak_fl = peak_of(dom)
    ridge = peak_fl * 1e12 / (HBM_PEAK_GBS * 1e9)
    if nb > 0 and fl / nb < ridge:
        achieved = nb / secs / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4)}
    else:
        achieved = fl / secs / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak_fl, "unit": "TFLOP/s",
                "frac": round(achieved / peak_fl, 4)}
    tf = traffic_file or PMC_TRAFFIC
    traffic = pmc_traffic(dom, tf)
    roof.update({"traffic": traffic, "traffic_source": os.path.relpath(tf, ROOT) if traffic is not None else None,
                 "traffic_over_algorithmic": round(traffic / (nb / cnt), 3) if traffic and nb else None,
                 # reads by request size (FETCH_SIZE x 2 over-counts 64-B requests 2x)
                 "traffic_by_request_size": pmc_traffic_by_size(dom, tf),
                 "kernel": dom, "launches": cnt, "avg_launch_us": round(secs / cnt * 1e6, 2),
                 "avg_launch_flops": fl / cnt, "avg_launch_bytes": nb / cnt,
                 "intensity_flop_per_byte": round(fl / nb, 1) if nb else None,
                 "frac_launch_roofline": round(rt / secs, 4),
                 "step_launch_roofline": round(sum(v[4] for v in agg.values()) / sum(v[1] for v in agg.values()), 4),
                 "per_kernel": {k: {"launches": v[2], "avg_us": round(v[1] / v[2] * 1e6, 2),
                                    "tflops": round(v[0] / v[1] / 1e12, 1),
                                    "gbs": round(v[3] / v[1] / 1e9, 1), "share_s": round(v[1], 4),
                                    "roof_frac": round(v[4] / v[1], 4)}
                                for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])},
                 # kernel ms summed over the profiled launches (divide by the steps for ms/step)
                 "families": {f: {"kernel_ms": round(v[0], 3), "launches": v[1],
                                  "tflops": round(v[2] / (v[0] / 1e3) / 1e12, 1) if v[0] else None,
                                  "gbs": round(v[3] / (v[0] / 1e3) / 1e9, 1) if v[0] else None}
                              for f, v in sorted(fam.items(), key=lambda kv: -kv[1][0])},
                 # the caller's stream (the step's main stream) by its handle, the others by theirs
                 "streams_kernel_ms": {("main" if sid == main_sid else f"stream_{sid:x}"): round(ms, 3)
                                       for sid, ms in sorted(streams.items(), key=lambda kv: -kv[1])}})
    return roof


def launch_family(kernel, tag):
    """the step's kernel families: forward convolutions / GEMMs, fused BN-backward
    data gradients, plain data gradients, weight gradients (the overlapped side
    stream), the elementwise BatchNorm / ReLU / pool passes, everything else"""
    t = (tag or "").split(" ")[0]
    if t.startswith(("dgrad+bn", "dgrad_fold+bn")):
        return "bn_backward_dgrad"
    if t in ("dgrad", "dgrad_fold"):
        return "dgrad"
    if t in ("wgrad", "gemm_tn", "wgrad_fold", "gram", "fold_combine"):
        return "weight_gradient"
    if t in ("fwd", "fwd_act", "gemm_nt"):
        return "forward_gemm"
    if t.startswith(("act_pool", "block_out", "bn_", "fold_prep")):
        return "elementwise_bn"
    return "other"



def preprocess_leg(dev, rank, world, n_triplets=384, reps=5):
    """the input transform of the training step (models.py:289-295:
    Resize(224, bicubic) -> CenterCrop -> RGB -> ToTensor -> Normalize) for one
    step's 3 x n_triplets decoded images, as train.py --gpu_preprocess runs it:
    one preprocess.ClipPreprocess call on a batch whose uint8 pixels are already
    in HBM.  Images: data_preparation.synthetic_pixels stand-ins of decoded files
    (sketches 256 x 256 grayscale, photos RGB 256..640 px per side, ragged).
    Algorithmic bytes per image: its decoded pixels read once + the 3 x 224 x 224
    f32 output written once.  Also: the PCIe-inclusive rate (host pixels ->
    pinned staging -> HBM -> transform), the host's JPEG decode rate per core
    (what the DataLoader workers still do) and the CPU transform as cpu_baseline."""
    import _hip
    import data_preparation as dp
    import preprocess
    imgs = []
    for i in range(n_triplets):
        imgs.append(dp.synthetic_pixels(f"bench/sketches/s{rank}_{i}.png", "sketch"))
        imgs.append(dp.synthetic_pixels(f"bench/photos/p{rank}_{i}.jpg", "photo"))
        imgs.append(dp.synthetic_pixels(f"bench/photos/n{rank}_{i}.jpg", "photo"))
    pre = preprocess.ClipPreprocess(RES, device=dev)
    in_bytes = float(sum(a.nbytes for a in imgs))
    out_bytes = float(len(imgs) * 3 * RES * RES * 4)
    devbuf, descs = pre.stage(imgs)
    out = pre.run(devbuf, descs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    prof = []
    _hip.PROFILE = prof
    t0 = time.perf_counter()
    for _ in range(reps):
        pre.run(devbuf, descs, out=out, nbytes=in_bytes + out_bytes)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    _hip.PROFILE = None
    kern_s = sum(e0.elapsed_time(e1) for _, _, _, e0, e1, *_ in prof) / 1e3 / len(prof)
    # PCIe-inclusive: host pixels staged to pinned memory, copied, transformed
    t1 = time.perf_counter()
    for _ in range(2):
        pre(imgs)
    torch.cuda.synchronize()
    pcie = (time.perf_counter() - t1) / 2
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    n = len(imgs)
    achieved = (in_bytes + out_bytes) / kern_s / 1e9
    return {"metric": "images/s through the GPU input transform (train.py --gpu_preprocess)",
            "value": round(n * world / el, 1), "unit": "images/s", "images_per_call": n, "n_gpus": world,
            "ms_per_call": round(el * 1e3, 3), "pcie_inclusive_images_per_s": round(n / pcie, 1),
            "input_mb_per_call": round(in_bytes / 1e6, 1),
            "bit_exact_vs": "models.ClipTransform (Pillow) — tests/test_preprocess_gpu.py",
            "roofline": {"bound": "hbm", "kernel": "pp_horizontal_kernel + pp_vertical_kernel (one call)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "avg_launch_us": round(kern_s * 1e6, 2),
                         "avg_launch_bytes": in_bytes + out_bytes, "traffic": None,
                         "note": "priced against HBM as the contract asks; the passes are bound by byte-gather "
                                 "issue (Pillow's integer bicubic taps: ~3 byte loads + 3 MACs per tap and channel, "
                                 "profiles/r3_preprocess_kernel_stats.csv), not by HBM bytes"}}


def cpu_preprocess_baseline(n=96, budget_s=10.0):
    """the reference's input path on the host cores: JPEG/PNG decode (PIL) and
    the model transform (models.ClipTransform = models.py:289-295 on Pillow) in a
    thread pool of every core; decode is also timed alone, per core"""
    import io
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image
    import data_preparation as dp
    import models
    cores = cpu_cores()
    files = []
    for i in range(n):
        kind = "sketch" if i % 3 == 0 else "photo"
        a = dp.synthetic_pixels(f"bench/cpu/{i}", kind)
        buf = io.BytesIO()
        Image.fromarray(a).save(buf, format="PNG" if kind == "sketch" else "JPEG", quality=90)
        files.append(buf.getvalue())
    tr = models.ClipTransform(RES)

    def decode(b):
        with Image.open(io.BytesIO(b)) as im:
            im.load()
            return im.copy()
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s / 4 and done < 4 * n:
        decode(files[done % n])
        done += 1
    dec1 = done / (time.perf_counter() - t0)

    def full(b):
        return tr(decode(b))
    with ThreadPoolExecutor(cores) as ex:
        list(ex.map(full, files[:cores]))
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < budget_s and done < 20 * n:
            list(ex.map(full, files))
            done += n
        dt = time.perf_counter() - t0
    return {"value": round(done / dt, 1), "unit": "images/s", "cores": cores, "kind": "port", "cpu": cpu_model(),
            "decode_only_per_core": round(dec1, 1),
            "sample": f"{done} images (1/3 256^2 PNG sketches, 2/3 JPEG q90 photos 256..640 px): PIL decode + "
                      f"models.ClipTransform in a {cores}-thread pool; decode alone on 1 core"}


def cgroup_cpu_quota():
    """the CPU bandwidth limit of this process's cgroup in cores (cgroup v2
    cpu.max "quota period"), or None when unlimited / unreadable"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else float(quota) / float(period)
    except (OSError, ValueError):
        return None


def cpu_cores():
    """every core this process may run on (torch.set_num_threads(len(
    os.sched_getaffinity(0)))), capped only by a cgroup CPU quota if one is set
    (threads beyond the quota would just be throttled); ARTSBIR_CPU_THREADS overrides"""
    forced = int(os.environ.get("ARTSBIR_CPU_THREADS", "0") or 0)
    if forced:
        return forced
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q)) if q else n)


def cpu_info():
    """what the CPU baselines ran on (stated in the line)"""
    return {"cpu": cpu_model(), "affinity_cores": len(os.sched_getaffinity(0)), "cgroup_quota_cores": cgroup_cpu_quota(),
            "threads_used": cpu_cores()}


def cpu_baseline(batch=32, steps=3, layers=LAYERS, out_dim=OUT_DIM):
    """The oracle (torch CPU fp32 restatement of the reference path: three
    separate forwards, nn.TripletMarginLoss, torch.optim.Adam — train.py:27-37,
    59-70) on the host cores: a bounded sample of `batch` triplets per step."""
    from oracle import encoder as oenc, steps as osteps
    cores = cpu_cores()
    torch.set_num_threads(cores)
    m = osteps.build(layers, out_dim, HEADS, RES, WIDTH)
    opt = osteps.make_optimizer(m)
    loss = osteps.make_loss(0.2)
    el = list(oenc.synthetic_triplet(batch, RES))
    osteps.train_step(m, opt, loss, el)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        osteps.train_step(m, opt, loss, el)
    dt = time.perf_counter() - t0
    return {"value": round(3 * batch * steps / dt, 3), "unit": "triplet-images/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(), "host": cpu_info(),
            "sample": f"oracle/steps.py train_step, ModifiedResNet({layers},{out_dim}) fp32 224^2, {steps} timed "
                      f"steps x {batch} triplets after 1 warm-up, torch CPU {torch.__version__}"}


def retrieval_leg(dev, rank, world, N=1_000_000, D=512, Q=10_000, k=10, reps=3, noise=0.5):
    """BASELINE metric, second half: gallery kNN QPS at 1M x 512.
    Synthetic gallery G ~ N(0,1); query i = G[(i*7919) mod N] + noise * N(0,1), so
    each query has one planted positive (noise 0.5: the positive is the nearest;
    noise 3.0: ranks spread, mAP@10 < 1).  Timed: knn.knn (or knn_sharded over the
    ranks: gallery rows split, one all_gather + all_reduce) producing the exact
    top-10 and the rank of the positive for all Q queries; inputs resident in HBM."""
    import knn
    g = torch.Generator(device=dev).manual_seed(7)
    lo, hi = rank * N // world, (rank + 1) * N // world
    gal = torch.randn(N, D, device=dev, generator=g)  # same full gallery on every rank (seeded)
    pos = (torch.arange(Q, device=dev, dtype=torch.int64) * 7919) % N
    qs = gal[pos] + noise * torch.randn(Q, D, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
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
    import ctypes
    import _hip
    lib = _hip.lib()
    lib.artsbir_scan_profile(1)  # HIP events around the scan kernel inside the one call
    t0 = time.perf_counter()
    for _ in range(reps):
        idx, dd, r = run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    tot, cnt = ctypes.c_double(0.0), ctypes.c_int(0)
    lib.artsbir_scan_profile_read(ctypes.byref(tot), ctypes.byref(cnt))
    lib.artsbir_scan_profile(0)
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    scan_kernel = lib.artsbir_last_kernel().decode()
    scan_s = tot.value / 1e3 / max(cnt.value, 1)
    scan_fl = 2.0 * Q * (hi - lo) * D
    rk = r.double() + 1
    map10 = float(torch.where(rk <= k, 1.0 / rk, torch.zeros_like(rk)).mean())
    return {"metric": "gallery kNN QPS @1M x 512 (exact top-10 + rank of positive)", "value": round(Q / el, 1),
            "unit": "queries/s", "ms": round(el * 1e3, 3), "N": N, "D": D, "Q": Q, "k": k, "n_gpus": world,
            "scaling": "strong", "compute": "bf16 MFMA scan + exact f64 rerank", "noise": noise,
            "map@10": round(map10, 6),
            "mrr": round(float((1.0 / rk).mean()), 6),
            "roofline": {"bound": "mfma", "kernel": scan_kernel, "achieved": round(scan_fl / scan_s / 1e12, 2),
                         "peak": MFMA_PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                         "frac": round(scan_fl / scan_s / 1e12 / MFMA_PEAK_TFLOPS["bf16"], 4),
                         "avg_launch_us": round(scan_s * 1e6, 2), "avg_launch_flops": scan_fl,
                         "traffic": pmc_traffic(scan_kernel)}}


def cpu_retrieval_baseline(N=1_000_000, D=512, nq=100, budget_s=25.0):
    """SURVEY §8d retrieval CPU baseline on the host cores, torch fp32:
      per_query — the reference's op sequence per query (inference.py:43-56:
                  nn.PairwiseDistance(p=2) of [1,D] vs the [N,D] gallery, full
                  topk(N, largest=False), position of the positive), over up to nq
                  queries of the C4 workload or until budget_s is spent;
      batched   — a fair CPU variant: one GEMM-form distance matrix for the same
                  queries and topk(10) per row, plus the rank of the positive."""
    cores = cpu_cores()
    torch.set_num_threads(cores)
    g = torch.randn(N, D, generator=torch.Generator().manual_seed(7))
    pos = (torch.arange(nq) * 7919) % N
    qs = g[pos] + 0.5 * torch.randn(nq, D, generator=torch.Generator().manual_seed(8))
    pdist = torch.nn.PairwiseDistance(p=2)
    pdist(qs[:1], g).topk(N, largest=False)  # warm-up
    done = 0
    t0 = time.perf_counter()
    while done < nq and time.perf_counter() - t0 < budget_s:
        d = pdist(qs[done:done + 1], g)
        _, idx = d.topk(N, largest=False)
        int((idx == pos[done]).nonzero()[0, 0])
        done += 1
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    gsq = (g * g).sum(1)
    d2 = (qs * qs).sum(1)[:, None] + gsq[None, :] - 2.0 * (qs @ g.T)
    d2.topk(10, dim=1, largest=False)
    (d2 < d2.gather(1, pos[:, None])).sum(1)
    dtb = time.perf_counter() - t1
    return {"value": round(done / dt, 3), "unit": "queries/s", "cores": cores, "kind": "port", "cpu": cpu_model(),
            "sample": f"{done} queries (of {nq}, {budget_s:.0f} s budget) x full {N}x{D} gallery: torch fp32 "
                      f"nn.PairwiseDistance + topk(N) per query like inference.py:43-56, {cores} threads",
            "batched": {"value": round(nq / dtb, 3), "unit": "queries/s",
                        "sample": f"{nq} queries as one fp32 GEMM-form distance matrix + topk(10) + rank, "
                                  f"{cores} threads"}}


def embed_leg(model, batch, dtype_name, world, reps):
    """Embed-only throughput of C2 (the BASELINE metric's "triplet-images/sec
    embedded"): eval-mode BatchNorm (running statistics), no autograd, the 3 x B
    images of one triplet batch per pass — inference.py:72-92's
    compute_image_features arithmetic on the triplet workload."""
    import _hip
    model.eval()
    with torch.no_grad():
        model.forward_branches(batch)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = model.forward_branches(batch)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # a separate profiled pass set: per-launch HIP events (roofline), not in the timed region
        prof = []
        _hip.PROFILE = prof
        for _ in range(reps):
            model.forward_branches(batch)
        torch.cuda.synchronize()
        _hip.PROFILE = None
    model.train()
    if world > 1:
        t = torch.tensor([el], device=batch[0].device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    images = sum(x.shape[0] for x in batch) * reps * world
    gpu_s = sum(e0.elapsed_time(e1) for _, _, _, e0, e1, *_ in prof) / 1e3
    fl = encoder_flops_per_image() * images / world
    # the dominant kernel of the pass, priced per launch like the step's
    roof = roofline(prof, lambda k: MFMA_PEAK_TFLOPS[dtype_name], PMC_TRAFFIC_EMBED) if prof else None
    return {"metric": "triplet-images/s embedded (eval BatchNorm, no backward)", "value": round(images / el, 2),
            "unit": "triplet-images/s", "ms_per_pass": round(el / reps * 1e3, 3), "n_gpus": world,
            "images_per_pass": sum(x.shape[0] for x in batch), "dtype": dtype_name,
            "finite": bool(torch.isfinite(torch.cat(out)).all()),
            "roofline": roof,
            "pass_mfma": {"achieved": round(fl / el / 1e12, 2), "peak": MFMA_PEAK_TFLOPS[dtype_name],
                          "unit": "TFLOP/s", "frac": round(fl / el / 1e12 / MFMA_PEAK_TFLOPS[dtype_name], 4),
                          "kernel_time_share": round(gpu_s / el, 3) if el else None,
                          "note": "whole forward pass: algorithmic encoder FLOPs (bench.encoder_flops_per_image) "
                                  "over wall time"}}


def cpu_embed_baseline(batch=48, reps=2):
    """oracle eval-mode embedding (inference.py:72-92 in batches of 50) of a
    bounded sample on the host cores"""
    from oracle import encoder as oenc, steps as osteps
    cores = cpu_cores()
    torch.set_num_threads(cores)
    m = osteps.build(LAYERS, OUT_DIM, HEADS, RES, WIDTH)
    imgs = torch.cat(oenc.synthetic_triplet(batch // 3, RES))
    osteps.embed(m, imgs[:8])
    t0 = time.perf_counter()
    for _ in range(reps):
        osteps.embed(m, imgs)
    dt = time.perf_counter() - t0
    return {"value": round(len(imgs) * reps / dt, 3), "unit": "triplet-images/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(), "sample": f"oracle/steps.py embed (eval BN, batches of 50), {len(imgs)} images x "
                                          f"{reps}, ModifiedResNet((3,4,6,3),512) fp32 224^2"}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(n: int, argv, port: int):
    """the command that runs this benchmark as n ranks, one process per GPU
    (torch.distributed.run on 127.0.0.1: RANK / LOCAL_RANK / WORLD_SIZE in each
    child's environment, so the children do not launch again)"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` outside a launcher: start the N ranks as child
    processes and return their exit status.  Nothing in this process has
    touched the GPU (no HIP call, no torch.cuda query), and it never execs —
    it waits for the children and passes their status on."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_command(n, argv, free_port()), env=env)


def launch_check(world, rank):
    """--launch-check: the rank protocol alone (no GPU work): every rank joins the
    process group, the ranks agree on the world size by an all-reduce, rank 0
    prints one JSON line — tests/test_bench_launch.py runs it on the CPU (gloo)"""
    import ddp
    ddp.init_distributed()
    t = torch.ones(1)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "world_size": dist.get_world_size(),
                          "all_reduce": float(t.item()), "backend": dist.get_backend()}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE, else 1); without a launcher's WORLD_SIZE, "
                         "N > 1 starts the N ranks itself under torch.distributed.run")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=384, help="triplets per GPU per step")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the live per-launch event timing")
    ap.add_argument("--no-retrieval", action="store_true", help="skip the 1M x 512 kNN leg")
    ap.add_argument("--unbatched", dest="batched", action="store_false",
                    help="three separate encoder calls per step instead of forward_branches")
    ap.add_argument("--no-embed", action="store_true", help="skip the embed-only (eval-BN) leg")
    ap.add_argument("--no-preprocess", action="store_true", help="skip the GPU input-transform leg")
    ap.add_argument("--sync-warmup", action="store_true", help="synchronize after every warmup step")
    ap.add_argument("--c5", action="store_true", default=True,
                    help="the C5 leg: ViT-B/16 768-d triplet training step, fp8 projections, 512 triplets (default)")
    ap.add_argument("--no-c5", dest="c5", action="store_false", help="skip the C5 leg")
    ap.add_argument("--c5-batch", type=int, default=512, help="C5 triplets per GPU per step")
    ap.add_argument("--no-loss-check", action="store_true", help="skip the f32 step-0 loss check")
    ap.add_argument("--tune-cache", default=TUNE_CACHE,
                    help="autotuner choices loaded before the first step when the file exists (default: the "
                         "committed MI355X table, so every run and every profiling pass launches the same kernel "
                         "per shape; 'none': tune every shape on its first call)")
    ap.add_argument("--tune-save", default=None,
                    help="write the autotuner's choices after every leg has run (shapes of all legs)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or 1)
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} under a launcher of {env_world} ranks")
    if args.launch_check:
        return launch_check(int(env_world or 1), int(os.environ.get("RANK", "0")))

    import _hip
    import ddp
    import losses
    import models
    import optim

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        # RCCL ("nccl") over xGMI, one GPU per rank; ARTSBIR_DIST_BACKEND=gloo lets
        # several ranks share one device (a rehearsal of the N > 1 code path)
        ddp.init_distributed()
        backend = dist.get_backend()
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group of {dist.get_world_size()} ranks for --gpus {args.gpus}")
    dev = torch.device("cuda", torch.cuda.current_device())
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

    if args.tune_cache and args.tune_cache != "none" and os.path.exists(args.tune_cache):
        n = _hip.lib().artsbir_tune_load(args.tune_cache.encode())
        if n < 0:
            raise RuntimeError(f"tune cache {args.tune_cache}: {_hip.lib().artsbir_last_error().decode()}")

    # step-0 loss check: the f32 parity mode of the same library (within 1e-3 of
    # the oracle, tests/test_c2_gpu.py) on the same batch and initial weights;
    # the bf16 step's loss must agree (running stats restored afterwards)
    loss_f32 = dscale = None
    if not args.no_loss_check:
        saved = {k: v.clone() for k, v in model.state_dict().items() if "running" in k or "num_batches" in k}
        model.compute_dtype = torch.float32
        with torch.no_grad():
            a32, p32, n32 = model.forward_branches(batch)
            loss_f32 = float(loss_fn(a32, p32, n32).item())
            # the hinge's argument is a difference of distances: its error scales with them
            dscale = float(((a32 - p32).norm(dim=1) + (a32 - n32).norm(dim=1)).mean())
            del a32, p32, n32
        model.compute_dtype = dtype
        model.load_state_dict(saved, strict=False)
        torch.cuda.empty_cache()

    reducer = ddp.attach_overlapped_reducer(model)

    def step():
        # the three branch forwards of train.py:28-30 (per-branch BN statistics),
        # each GEMM launched once over the 3 x B images
        outs = model.forward_branches(batch) if args.batched else [model(x) for x in batch]
        loss = loss_fn(*outs)
        opt.zero_grad(set_to_none=False)
        loss.backward()  # N > 1: all-reduce buckets start inside the backward (ddp.OverlappedReducer)
        reducer.finish()
        opt.step()
        return loss

    # the step runs on a high-priority stream: the dispatcher then serves the
    # HBM-bound data-gradient / BatchNorm chain first and the weight gradients
    # of the side stream (engine.py) fill in (ARTSBIR_STEP_PRIO=0: torch's stream)
    prio = int(os.environ.get("ARTSBIR_STEP_PRIO", "-1"))
    if prio:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=prio))
    loss0 = None
    for i in range(max(args.warmup, 1)):
        li = step()
        if i == 0:
            loss0 = float(li.item())
        if args.sync_warmup:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        ddp.broadcast_buffers(model)
        dist.barrier()
    torch.cuda.synchronize()
    ms0 = torch.cuda.memory_stats(dev)
    # the timed region: K steps, nothing recorded per launch (the per-launch HIP
    # events of the profiling pass cost host time that shows up as GPU idle gaps
    # once the step is this short)
    step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    step_ev[0].record()
    for i in range(args.steps):
        loss = step()
        step_ev[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last_loss = float(loss.item())
    ms1 = torch.cuda.memory_stats(dev)
    alloc = {"step_ms": [round(step_ev[i].elapsed_time(step_ev[i + 1]), 2) for i in range(args.steps)],
             "retries_timed": ms1.get("num_alloc_retries", 0) - ms0.get("num_alloc_retries", 0),
             "device_mallocs_timed": ms1.get("num_device_alloc", 0) - ms0.get("num_device_alloc", 0),
             "reserved_peak_gb": round(ms1.get("reserved_bytes.all.peak", 0) / 2**30, 1),
             "allocated_peak_gb": round(ms1.get("allocated_bytes.all.peak", 0) / 2**30, 1)}
    # the roofline pass: the same K steps again, every launch bracketed by HIP
    # events on the stream it runs on (kernel durations, not the step time)
    prof = [] if not args.no_profile else None
    if prof is not None:
        _hip.PROFILE = prof
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        _hip.PROFILE = None

    if rank == 0:
        images = 3 * B * world * args.steps
        value = images / elapsed
        roof = roofline(prof, lambda k: MFMA_PEAK_TFLOPS[args.dtype]) if prof else None
        step_flops = train_flops_per_triplet() * B
        line = {
            "metric": "triplet-images/sec embedded @224² bf16, 1→8 GPU; gallery kNN QPS @1M×512",
            "value": round(value, 2), "unit": "triplet-images/s", "n_gpus": world, "world_size": world,
            "backend": backend, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": "triplet training step (train.py:59-70): 3x encoder fwd + TripletMarginLoss "
                                   "+ backward + Adam", "model": "ModifiedResNet((3,4,6,3), output_dim=512)",
                       "global_batch": B * world, "triplets_per_gpu": B, "seq_len": None, "resolution": RES,
                       "parallelism": f"dp{world}"},
            "triplets_per_s": round(value / 3, 2),
            "step_tflops": round(step_flops * world / (elapsed / args.steps) / 1e12, 2),
            "loss": last_loss,
            "loss_step0": loss0,
            "loss_step0_f32": loss_f32,
            "loss_step0_rel_diff": (round(abs(loss0 - loss_f32) / max(abs(loss_f32), 1e-12), 6)
                                    if loss_f32 is not None else None),
            "loss_step0_rel_to_distance_scale": (round(abs(loss0 - loss_f32) / max(dscale, 1e-12), 6)
                                                 if loss_f32 is not None else None),
            "roofline": roof,
            "allocator": alloc,
        }
    emb = None if args.no_embed else embed_leg(model, batch, args.dtype, world, args.steps)
    c5 = c5_leg(dev, rank, world, args.c5_batch, max(2, args.steps // 2), profile=not args.no_profile,
                loss_check=not args.no_loss_check) if args.c5 else None
    pre = None if args.no_preprocess else preprocess_leg(dev, rank, world, args.batch)
    ret = None if args.no_retrieval else retrieval_leg(dev, rank, world)
    if ret is not None:
        # the same workload with queries far from their positives (ranks spread,
        # more list insertions and rank-band decisions in the scan)
        hard = retrieval_leg(dev, rank, world, reps=2, noise=3.0)
        ret["noise3"] = {k: hard[k] for k in ("value", "unit", "ms", "map@10", "mrr")}
        ret["noise3"]["scan_frac"] = hard["roofline"]["frac"]
    if args.tune_save and rank == 0:
        _hip.lib().artsbir_tune_save(args.tune_save.encode())
    if rank == 0:
        line["tune_cache"] = (os.path.relpath(args.tune_cache, ROOT) if args.tune_cache and args.tune_cache != "none"
                              and os.path.exists(args.tune_cache) else None)
        if emb is not None:
            line["embed"] = emb
        if ret is not None:
            line["retrieval"] = ret
        if c5 is not None:
            line["c5"] = c5
        if pre is not None:
            line["preprocess"] = pre
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
            # C1 (BASELINE configs[0]): the "ResNet18 128-d" config = ModifiedResNet((2,2,2,2),128), batch 32
            line["cpu_baseline"]["c1"] = cpu_baseline(batch=32, steps=2, layers=(2, 2, 2, 2), out_dim=128)
            if emb is not None:
                emb["cpu_baseline"] = cpu_embed_baseline()
            if ret is not None:
                ret["cpu_baseline"] = cpu_retrieval_baseline()
            if c5 is not None:
                c5["cpu_baseline"] = cpu_c5_baseline()
            if pre is not None:
                pre["cpu_baseline"] = cpu_preprocess_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def c5_leg(dev, rank, world, B, steps, warmup=1, profile=True, loss_check=True):
    """BASELINE configs[4] / SURVEY C5: ViT-B/16 (CLIP VisionTransformer, 224^2, patch 16,
    12 x 768, 12 heads) -> 768-d, triplet step (3 branch calls as one batch: no
    BatchNorm in a ViT), fp8 e4m3 projection GEMMs in the forward, bf16 elsewhere,
    Adam; synthetic normalised images resident in HBM.  Algorithmic work: 3 x
    (forward FLOPs) per image, forward = 35.1 GFLOP.  Step-0 check:
    the fp8 step's loss against the f32 mode of the same library on the same batch
    and weights (tests/test_c5_gpu.py holds every mode against the float64 oracle)."""
    import _hip
    import ddp
    import losses
    import optim
    import vit
    torch.manual_seed(4321)
    model = vit.VisionTransformer(224, 16, 768, 12, 12, 768).to(dev)
    model.train()
    opt = optim.Adam(model.parameters(), lr=1e-5, weight_decay=0.002)
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    g = torch.Generator(device=dev).manual_seed(200 + rank)
    xs = [torch.randn(B, 3, 224, 224, device=dev, generator=g) for _ in range(3)]
    check = None
    if loss_check:
        model.compute_dtype = torch.float32
        with torch.no_grad():
            a, p, n = model.forward_branches(xs)
            l32 = float(loss_fn(a, p, n).item())
            scale = float(((a - p).norm(dim=1) + (a - n).norm(dim=1)).mean())
        del a, p, n
        torch.cuda.empty_cache()
        check = {"loss_step0_f32": l32, "distance_scale": round(scale, 6)}
    model.compute_dtype = "fp8"

    def step():
        outs = model.forward_branches(xs)
        loss = loss_fn(*outs)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        ddp.allreduce_gradients(model)  # N > 1: coalesced bucketed all-reduce of the autograd gradients
        opt.step()
        return loss
    for i in range(warmup):
        li = step()
        if i == 0 and check is not None:
            check["loss_step0"] = float(li.item())
            # the hinge's argument is a difference of distances: its error scales with them
            check["rel_to_distance_scale"] = round(abs(check["loss_step0"] - l32) / max(scale, 1e-12), 6)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    roof = None
    if profile:
        prof = []
        _hip.PROFILE = prof
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        _hip.PROFILE = None
        roof = roofline(prof, lambda k: MFMA_PEAK_TFLOPS["fp8" if "fp8" in k else "bf16"], PMC_TRAFFIC_C5)
    images = 3 * B * world * steps
    flops = 3 * 35.1e9 * images
    out = {"metric": "triplet-images/sec, ViT-B/16 768-d fp8 (C5)", "value": round(images / el, 2),
           "unit": "triplet-images/s", "steps": steps, "ms_per_step": round(el / steps * 1e3, 2),
           "triplets_per_gpu": B, "dtype": "fp8 e4m3 projections (forward), bf16 otherwise",
           "tflops": round(flops / el / 1e12, 1), "loss": float(loss.item()), "data": "synthetic",
           "roofline": roof, "step0_check": check}
    return out


def cpu_c5_baseline(batch=2, steps=2):
    """the oracle's ViT-B/16 (oracle/encoder.vision_transformer, CLIP keys) in torch
    CPU fp32: three separate branch forwards, nn.TripletMarginLoss(0.2), backward,
    torch.optim.Adam — a bounded sample of `batch` triplets per step"""
    from oracle import encoder as oenc
    import vit
    cores = cpu_cores()
    torch.set_num_threads(cores)
    torch.manual_seed(4321)
    sd = {k: v.detach().float().clone().requires_grad_(True)
          for k, v in vit.VisionTransformer(224, 16, 768, 12, 12, 768).state_dict().items()}
    opt = torch.optim.Adam(list(sd.values()), lr=1e-5, weight_decay=0.002)
    loss_fn = torch.nn.TripletMarginLoss(margin=0.2)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(batch, 3, 224, 224, generator=g) for _ in range(3)]

    def step():
        outs = [oenc.vision_transformer(x, sd, 16, 12) for x in xs]
        loss = loss_fn(*outs)
        opt.zero_grad()
        loss.backward()
        opt.step()
    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": round(3 * batch * steps / dt, 3), "unit": "triplet-images/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(), "sample": f"oracle/encoder.vision_transformer ViT-B/16 fp32 224^2, {steps} timed "
                                          f"steps x {batch} triplets after 1 warm-up (3 branch forwards, "
                                          f"TripletMarginLoss, Adam), torch CPU {torch.__version__}"}


if __name__ == "__main__":
    main()
