"""Drop-in for /root/reference/inference.py on MI355X.

Same functions and result dictionary as the reference:
  get_ranking_position   inference.py:30-57   (name parsing -> positive -> rank)
  get_topk_images        inference.py:60-69
  compute_image_features inference.py:72-92   (eval-mode gallery embedding, batches of 50)
  process_inference      inference.py:94-136  (rank+1, MRR, topk_acc, describe() stats,
                                               10 retrieval samples chosen by random.seed(11))
  run_inference          inference.py:140-165 (+ the Kaggle/Mixed second pass with the
                                               Kaggle inference sketches, inference.py:154-163)
  run_inference_sharded  the same with the gallery sharded over ranks
  CLI                    inference.py:167-244 (--folder, -a/--all)
The per-query loop of the reference (one model call, one O(N) distance pass
and one full sort per sketch, with a device sync each) is replaced by batched
embedding and one fused all-pairs L2 scan over the whole gallery (knn.py);
the resulting order is exact (f64 distances, ties by gallery index).
Added: ``map@10`` (one relevant item per query: mean of 1/rank for rank <= 10).
"""
from __future__ import annotations

import argparse
import json
import random
import re
from pathlib import Path
from timeit import default_timer as timer
from typing import Dict, List, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader

import data_preparation
import knn
import utils

device = 'cuda' if torch.cuda.is_available() else 'cpu'


def sketch_target_name(sketch_path, image_paths):
    """inference.py:33-37."""
    stem = Path(sketch_path).stem
    parts = re.split('-', stem)
    if len(parts) <= 2:
        return stem if "artworks" in str(image_paths[0]) else parts[0]
    if len(parts) == 3:
        return parts[1]
    return None


def _search(sketch_features, image_features, k, positives, loss_type):
    """exact top-k (keys: ||q - g + 1e-6|| for 'euclidean', 1 - cos for 'cosine',
    utils.py:31-42) and 0-based ranks of the positives, one library call"""
    q, g = sketch_features.float(), image_features.float()
    if loss_type not in ('euclidean', 'cosine'):
        raise Exception(f"loss type not correct {loss_type}")  # inference.py:48
    k = min(k, g.shape[0])
    return knn.knn(q.contiguous(), g.contiguous(), k, positives, metric=loss_type)


def get_ranking_position(sketch_path, image_paths: List[Path], sketch_feature: torch.Tensor,
                         image_features: torch.Tensor, loss_type) -> int:
    name = sketch_target_name(sketch_path, image_paths)
    pos = utils.find_image_index(image_paths, name) if name is not None else -1
    if pos < 0:
        print(f"No image found: {sketch_path} | {name}")
        return len(image_paths)
    _, _, rank, _ = _search(sketch_feature.reshape(1, -1).to(image_features.device), image_features, 1,
                            torch.tensor([pos], dtype=torch.int64, device=image_features.device), loss_type)
    return int(rank[0].item())


def get_topk_images(k: int, image_paths: List[Path], sketch_feature: torch.Tensor, image_features: torch.Tensor,
                    loss_type) -> List[Tuple[str, float]]:
    idx, dist, _, _ = _search(sketch_feature.reshape(1, -1).to(image_features.device), image_features, k, None,
                              loss_type)
    return [(str(image_paths[i]), float(d)) for i, d in zip(idx[0].tolist(), dist[0].tolist())]


def _decoded(ds) -> bool:
    base = ds.dataset if isinstance(ds, torch.utils.data.Subset) else ds
    base = getattr(base, "ds", base)  # _Sketches
    return bool(getattr(base, "decode_only", False))


def _loader(ds, batch_size=50):
    """the reference's DataLoader(bs=50, workers=0); decode-only datasets keep
    their ragged uint8 images as lists (GPU preprocessing in _embed)"""
    return DataLoader(ds, batch_size=batch_size, num_workers=0, shuffle=False,
                      collate_fn=data_preparation.collate_decoded if _decoded(ds) else None)


@torch.no_grad()
def _embed(model, loader, with_classification):
    import preprocess
    feats = []
    res = getattr(model, "input_resolution", 224)
    for batch in loader:
        if isinstance(batch, (list, tuple)) and len(batch) and isinstance(batch[0], torch.Tensor) \
                and batch[0].dtype == torch.uint8:
            x = preprocess.to_device_batch(batch, res, device)  # decoded images: one GPU transform call
        else:
            x = batch[0] if isinstance(batch, (list, tuple)) else batch
            x = x.to(device)
        out = model(x)
        feats.append(out[0] if with_classification else out)
    return torch.cat(feats) if feats else torch.empty(0)


def _gallery(dataset):
    """InferenceDataset of the dataset's photos (data_preparation.py:24-41), in the dataset's pixel mode"""
    return data_preparation.InferenceDataset(dataset.photo_paths, dataset.transform,
                                             getattr(dataset, "resolution", 224), getattr(dataset, "pixels", False),
                                             getattr(dataset, "decode_only", False))


def compute_image_features(model, dataset, with_classification: bool):
    inference_dataset = _gallery(dataset)
    loader = _loader(inference_dataset)
    model.to(device)
    model.eval()
    image_features = _embed(model, loader, with_classification)
    feature_path = utils.save_image_features(model.__class__.__name__, dataset.state_dict['dataset'],
                                             inference_dataset, image_features)
    return inference_dataset, image_features, feature_path


def retrieval_stats(ranks0, k=10):
    """inference.py:116-134 from 0-based ranks (+ map@k)."""
    ranks1 = [r + 1 for r in ranks0]
    mrr = float(np.mean([1.0 / r for r in ranks1])) if ranks1 else 0.0
    acc = np.zeros(k)
    for r in ranks0:
        if r < k:
            acc[r:] += 1
    acc /= max(len(ranks0), 1)
    s = pd_describe(ranks1)
    out = {"mean_reciprocal_rank": mrr}
    out.update(s)
    out["topk_acc"] = list(acc)
    out[f"map@{k}"] = float(np.mean([1.0 / r if r <= k else 0.0 for r in ranks1])) if ranks1 else 0.0
    return out


def pd_describe(values):
    """pandas DataFrame.describe() of one column (count, mean, std, min, 25/50/75 %, max)."""
    r = np.asarray(values, np.float64)
    if len(r) == 0:
        return {}
    d = {"count": float(len(r)), "mean": float(r.mean()), "std": float(r.std(ddof=1)) if len(r) > 1 else float("nan"),
         "min": float(r.min())}
    for q, key in ((0.25, "25%"), (0.5, "50%"), (0.75, "75%")):
        d[key] = float(np.quantile(r, q))
    d["max"] = float(r.max())
    return d


def _positives(dataset, paths):
    out = []
    for sp in dataset.sketch_paths:
        name = sketch_target_name(sp, paths)
        out.append(utils.find_image_index(paths, name) if name is not None else -1)
    return out


def _stats(dataset, inference_dataset, positives, idx, dist_, rank, start_time, k=10):
    """inference.py:94-136 from the batched search results"""
    random.seed(11)
    random_indices = [random.randrange(0, len(dataset)) for _ in range(10)]
    paths = inference_dataset.image_paths
    ranks = [int(r) if p >= 0 else len(paths) for r, p in zip(rank.tolist(), positives)]
    for sp, p in zip(dataset.sketch_paths, positives):
        if p < 0:
            print(f"No image found: {sp}")
    samples = []
    for i in sorted(set(random_indices)):
        for _ in range(random_indices.count(i)):
            samples.append({str(dataset.sketch_paths[i]): [(str(paths[j]), float(d))
                                                           for j, d in zip(idx[i].tolist(), dist_[i].tolist())]})
    stats = {"mean_reciprocal_rank": None, "size": len(inference_dataset), "inference_time": timer() - start_time}
    stats.update(retrieval_stats(ranks, k))
    stats["retrieval_samples"] = samples
    return stats


def process_inference(model, dataset, inference_dataset, dataloader, image_features, start_time,
                      with_classification, loss_type):
    k = 10
    image_features = image_features.to(device)
    model.to(device)
    model.eval()
    with torch.no_grad():
        sketch_features = _embed(model, dataloader, with_classification)
    positives = _positives(dataset, inference_dataset.image_paths)
    pos_t = torch.tensor(positives, dtype=torch.int64, device=device)
    idx, dist_, rank, _ = _search(sketch_features, image_features, k, pos_t, loss_type)
    return _stats(dataset, inference_dataset, positives, idx, dist_, rank, start_time, k)


# ------------------------------------------------- gallery sharded over ranks
# the reference embeds the gallery in one loop
# (inference.py:72-92); with one process per GPU each rank embeds a contiguous
# shard of the (sorted, de-duplicated) gallery, keeps it resident, and the
# retrieval runs shard-parallel (knn.knn_sharded: exact top-k per shard,
# all-gather of k (key, index) pairs per query, merge).  Queries are sharded
# the same way and all-gathered (they are few).  Only rank 0 writes the feature
# file, from the gathered gallery.

def shard_bounds(n: int, world: int) -> List[int]:
    """contiguous ragged shards: rank r owns rows [b[r], b[r+1])"""
    return [n * r // world for r in range(world + 1)]


def gather_rows(local: torch.Tensor, bounds: List[int]) -> torch.Tensor:
    """all-gather of ragged row shards (rank r holds bounds[r+1]-bounds[r] rows)
    into the full [bounds[-1], ...] tensor on every rank"""
    import torch.distributed as dist
    world = len(bounds) - 1
    rows = max(bounds[r + 1] - bounds[r] for r in range(world))
    pad = torch.zeros((rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((world * rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad)
    return torch.cat([out[r * rows:r * rows + bounds[r + 1] - bounds[r]] for r in range(world)])


def _embed_shard(model, ds, with_classification, batch_size=50):
    import torch.distributed as dist
    b = shard_bounds(len(ds), dist.get_world_size())
    r = dist.get_rank()
    loader = _loader(torch.utils.data.Subset(ds, range(b[r], b[r + 1])), batch_size)
    with torch.no_grad():
        feats = _embed(model, loader, with_classification)
    if feats.numel() == 0:  # an empty shard still needs the feature width for the gather
        feats = feats.reshape(0, 0)
    return feats, b


def compute_image_features_sharded(model, dataset, with_classification: bool, save: bool = True):
    """-> (inference_dataset, this rank's gallery rows, g_base, feature_path or None)"""
    import torch.distributed as dist
    inference_dataset = _gallery(dataset)
    model.to(device)
    model.eval()
    feats, b = _embed_shard(model, inference_dataset, with_classification)
    feature_path = None
    if save:
        full = gather_rows(_widen(feats, model, inference_dataset, with_classification), b)
        if dist.get_rank() == 0:
            feature_path = utils.save_image_features(model.__class__.__name__, dataset.state_dict['dataset'],
                                                     inference_dataset, full.cpu())
    return inference_dataset, feats, b[dist.get_rank()], feature_path


def _widen(feats, model, ds, with_classification):
    """an empty shard as [0, D] (D from one probe embedding) so every rank gathers the same width"""
    if feats.shape[0] > 0 or len(ds) == 0:
        return feats
    with torch.no_grad():
        probe = _embed(model, _loader(torch.utils.data.Subset(ds, [0]), 1), with_classification)
    return probe[:0]


def process_inference_sharded(model, dataset, inference_dataset, sketches, shard_features, g_base, start_time,
                              with_classification, loss_type, **search):
    """process_inference with the gallery sharded over the ranks (every rank
    returns the same stats).  ``search``: knn.knn_sharded's stand-in hooks (tests)."""
    k = 10
    if loss_type not in ('euclidean', 'cosine'):
        raise Exception(f"loss type not correct {loss_type}")
    model.to(device)
    model.eval()
    q_local, qb = _embed_shard(model, sketches, with_classification)
    queries = gather_rows(_widen(q_local, model, sketches, with_classification), qb).float()
    positives = _positives(dataset, inference_dataset.image_paths)
    pos_t = torch.tensor(positives, dtype=torch.int64, device=queries.device)
    kk = min(k, len(inference_dataset))
    idx, dist_, rank = knn.knn_sharded(queries.contiguous(), shard_features.float().contiguous(), g_base, kk, pos_t,
                                       metric=loss_type, **search)
    return _stats(dataset, inference_dataset, positives, idx, dist_, rank, start_time, k)


def _second_pass(model, dataset, inference_dataset, image_features, first, with_classification, loss_type,
                 sharded=None, **search):
    """inference.py:154-165: Kaggle / Mixed test sets are also ranked with the
    Kaggle inference sketches (sketch_type 'sketches') against the same gallery"""
    _, dataset2 = data_preparation.get_datasets('KaggleInferenceV1', sketch_type='sketches',
                                                transform=dataset.transform)
    if sharded is not None:
        shard, g_base = sharded
        return process_inference_sharded(model, dataset2, inference_dataset, _Sketches(dataset2), shard, g_base,
                                         first['inference_time'], with_classification, loss_type, **search)
    loader2 = _loader(_Sketches(dataset2))
    return process_inference(model, dataset2, inference_dataset, loader2, image_features, first['inference_time'],
                             with_classification, loss_type)


def _needs_second_pass(dataset) -> bool:
    name = dataset.state_dict['dataset']
    return 'Kaggle' in name or 'Mixed' in name


def run_inference(model, dataset, folder_name: str = None, loss_type='euclidean') -> Dict:
    start_time = timer()
    with_classification = 'with_classification' in type(model).__name__
    import ddp
    if ddp.is_distributed():
        return run_inference_sharded(model, dataset, loss_type, start_time, folder_name=folder_name)
    if folder_name:
        image_paths, image_features = utils.load_image_features(folder_name)
        inference_dataset = data_preparation.InferenceDataset(image_paths, getattr(model, "transform", None))
        feature_folder = folder_name
        print("Image features loaded from file")
    else:
        inference_dataset, image_features, feature_folder = compute_image_features(model, dataset, with_classification)
    dataloader = _loader(_Sketches(dataset))
    inference_dict = process_inference(model, dataset, inference_dataset, dataloader, image_features, start_time,
                                       with_classification, loss_type)
    if not _needs_second_pass(dataset):
        inference_dict['image_features'] = feature_folder
        return inference_dict
    inference_dict2 = _second_pass(model, dataset, inference_dataset, image_features, inference_dict,
                                   with_classification, loss_type)
    return {'image_features': feature_folder, 'drawing_stats': inference_dict, 'sketch_stats': inference_dict2}


def run_inference_sharded(model, dataset, loss_type='euclidean', start_time=None, folder_name: str = None,
                          **search) -> Dict:
    """run_inference with one process per GPU: sharded gallery embedding and
    shard-parallel retrieval; every rank returns the same dictionary, rank 0
    wrote the feature file (its path is broadcast).  With a feature folder
    (--feature_folder) every rank reads the file and keeps only its contiguous
    row shard, so the retrieval stays sharded instead of every rank scanning
    the whole gallery."""
    import torch.distributed as dist
    import ddp
    start_time = timer() if start_time is None else start_time
    with_classification = 'with_classification' in type(model).__name__
    # every rank embeds its shard with the same eval model: rank 0's BatchNorm
    # running statistics (each rank's own came from its own minibatches)
    ddp.broadcast_buffers(model)
    if folder_name:
        image_paths, image_features = utils.load_image_features(folder_name)
        inference_dataset = data_preparation.InferenceDataset(image_paths, getattr(model, "transform", None))
        b = shard_bounds(len(inference_dataset), dist.get_world_size())
        r = dist.get_rank()
        shard = torch.as_tensor(image_features)[b[r]:b[r + 1]].to(device)
        g_base = b[r]
        feature_folder = folder_name
        print("Image features loaded from file")
    else:
        inference_dataset, shard, g_base, feature_path = compute_image_features_sharded(model, dataset,
                                                                                        with_classification)
        box = [str(feature_path) if feature_path is not None else None]
        dist.broadcast_object_list(box, src=0)
        feature_folder = box[0]
    first = process_inference_sharded(model, dataset, inference_dataset, _Sketches(dataset), shard, g_base,
                                      start_time, with_classification, loss_type, **search)
    if not _needs_second_pass(dataset):
        first['image_features'] = feature_folder
        return first
    second = _second_pass(model, dataset, inference_dataset, None, first, with_classification, loss_type,
                          sharded=(shard, g_base), **search)
    return {'image_features': feature_folder, 'drawing_stats': first, 'sketch_stats': second}


class _Sketches(torch.utils.data.Dataset):
    """the sketch element of each triplet (the reference draws full triplets with batch 1)."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        if hasattr(self.ds, "sketch"):
            return self.ds.sketch(i)
        return self.ds[i][0]


def main(argv=None):
    parser = argparse.ArgumentParser(description='recomputes Inference for given folder')
    parser.add_argument('--folder', default=None, help="Folder on which rerunning inference")
    parser.add_argument('-a', '--all', action="store_true",
                        help="Rerun inference for all Modified_ResNet* models where results folder exist")
    args = parser.parse_args(argv)
    import ddp
    import os
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        ddp.init_distributed()  # torchrun: gallery embedding and retrieval sharded over the ranks
    rank0 = int(os.environ.get("RANK", "0")) == 0
    folders = [] if not args.folder else [args.folder]
    if args.all:
        folders = [p.stem for p in Path("./models").glob("ModifiedResNet*.pth")]
    print(folders, flush=True)
    for folder in folders:
        model_file = folder + '.pth'
        model_type = folder.split('_')[0] if len(folder.split('_')) == 4 else "ModifiedResNet_with_classification"
        if not Path(f"models/{model_file}").is_file():
            print(f"Model {model_file} is not available", flush=True)
            continue
        if not Path(f"results/{folder}").is_dir():
            print(f"Results {folder} are not available", flush=True)
            continue
        with open(Path("results") / folder / "data_params.json") as f:
            data_dict = json.load(f)
        with open(Path("results") / folder / "training_params.json") as f:
            param_dict = json.load(f)
        dataset = data_dict['dataset']
        model = utils.load_model(model_file, dataset=dataset, model_type=model_type).to(device)
        _, test_dataset = data_preparation.get_datasets(dataset=dataset, size=data_dict.get('size', 1.0),
                                                        transform=model.transform)
        inference_dict = run_inference(model, test_dataset, None, param_dict.get('loss_type', 'euclidean'))
        if not rank0:
            continue
        with open(Path("results") / folder / "inference_updated.json", "w") as f:
            json.dump(inference_dict, f, indent=4)
        import visualization
        visualization.visualize(Path("results") / folder, None, inference_dict)  # inference.py:242
        print(f"RUN INFERENCE FOR {folder}", flush=True)


if __name__ == "__main__":
    main()
