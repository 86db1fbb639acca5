"""Drop-in for /root/reference/inference.py on MI355X.

Same functions and result dictionary as the reference:
  get_ranking_position   inference.py:30-57   (name parsing -> positive -> rank)
  get_topk_images        inference.py:60-69
  compute_image_features inference.py:72-92   (eval-mode gallery embedding, batches of 50)
  process_inference      inference.py:94-136  (rank+1, MRR, topk_acc, describe() stats,
                                               10 retrieval samples chosen by random.seed(11))
  run_inference          inference.py:140-165
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


@torch.no_grad()
def _embed(model, loader, with_classification):
    feats = []
    for batch in loader:
        x = batch[0] if isinstance(batch, (list, tuple)) else batch
        out = model(x.to(device))
        feats.append(out[0] if with_classification else out)
    return torch.cat(feats) if feats else torch.empty(0)


def compute_image_features(model, dataset, with_classification: bool):
    inference_dataset = data_preparation.InferenceDataset(dataset.photo_paths, dataset.transform,
                                                          getattr(dataset, "resolution", 224))
    loader = DataLoader(inference_dataset, batch_size=50, num_workers=0, shuffle=False)
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


def process_inference(model, dataset, inference_dataset, dataloader, image_features, start_time,
                      with_classification, loss_type):
    k = 10
    random.seed(11)
    random_indices = [random.randrange(0, len(dataset)) for _ in range(10)]
    image_features = image_features.to(device)
    model.to(device)
    model.eval()
    paths = inference_dataset.image_paths
    with torch.no_grad():
        sketch_features = _embed(model, dataloader, with_classification)
    positives = []
    for sp in dataset.sketch_paths:
        name = sketch_target_name(sp, paths)
        positives.append(utils.find_image_index(paths, name) if name is not None else -1)
    pos_t = torch.tensor(positives, dtype=torch.int64, device=device)
    idx, dist, rank, _ = _search(sketch_features, image_features, k, pos_t, loss_type)
    ranks = [int(r) if p >= 0 else len(paths) for r, p in zip(rank.tolist(), positives)]
    for sp, p in zip(dataset.sketch_paths, positives):
        if p < 0:
            print(f"No image found: {sp}")
    samples = []
    for i in sorted(set(random_indices)):
        for _ in range(random_indices.count(i)):
            samples.append({str(dataset.sketch_paths[i]): [(str(paths[j]), float(d))
                                                           for j, d in zip(idx[i].tolist(), dist[i].tolist())]})
    stats = {"mean_reciprocal_rank": None, "size": len(inference_dataset), "inference_time": timer() - start_time}
    stats.update(retrieval_stats(ranks, k))
    stats["retrieval_samples"] = samples
    return stats


def run_inference(model, dataset, folder_name: str = None, loss_type='euclidean') -> Dict:
    start_time = timer()
    with_classification = 'with_classification' in type(model).__name__
    if folder_name:
        image_paths, image_features = utils.load_image_features(folder_name)
        inference_dataset = data_preparation.InferenceDataset(image_paths, getattr(model, "transform", None))
        feature_folder = folder_name
        print("Image features loaded from file")
    else:
        inference_dataset, image_features, feature_folder = compute_image_features(model, dataset, with_classification)
    dataloader = DataLoader(_Sketches(dataset), batch_size=50, num_workers=0, shuffle=False)
    inference_dict = process_inference(model, dataset, inference_dataset, dataloader, image_features, start_time,
                                       with_classification, loss_type)
    inference_dict['image_features'] = feature_folder
    return inference_dict


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
        with open(Path("results") / folder / "inference_updated.json", "w") as f:
            json.dump(inference_dict, f, indent=4)
        print(f"RUN INFERENCE FOR {folder}", flush=True)


if __name__ == "__main__":
    main()
