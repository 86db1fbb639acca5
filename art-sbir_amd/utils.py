"""Drop-in for the hot-path parts of /root/reference/utils.py on libartsbir_hip.

  find_image_index                 utils.py:22-25
  CosineLoss / cosine_distance     utils.py:31-40
  euclidean_distance               utils.py:42   (nn.PairwiseDistance(p=2, eps=1e-6))
  TripletMarginLoss_with_classification{,2}   utils.py:49-75
  MARGIN                           utils.py:77
  load_model / save_model          utils.py:132-254 (ModifiedResNet branches)
  load_image_features / save_image_features   utils.py:258-284 (same CSV files,
                                   plus an image_features.npy sidecar that loads
                                   without parsing 1M x 512 CSV numbers)
The distance / loss callables run on the GPU kernels; they raise for CPU
tensors (no silent CPU path).
"""
from __future__ import annotations

import csv
import json
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np
import torch
from torch import nn

import _hip
import losses
import models
from _hip import call, ptr

MARGIN = 0.2  # Sketching without Worrying (utils.py:77)


def find_image_index(image_paths: List[Path], sketch_name: str) -> int:
    for idx, path in enumerate(image_paths):
        if Path(path).stem == sketch_name:
            return idx
    return -1


class PairwiseDistance(nn.Module):
    """nn.PairwiseDistance(p=2, eps=1e-6, keepdim=False) on the GPU: ||x1 - x2 + eps||."""

    def __init__(self, p: float = 2.0, eps: float = 1e-6, keepdim: bool = False):
        super().__init__()
        if p != 2.0:
            raise NotImplementedError("only p=2 (utils.py:42)")
        self.p, self.eps, self.keepdim = p, eps, keepdim

    def forward(self, x1, x2):
        if not (x1.is_cuda and x2.is_cuda):
            raise RuntimeError("euclidean_distance on libartsbir_hip needs CUDA tensors")
        if torch.is_grad_enabled() and (x1.requires_grad or x2.requires_grad):
            return losses.pairwise_l2_autograd(x1, x2, self.eps)
        a = x1.detach().contiguous().float().reshape(-1, x1.shape[-1])
        b = x2.detach().contiguous().float().reshape(-1, x2.shape[-1])
        n = max(a.shape[0], b.shape[0])
        out = torch.empty(n, dtype=torch.float32, device=a.device)
        call("artsbir_pairwise_l2", ptr(a), a.shape[0], ptr(b), b.shape[0], a.shape[1], self.eps, ptr(out),
             _hip.stream())
        return out.unsqueeze(-1) if self.keepdim else out


class CosineLoss(nn.Module):
    """1 - cos(x1, x2) along dim 1 (utils.py:31-38)."""

    def forward(self, sketch_tensor, image_tensor):
        return losses.cosine_distance(sketch_tensor, image_tensor)


cosine_distance = CosineLoss()
euclidean_distance = PairwiseDistance(p=2, keepdim=False)


class TripletMarginLoss_with_classification(nn.Module):
    """triplet + w * (CE(cs, labels) + CE(cp, labels))  (utils.py:49-60)."""

    def __init__(self, margin, classification_weight=0.5, distance_f=euclidean_distance):
        super().__init__()
        self.classification_weight = classification_weight
        self.classification_weight2 = 0
        self.margin = margin
        self.triplet_loss = losses.TripletMarginWithDistanceLoss(margin=margin, distance_function=distance_f)
        self.classification_loss = losses.CrossEntropyLoss()

    def forward(self, s_logits, p_logits, n_logits, cs_logits, cp_logits, labels):
        return self.triplet_loss(s_logits, p_logits, n_logits) + self.classification_weight * (
            self.classification_loss(cs_logits, labels) + self.classification_loss(cp_logits, labels))


class TripletMarginLoss_with_classification2(nn.Module):
    """triplet + w*CE(styles) + w2*CE(genres)  (utils.py:62-75)."""

    def __init__(self, margin, classification_weight=0.25, classification_weight2=0.5, distance_f=euclidean_distance):
        super().__init__()
        self.classification_weight = classification_weight
        self.classification_weight2 = classification_weight2
        self.margin = margin
        self.triplet_loss = losses.TripletMarginWithDistanceLoss(margin=margin, distance_function=distance_f)
        self.classification_loss = losses.CrossEntropyLoss()

    def forward(self, s_logits, p_logits, n_logits, cs_logits, cp_logits, cs_logits2, cp_logits2, labels, labels2):
        c1 = self.classification_loss(cs_logits, labels) + self.classification_loss(cp_logits, labels)
        c2 = self.classification_loss(cs_logits2, labels2) + self.classification_loss(cp_logits2, labels2)
        return self.triplet_loss(s_logits, p_logits, n_logits) + self.classification_weight * c1 + \
            self.classification_weight2 * c2


# ----------------------------------------------------------------- model IO
DATASETS_V1 = ['SketchyV1', 'SketchyDatasetV1', 'Sketchy', 'KaggleV1', 'KaggleDatasetV1', 'Kaggle', 'AugmentedKaggleV1',
               'AugmentedKaggleDatasetV1', 'MixedDatasetV1', 'MixedDatasetV2', 'MixedDatasetV3', 'MixedDatasetV4']


def build_model(dataset: str = None, model_type: str = None, layers=(3, 4, 6, 3), output_dim=1024, **kw) -> nn.Module:
    """The ModifiedResNet branches of utils.load_model (utils.py:166-197), and the
    ViT-B/16 encoder of configuration C5 (model_type 'VisionTransformer')."""
    if model_type in ('VisionTransformer', 'ViT-B/16'):
        # ViT-B/16 by default; vit_width / vit_layers / patch_size select a smaller one (tests)
        width = kw.get('vit_width', 768)
        return models.VisionTransformer(kw.get('input_resolution', 224), kw.get('patch_size', 16), width,
                                        kw.get('vit_layers', 12), width // 64, output_dim)
    kw = {k: v for k, v in kw.items() if k not in ('vit_width', 'vit_layers', 'patch_size')}
    if model_type == 'ModifiedResNet' or dataset in DATASETS_V1:
        return models.ModifiedResNet(layers=layers, output_dim=output_dim, **kw)
    if model_type == 'ModifiedResNet_with_classification' and dataset in ['SketchyV2', 'SketchyDatasetV2']:
        return models.ModifiedResNet_with_classification(layers=layers, output_dim=output_dim, **kw)
    if model_type == 'ModifiedResNet_with_classification' and dataset in [
            'KaggleV2', 'KaggleDatasetV2', 'AugmentedKaggleV2', 'AugmentedKaggleDatasetV2']:
        return models.ModifiedResNet_with_classification(layers=layers, output_dim=output_dim, num_classes=70,
                                                         num_classes2=32, **kw)
    if model_type == 'ModifiedResNet_with_classification' and dataset == 'CategorizedMixedDatasetV2':
        return models.ModifiedResNet_with_classification(layers=layers, output_dim=output_dim, num_classes=33, **kw)
    if model_type == 'ModifiedResNet_with_classification':
        return models.ModifiedResNet_with_classification(layers=layers, output_dim=output_dim, **kw)
    raise Exception(f"No model found with {model_type} and {dataset}")


def load_model(name: str, dataset: str = None, model_type: str = None, max_seq_len=0, options=None) -> nn.Module:
    """utils.py:132-206 for the encoder: models/<name> state_dict -> model
    (strict=False, as the reference).  Loaded with weights_only=True."""
    path = Path("models/") / name
    model = build_model(dataset, model_type)
    if path.is_file():
        loaded = torch.load(path, map_location=torch.device('cpu'), weights_only=True)
        if not isinstance(loaded, dict):
            raise Exception(f"{path}: expected a state_dict")
        own = model.state_dict()
        shared = [k for k in loaded if k in own]
        if not shared:
            # strict=False would load nothing and train from random weights while
            # reporting a loaded checkpoint (e.g. an RN50 file for --model_type VisionTransformer)
            raise Exception(f"{path} shares no parameter name with {type(model).__name__}: wrong --model / "
                            f"--model_type?")
        skipped = len(loaded) - len(shared)
        missing = len(own) - len(shared)
        if skipped or missing:
            print(f"load_model: {len(shared)} tensors loaded, {skipped} in the file unused, {missing} of the model "
                  f"not in the file (strict=False, as utils.py:168)")
        try:
            model.load_state_dict(loaded, strict=False)
        except RuntimeError:
            # classifier-size mismatch (utils.py:179-197): load without the head, then re-create it
            head = {k: v for k, v in loaded.items() if not k.startswith("classifier")}
            model.load_state_dict(head, strict=False)
        print("Dictionary used to load model")
    else:
        print(f"Model file {path} not found: random initialisation")
    print(f"Model {name} loaded", flush=True)
    return model


def save_model(model: nn.Module, data_dict: Dict, training_dict: Dict = {}, param_dict: Dict = {},
               inference_dict: Dict = {}) -> Path:
    """utils.py:210-254: models/<Cls>_<dataset>_<ts>.pth + results/<name>/*.json"""
    date_time = datetime.now().strftime("%Y-%m-%d_%H-%M")
    model_name = f"{model.__class__.__name__}_{data_dict['dataset']}_{date_time}"
    if training_dict:
        model_path = Path("models") / f"{model_name}.pth"
        model_path.parent.mkdir(parents=True, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, model_path)
        print(f"Model saved as {model_name}.pth")
    else:
        print("No model saved")
    result_path = Path("results") / model_name
    result_path.mkdir(parents=True, exist_ok=True)
    for fname, obj in (("data_params.json", data_dict), ("training.json", training_dict),
                       ("training_params.json", param_dict), ("inference.json", inference_dict)):
        with open(result_path / fname, "w") as f:
            json.dump(obj, f, indent=4)
    print(f"Data saved in {str(result_path)}", flush=True)
    return result_path


def load_image_features(folder_name: str) -> Tuple[List[Path], torch.Tensor]:
    """utils.py:258-263 (features come back as float64, like pandas' CSV parse)."""
    path = Path("data/image_features") / folder_name
    with open(path / "image_paths.csv") as f:
        image_paths = [Path(row[0]) for row in csv.reader(f) if row]
    npy = path / "image_features.npy"
    if npy.is_file():
        feats = np.load(npy, allow_pickle=False).astype(np.float64)
    else:
        feats = np.loadtxt(path / "image_features.csv", delimiter=",", dtype=np.float64, ndmin=2)
    return image_paths, torch.from_numpy(feats)


def save_image_features(model_name: str, dataset_name: str, inference_dataset, image_features) -> str:
    """utils.py:265-284, plus image_features.npy (float32) next to the CSV."""
    feature_path = Path("data/image_features")
    date_time = datetime.now().strftime("%Y-%m-%d_%H-%M")
    feature_path = feature_path / f"{model_name}_{dataset_name}_{date_time}"
    feature_path.mkdir(parents=True, exist_ok=True)
    with open(feature_path / "image_paths.csv", "w") as f:
        csv.writer(f).writerows([[str(p)] for p in inference_dataset.image_paths])
    feats = image_features.detach().cpu().numpy()
    with open(feature_path / "image_features.csv", "w") as f:
        csv.writer(f).writerows(feats)
    np.save(feature_path / "image_features.npy", feats.astype(np.float32), allow_pickle=False)
    print(f"Image features saved in {feature_path / 'image_features.csv'}")
    return feature_path.name
