"""Result figures of a training / inference run (/root/reference/visualization.py:
visualize at :262-273 and the three figure kinds it draws, :83-113 loss curves,
:128-155 top-k accuracy bars, :196-241 retrieval-sample grids).

Same files in the result folder as the reference: loss_curves[.png],
loss_curves_iter, retrieval_samples[_original], topk_accuracy — or, for the
nested Kaggle/Mixed result, the _drawings / _sketches variants.  Images of the
synthetic datasets (no files on disk) are rendered from their generator; real
image files are read with PIL.  matplotlib runs headless (Agg); seaborn's
despine is done by hand (seaborn is not installed)."""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List

import numpy as np


class Color:
    BLACK = (0, 0, 0)
    BLUE = (55 / 256, 88 / 256, 136 / 256)
    GREEN = (141 / 256, 201 / 256, 20 / 256)
    YELLOW = (227 / 256, 193 / 256, 0)
    LIGHT_GREY = (240 / 256, 240 / 256, 240 / 256)


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _save(plt, file: Path):
    file = Path(file)
    file.parent.mkdir(parents=True, exist_ok=True)
    plt.savefig(fname=file.with_suffix(".png") if not file.suffix else file, dpi=100, bbox_inches='tight')
    plt.close("all")


def _despine(ax):
    for side in ("left", "bottom", "right", "top"):
        ax.spines[side].set_visible(False)


def show_loss_curves(train_losses: List[float], test_losses: List[float], filename: Path, title=None,
                     x_label='Epoch') -> None:
    plt = _plt()
    if x_label == 'Iteration':
        xs = np.arange(10000, (len(train_losses) + 1) * 10000, 10000)
    else:
        xs = np.arange(1, len(train_losses) + 1, 1)
    fig, ax = plt.subplots(figsize=(7, 3.5))
    ax.plot(xs, train_losses, c=Color.YELLOW, label="Train loss")
    ax.plot(xs, test_losses[:len(xs)], c=Color.BLUE, label="Test loss")
    if title:
        plt.title(title)
    plt.xlabel("Epoch")
    plt.ylabel("Loss")
    plt.legend()
    ax.grid(True, color=Color.LIGHT_GREY)
    ax.tick_params(direction="in", length=0)
    ax.set_axisbelow(True)
    _despine(ax)
    _save(plt, filename)


def show_topk_accuracy(topk_acc: List[float], filename: Path, title: str = None) -> None:
    plt = _plt()
    labels = [f"top-{k}" for k in range(1, len(topk_acc) + 1)]
    acc = [x * 100 for x in topk_acc]
    fig, ax = plt.subplots(figsize=(10, 4))
    bars = ax.bar(labels, acc, color=Color.BLUE, label="Sketches")
    ax.bar_label(bars, [f"{round(a, 1):.1f}" for a in acc], padding=2, size=13)
    if title:
        plt.title(title)
    plt.ylabel("Accuracy (%)")
    plt.xlabel("Top-k positions")
    plt.legend()
    plt.ylim([0, 100])
    ax.grid(True, color=Color.LIGHT_GREY)
    ax.tick_params(direction="in", length=0)
    ax.set_axisbelow(True)
    _despine(ax)
    _save(plt, filename)


def _image(path: Path, query: bool, photo_hint=None) -> np.ndarray:
    """HxWx3 in [0, 1]: the file if it exists, else the synthetic dataset's render"""
    if path.is_file():
        from PIL import Image
        return np.asarray(Image.open(path).convert("RGB"), dtype=np.float32) / 255.0
    import data_preparation as dp
    res = 64
    t = dp.synthetic_sketch(path, photo_hint or path, res) if query else dp.synthetic_photo(path, res)
    img = t.numpy() * dp.STD + dp.MEAN  # undo the CLIP normalize
    return np.clip(img.transpose(1, 2, 0), 0.0, 1.0)


def _frame(ax, color, lw):
    for side in ("left", "bottom", "right", "top"):
        ax.spines[side].set_visible(True)
        ax.spines[side].set_color(color)
        ax.spines[side].set_linewidth(lw)


def show_retrieval_samples(samples: List[Dict], show_original: bool = False, filename: Path = None,
                           title: str = None) -> None:
    """one row per sample: the query, then its top-10; the correct photo framed green"""
    if not samples:
        return
    plt = _plt()
    rows, cols = len(samples), 11
    fig, axes = plt.subplots(nrows=rows, ncols=cols, figsize=(cols, rows + 0.4), squeeze=False)
    for i, sample in enumerate(samples):
        (sketch_path, top), = sample.items()
        sketch_path = Path(sketch_path)
        parts = sketch_path.stem.split("-")
        target = parts[1] if len(parts) == 3 else parts[0]
        hint = None
        for p, _ in top:  # the synthetic sketch is drawn from its photo
            if Path(p).stem.split('-')[0] == target:
                hint = Path(p)
        for j, ax in enumerate(axes[i]):
            ax.set_xticks([])
            ax.set_yticks([])
            _despine(ax)
            if j == 0:
                ax.imshow(_image(sketch_path, True, hint))
                _frame(ax, Color.BLACK, 0.4)
            elif j - 1 < len(top):
                p = Path(top[j - 1][0])
                ax.imshow(_image(p, False))
                if p.stem.split('-')[0] == target:
                    _frame(ax, Color.GREEN, 2.0)
            if i == 0:
                ax.set_title('Query' if j == 0 else str(j), fontdict={'fontsize': 10})
    plt.suptitle(title or "Retrieval samples")
    _save(plt, filename)


def visualize(folder_path: Path, training_dict: Dict = None, inference_dict: Dict = None) -> None:
    """visualization.py:262-273: the figures of one run into its result folder"""
    folder_path = Path(folder_path)
    training_dict = training_dict or {}
    inference_dict = inference_dict or {}
    if training_dict:
        show_loss_curves(training_dict["train_losses"], training_dict['test_losses'], folder_path / "loss_curves")
    if training_dict and training_dict.get('iteration_loss_frequency', 0) > 0 and training_dict["itrain_losses"]:
        show_loss_curves(training_dict["itrain_losses"], training_dict["itest_losses"],
                         folder_path / "loss_curves_iter", x_label="Iteration")
    if len(inference_dict.keys()) > 3:  # one inference pass
        show_retrieval_samples(inference_dict['retrieval_samples'], False, folder_path / 'retrieval_samples')
        show_retrieval_samples(inference_dict['retrieval_samples'], True, folder_path / 'retrieval_samples_original')
        show_topk_accuracy(inference_dict['topk_acc'], folder_path / 'topk_accuracy')
    elif len(inference_dict.keys()) == 3:  # Kaggle / Mixed: drawings and sketches
        show_retrieval_samples(inference_dict['drawing_stats']['retrieval_samples'], False,
                               folder_path / 'retrieval_samples_drawings', title="Retrieval samples (Drawings)")
        show_retrieval_samples(inference_dict['sketch_stats']['retrieval_samples'], False,
                               folder_path / 'retrieval_samples_sketches', title="Retrieval samples (Sketches)")
        show_topk_accuracy(inference_dict['drawing_stats']['topk_acc'], folder_path / 'topk_accuracy_drawings',
                           title="Top_k accuracy (Drawings)")
        show_topk_accuracy(inference_dict['sketch_stats']['topk_acc'], folder_path / 'topk_accuracy_sketches',
                           title="Top_k accuracy (Sketches)")
