"""Classification metrics from device confusion matrices (sklearn semantics).

Replaces ``Trainer._compute_metrics`` (``trainer.py:387-443``), which copies the
predictions to the host and calls sklearn 4 + num_graphs times per batch.  The
device kernel ``vg_confusion`` counts (truth, argmax prediction) pairs per
building in one launch; this module turns the small [G, K, K] count tensor into
exactly what sklearn returns for ``average="macro", zero_division=0``:

* the label set is the union of labels present in y_true or y_pred;
* per label: precision = tp / (tp + fp), recall = tp / (tp + fn),
  f1 = 2 tp / (2 tp + fp + fn) -- 0 where the denominator is 0;
* macro = unweighted mean over that label set; accuracy = trace / total.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def scores(conf: np.ndarray) -> Tuple[float, float, float, float]:
    """(f1, precision, recall, accuracy) of one K x K confusion matrix [truth, pred]."""
    conf = np.asarray(conf, dtype=np.float64)
    tp = np.diag(conf)
    row = conf.sum(1)  # support (true count)
    col = conf.sum(0)  # predicted count
    present = (row > 0) | (col > 0)
    total = conf.sum()
    if not present.any():
        return 0.0, 0.0, 0.0, 0.0
    fp = col - tp
    fn = row - tp
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(tp + fp > 0, tp / np.maximum(tp + fp, 1e-300), 0.0)
        rec = np.where(tp + fn > 0, tp / np.maximum(tp + fn, 1e-300), 0.0)
        f1 = np.where(2 * tp + fp + fn > 0, 2 * tp / np.maximum(2 * tp + fp + fn, 1e-300), 0.0)
    acc = float(tp.sum() / total) if total > 0 else 0.0
    return float(f1[present].mean()), float(prec[present].mean()), float(rec[present].mean()), acc


def batch_metrics(conf_graphs: np.ndarray, conf_all: np.ndarray):
    """Return the tuple of ``trainer.py:443``: f1, per-graph f1 list, precision, recall, accuracy."""
    f1, prec, rec, acc = scores(conf_all)
    per_graph: List[float] = [scores(c)[0] for c in conf_graphs]
    return f1, per_graph, prec, rec, acc
