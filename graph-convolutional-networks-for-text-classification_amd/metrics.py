"""Evaluation metrics of the reference's trainer on the GPU, one host sync per
evaluation.

``accuracy`` / ``macro_f1`` keep the signatures and arithmetic of the
reference's utils.py:25-109 (argmax = first maximal logit; per-class
precision / recall with 0/0 -> 0, macro means, F1 from the means), but the
counts come from one gcnk_class_stats launch and one device->host copy
instead of 3 * nclass + 1 ``.item()`` syncs.  ``evaluate`` returns all four
from a single launch (what TopicGCNTrainer.val computes, trainer.py:378-398).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .sparse import require_device


def class_stats(pred, targ, idx=None):
    """int32 device tensor [3*nclass + 1] = TP | FP | FN | correct over the rows
    ``idx`` (all rows when None) of logits ``pred`` [rows x nclass]."""
    require_device(pred, "pred")
    if pred.dtype != torch.float32 or pred.dim() != 2 or pred.stride(1) != 1:
        pred = pred.float().contiguous()
    targ = targ.to(device=pred.device, dtype=torch.int64).contiguous()
    if idx is not None:
        idx = idx.to(device=pred.device, dtype=torch.int64).contiguous()
    nclass = pred.shape[1]
    n = idx.numel() if idx is not None else pred.shape[0]
    counts = torch.empty(3 * nclass + 1, dtype=torch.int32, device=pred.device)
    lib = _lib.load()
    with torch.cuda.device(pred.device):
        _lib.check(lib.gcnk_class_stats(pred.data_ptr(), pred.stride(0), targ.data_ptr(),
                                        idx.data_ptr() if idx is not None else None, n, nclass, counts.data_ptr(),
                                        ctypes.c_void_p(torch.cuda.current_stream(pred.device).cuda_stream)),
                   "gcnk_class_stats")
    return counts


def _from_counts(c, nclass, num_classes, n):
    tp, fp, fn, correct = c[:nclass], c[nclass:2 * nclass], c[2 * nclass:3 * nclass], int(c[3 * nclass])
    if num_classes is None:   # utils.py:53-54: only the classes present in the targets
        keep = (tp + fn) > 0
        tp, fp, fn = tp[keep], fp[keep], fn[keep]
    with np.errstate(divide="ignore", invalid="ignore"):
        precision = tp / (tp + fp)
        precision[np.isnan(precision)] = 0
        precision = np.mean(precision)
        recall = tp / (tp + fn)
        recall[np.isnan(recall)] = 0
        recall = np.mean(recall)
        f1 = 2 * (precision * recall) / (precision + recall)
    return correct / n, f1, precision, recall


def evaluate(pred, targ, idx=None, num_classes=None):
    """(accuracy, macro_f1, precision, recall) of utils.py:25-109 from one launch
    and one device->host copy.  ``pred``: logits [rows x nclass]; ``targ``:
    labels indexed like the rows of ``pred``; ``idx``: rows to score."""
    counts = class_stats(pred, targ, idx).cpu().numpy().astype(np.int64)
    n = idx.numel() if idx is not None else pred.shape[0]
    return _from_counts(counts, pred.shape[1], num_classes, n)


def macro_f1(pred, targ, num_classes=None):
    """utils.py:25-86 signature: (f1, precision, recall) over all rows of pred."""
    _, f1, p, r = evaluate(pred, targ, None, num_classes)
    return f1, p, r


def accuracy(pred, targ):
    """utils.py:89-109 signature: fraction of rows whose argmax equals targ."""
    return evaluate(pred, targ)[0]
