"""Label tables and top-k decoding (E3).

Reference: ``DeepLearning_standalone_trial.ipynb:388-389`` reads ImageNet's
``imagenet1000_clsidx_to_labels.txt`` (a ``{0: 'tench, Tinca tinca', 1: ...}`` listing, one class
per line) and ``Standalone_Inference_Imagenette_trial.ipynb:161-162`` defines the 10-class
Imagenette ``label_names`` dict.  The file is parsed with a regular expression -- never
``eval`` -- and plain ``one label per line`` files are accepted as well.  ``decode_topk`` is the
Keras ``decode_predictions`` equivalent (class id, label, probability) used by the single-image
sanity prediction.
"""
from __future__ import annotations

import re

import torch

from ..ops.kernels import topk_rows
from .imagefolder import IMAGENETTE_LABELS

_ENTRY = re.compile(r"""^\s*\{?\s*(\d+)\s*:\s*(['"])(.*?)\2\s*,?\s*\}?\s*$""")


def parse_label_table(text: str) -> list[str]:
    """``{idx: 'label', ...}`` listing (one entry per line) or plain one-label-per-line text."""
    entries, plain = {}, []
    for line in text.splitlines():
        if not line.strip():
            continue
        m = _ENTRY.match(line)
        if m:
            entries[int(m.group(1))] = m.group(3)
        else:
            plain.append(line.strip())
    if entries:
        n = max(entries) + 1
        missing = [i for i in range(n) if i not in entries]
        if missing:
            raise ValueError(f"label table misses class ids {missing[:5]}...")
        return [entries[i] for i in range(n)]
    return plain


def load_label_table(path: str) -> list[str]:
    with open(path, encoding="utf-8") as f:
        return parse_label_table(f.read())


def imagenette_labels() -> list[str]:
    return [IMAGENETTE_LABELS[k] for k in sorted(IMAGENETTE_LABELS)]


def decode_topk(logits_or_probs: torch.Tensor, labels: list[str] | None = None, k: int = 5,
                from_logits: bool = True):
    """Per sample, the k best (class id, label, probability) triples (Keras decode_predictions)."""
    x = logits_or_probs.float()
    p = torch.softmax(x, dim=-1) if from_logits else x
    val, idx = topk_rows(p, k)
    out = []
    for vi, ii in zip(val.tolist(), idx.tolist()):
        out.append([(c, labels[c] if labels is not None and c < len(labels) else str(c), v) for c, v in zip(ii, vi)])
    return out
