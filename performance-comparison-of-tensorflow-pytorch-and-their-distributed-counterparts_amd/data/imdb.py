"""IMDB text pipeline (pytorch_on_language_distr.py:31-149).

* ``rm_tags`` / ``read_files`` — pandas CSV reader, ``sentiment == 'positive'`` -> 1, HTML tags
  stripped (the reference's regex);
* ``split_reference`` — first 10,000 reviews train, 10,000..12,500 test (B11);
* ``encode`` — the native multithreaded pipeline ``torch.ops.pcmp.text_encode`` (BERT
  basic+WordPiece tokenisation, [CLS]/[SEP], truncation and post-padding to 128, attention
  masks) with a pure-Python fallback of identical semantics;
* ``build_vocab`` — the bert-base-uncased vocabulary cannot be downloaded here, so a WordPiece
  vocabulary with BERT's special-token ids ([PAD]=0, [UNK]=100, [CLS]=101, [SEP]=102,
  [MASK]=103) is built from corpus word frequencies (plus single characters and their '##'
  forms, so every word tokenises); a real ``vocab.txt`` is used when one is given;
* ``train_val_split`` — sklearn ``train_test_split(random_state=2020, test_size=0.1)`` applied
  identically to ids, labels and masks (B15).
"""
from __future__ import annotations

import re
import string
from collections import Counter

import torch

SPECIALS = {"[PAD]": 0, "[UNK]": 100, "[CLS]": 101, "[SEP]": 102, "[MASK]": 103}
_TAGS = re.compile(r"<[^>]+>")


def rm_tags(text):
    return _TAGS.sub(" ", text)


def read_files(path):
    import pandas as pd
    df = pd.read_csv(path)
    df["sentiment"] = (df["sentiment"] == "positive") * 1
    df["review"] = df["review"].apply(rm_tags)
    return df["review"].values, df["sentiment"].values


def split_reference(texts, labels):
    return (texts[:10000], labels[:10000]), (texts[10000:12500], labels[10000:12500])


def _native():
    from ..ops import _lib
    return _lib.load() and hasattr(torch.ops.pcmp, "text_encode")


_CJK = ((0x4E00, 0x9FFF), (0x3400, 0x4DBF), (0x20000, 0x2A6DF), (0x2A700, 0x2B73F), (0x2B740, 0x2B81F),
        (0x2B820, 0x2CEAF), (0xF900, 0xFAFF), (0x2F800, 0x2FA1F))
_WS = {0x9, 0xA, 0xB, 0xC, 0xD, 0x20, 0x85, 0xA0, 0x1680, *range(0x2000, 0x200B), 0x2028, 0x2029, 0x202F, 0x205F,
       0x3000}


def _is_punct(ch):
    import unicodedata
    cp = ord(ch)
    return (33 <= cp <= 47) or (58 <= cp <= 64) or (91 <= cp <= 96) or (123 <= cp <= 126) or \
        unicodedata.category(ch).startswith("P")


def _py_basic(text, lower=True, strip=True):
    """Pure-Python twin of the native basic tokenizer (csrc/runtime/text_core.h): HuggingFace
    BertNormalizer (clean text, isolate CJK ideographs, strip accents + lowercase) + BertPreTokenizer
    (whitespace split, punctuation isolated)."""
    import unicodedata
    if strip:
        text = rm_tags(text)
    buf = []
    for ch in text:
        cp = ord(ch)
        if ch in "\t\n\r":
            buf.append(" ")
            continue
        if cp == 0 or cp == 0xFFFD or unicodedata.category(ch)[0] == "C":
            continue
        if cp in _WS:
            buf.append(" ")
        elif any(lo <= cp <= hi for lo, hi in _CJK):
            buf.append(" " + ch + " ")
        else:
            buf.append(ch)
    text = "".join(buf)
    if lower:
        text = "".join(c.lower() for c in unicodedata.normalize("NFD", text) if unicodedata.category(c) != "Mn")
    out, cur = [], []
    for ch in text:
        if ch == " ":
            if cur:
                out.append("".join(cur)); cur = []
        elif _is_punct(ch):
            if cur:
                out.append("".join(cur)); cur = []
            out.append(ch)
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return out


def basic_tokenize(texts, lower=True, strip=True):
    texts = [str(t) for t in texts]
    if _native():
        return [s.split(" ") if s else [] for s in torch.ops.pcmp.text_basic_tokenize(texts, lower, strip)]
    return [_py_basic(t, lower, strip) for t in texts]


def build_vocab(texts, size=30522, lower=True):
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    chars = set()
    cnt = Counter()
    for toks in basic_tokenize(texts, lower):
        cnt.update(toks)
        for t in toks:
            chars.update(t)
    pieces = sorted(chars) + ["##" + c for c in sorted(chars)]
    seen = set(vocab)
    for p in pieces:
        if p not in seen:
            vocab.append(p); seen.add(p)
    for w, _ in cnt.most_common():
        if len(vocab) >= size:
            break
        if w not in seen:
            vocab.append(w); seen.add(w)
    return vocab


def load_vocab(path):
    with open(path, encoding="utf-8") as f:
        return [l.rstrip("\n") for l in f]


def _py_wordpiece(word, vmap, unk):
    if len(word) > 100:   # code points
        return [unk]
    out, start = [], 0
    while start < len(word):
        end, cur = len(word), None
        while start < end:
            sub = word[start:end]
            if start > 0:
                sub = "##" + sub
            if sub in vmap:
                cur = vmap[sub]
                break
            end -= 1
        if cur is None:
            return [unk]
        out.append(cur)
        start = end
    return out


def encode(texts, vocab, max_len=128, lower=True, strip=True, force_python=False):
    """-> (input_ids int64 [N,max_len], attention_mask int64 [N,max_len])."""
    texts = [str(t) for t in texts]
    if _native() and not force_python:
        ids, mask = torch.ops.pcmp.text_encode(texts, list(vocab), max_len, lower, strip)
        return ids, mask
    vmap = {w: i for i, w in enumerate(vocab)}
    unk, cls, sep = vmap.get("[UNK]", 100), vmap.get("[CLS]", 101), vmap.get("[SEP]", 102)
    ids = torch.zeros(len(texts), max_len, dtype=torch.long)
    for n, t in enumerate(texts):
        wp = []
        for tok in _py_basic(t, lower, strip):
            wp += _py_wordpiece(tok, vmap, unk)
            if len(wp) >= max_len:
                break
        row = [cls] + wp[: max_len - 2] + [sep]
        ids[n, : len(row)] = torch.tensor(row)
    return ids, (ids > 0).long()


def train_val_split(input_ids, labels, masks, random_state=2020, test_size=0.1):
    from sklearn.model_selection import train_test_split
    tr_i, va_i, tr_l, va_l = train_test_split(input_ids, labels, random_state=random_state, test_size=test_size)
    tr_m, va_m, _, _ = train_test_split(masks, labels, random_state=random_state, test_size=test_size)
    return (tr_i, tr_m, tr_l), (va_i, va_m, va_l)


class TensorTextDataset:
    """(ids, mask, labels) tensors; ``get_batch`` gathers rows onto the device."""

    def __init__(self, ids, mask, labels):
        self.ids = torch.as_tensor(ids, dtype=torch.long)
        self.mask = torch.as_tensor(mask, dtype=torch.long)
        self.labels = torch.as_tensor(labels, dtype=torch.long)

    def __len__(self):
        return self.ids.shape[0]

    def get_batch(self, idx, device=None):
        idx = torch.as_tensor(idx, dtype=torch.long)
        out = (self.ids[idx], self.mask[idx], self.labels[idx])
        if device is not None:
            out = tuple(t.to(device, non_blocking=True) for t in out)
        return out
