"""BiLSTM text classifier (north-star text path, BASELINE.json config 5).

Data contract kept from the reference's text pipeline (pytorch_on_language_distr.py:56-149):
token ids ``[B, 128]`` int64 (BERT vocabulary size 30522, id 0 = [PAD], padding 'post'),
``attention_mask = ids > 0`` (:84-103), 2 classes (IMDB sentiment), batch 32 per rank.

Architecture (fixed here and recorded in BASELINE.md): Embedding(30522, 256, padding_idx=0) ->
2 x bidirectional LSTM(hidden 256) -> masked mean pool over valid tokens -> Dropout(0.1) ->
Linear(512, 2).  LSTM gate order and weight layout match ``torch.nn.LSTM`` (i, f, g, o;
weight_ih [4H, Ein], weight_hh [4H, H], two biases), so ``load_torch_lstm`` maps weights 1:1.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from ..ops import _lib
from ..ops.rnn import BiLSTMLayerFn, EmbeddingFn, MaskedMeanFn
from .layers import Dropout, Linear


class Embedding(nn.Module):
    def __init__(self, num, dim, padding_idx=0):
        super().__init__()
        assert dim % 8 == 0
        w = torch.randn(num, dim)
        if padding_idx is not None:
            w[padding_idx].zero_()
        self.weight = nn.Parameter(w)
        self.padding_idx = -1 if padding_idx is None else padding_idx

    def forward(self, ids, dtype):
        return EmbeddingFn.apply(ids, self.weight, self.padding_idx, dtype)


class BiLSTMLayer(nn.Module):
    def __init__(self, in_dim, hidden):
        super().__init__()
        k = 1.0 / math.sqrt(hidden)
        self.hidden = hidden
        self.w_ih = nn.Parameter(torch.empty(8 * hidden, in_dim).uniform_(-k, k))   # [dir0 4H ; dir1 4H]
        self.b_ih = nn.Parameter(torch.empty(8 * hidden).uniform_(-k, k))
        self.b_hh = nn.Parameter(torch.empty(8 * hidden).uniform_(-k, k))
        self.w_hh = nn.Parameter(torch.empty(2, 4 * hidden, hidden).uniform_(-k, k))

    def forward(self, x, ids):
        return BiLSTMLayerFn.apply(x, ids, self.w_ih, self.b_ih, self.b_hh, self.w_hh)


class BiLSTMClassifier(nn.Module):
    def __init__(self, vocab_size=30522, embed_dim=256, hidden=256, num_layers=2, num_classes=2, dropout=0.1,
                 compute_dtype=None):
        super().__init__()
        self.embedding = Embedding(vocab_size, embed_dim, padding_idx=0)
        layers, d = [], embed_dim
        for _ in range(num_layers):
            layers.append(BiLSTMLayer(d, hidden))
            d = 2 * hidden
        self.layers = nn.ModuleList(layers)
        self.drop = Dropout(dropout)
        self.classifier = Linear(2 * hidden, num_classes)
        self.compute_dtype = compute_dtype
        self.num_classes = num_classes

    def _cdtype(self, device):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return _lib.default_compute_dtype(device)

    def forward_logits(self, input_ids, attention_mask=None):
        """``attention_mask`` is accepted for API parity; the mask is ``input_ids > 0``."""
        dt = self._cdtype(input_ids.device)
        h = self.embedding(input_ids, dt)
        for layer in self.layers:
            h = layer(h, input_ids)
        pooled = MaskedMeanFn.apply(h, input_ids)
        return self.classifier(self.drop(pooled))

    def forward(self, input_ids, attention_mask=None, labels=None):
        """HF-style: returns (loss, logits) when labels are given, else (logits,)."""
        from ..ops.functions import cross_entropy
        logits = self.forward_logits(input_ids, attention_mask)
        if labels is not None:
            return cross_entropy(logits, labels), logits
        return (logits,)

    @torch.no_grad()
    def load_torch_lstm(self, emb: nn.Embedding, lstm: nn.LSTM, fc: nn.Linear):
        self.embedding.weight.copy_(emb.weight)
        for i, L in enumerate(self.layers):
            L.w_ih.copy_(torch.cat([getattr(lstm, f"weight_ih_l{i}"), getattr(lstm, f"weight_ih_l{i}_reverse")]))
            L.b_ih.copy_(torch.cat([getattr(lstm, f"bias_ih_l{i}"), getattr(lstm, f"bias_ih_l{i}_reverse")]))
            L.b_hh.copy_(torch.cat([getattr(lstm, f"bias_hh_l{i}"), getattr(lstm, f"bias_hh_l{i}_reverse")]))
            L.w_hh.copy_(torch.stack([getattr(lstm, f"weight_hh_l{i}"), getattr(lstm, f"weight_hh_l{i}_reverse")]))
        self.classifier.load_torch(fc.weight, fc.bias)
        return self


class TorchBiLSTM(nn.Module):
    """Stock torch.nn equivalent (packed sequences) — parity reference and self-baseline."""

    def __init__(self, vocab_size=30522, embed_dim=256, hidden=256, num_layers=2, num_classes=2, dropout=0.1):
        super().__init__()
        self.embedding = nn.Embedding(vocab_size, embed_dim, padding_idx=0)
        self.lstm = nn.LSTM(embed_dim, hidden, num_layers, batch_first=True, bidirectional=True)
        self.drop = nn.Dropout(dropout)
        self.fc = nn.Linear(2 * hidden, num_classes)

    def forward(self, ids):
        lengths = (ids > 0).sum(1).clamp_min(1)
        x = self.embedding(ids)
        packed = nn.utils.rnn.pack_padded_sequence(x, lengths.cpu(), batch_first=True, enforce_sorted=False)
        out, _ = self.lstm(packed)
        out, _ = nn.utils.rnn.pad_packed_sequence(out, batch_first=True, total_length=ids.shape[1])
        m = (ids > 0).float().unsqueeze(-1)
        pooled = (out * m).sum(1) / m.sum(1).clamp_min(1.0)
        return self.fc(self.drop(pooled))
