"""BERT-base sequence classifier on the framework's HIP kernels (reference-faithful text encoder).

Reference parity: ``BertForSequenceClassification.from_pretrained("bert-base-uncased",
num_labels=2)`` of pytorch_on_language_distr.py:151-161: 12 layers, hidden 768,
12 heads, FFN 3072 with erf-GELU, LayerNorm eps 1e-12, dropout 0.1 (embeddings, attention
probabilities, hidden states, classifier), position embeddings 512, token types 2,
pooler = tanh(Linear(768,768)) of the [CLS] token, classifier Linear(768, 2), cross-entropy when
``labels`` is given; ``forward`` returns a tuple whose first element is the loss (or the logits),
like the HF model the reference calls with ``token_type_ids=None``.

MI355X execution: Q/K/V are one fused [2304 x 768] MFMA GEMM, attention is one fused kernel per
(batch, head) with the 128x128 score tile on chip, the residual add is fused into LayerNorm.
Pretrained weights are not downloadable here (no network); ``load_hf`` maps a HF
``BertForSequenceClassification`` state (e.g. a random-init one) 1:1 for parity tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
from torch import nn

from ..ops import _lib
from ..ops.functions import cross_entropy
from ..ops.rnn import EmbeddingFn
from ..ops.transformer import BertAttentionBlockFn, BertFFNBlockFn, EmbedLayerNormFn, attention, gelu, layer_norm, tanh
from .layers import Dropout, Linear

# PCMP_BERT_FUSED=0: the op-by-op layer (separate dropout / GELU / LayerNorm-backward / bias-grad
# launches and the autograd add of h's two gradients) -- for A/B runs and parity tests
_FUSED = os.environ.get("PCMP_BERT_FUSED", "1") != "0"
_EMB_FUSED = os.environ.get("PCMP_BERT_EMB_FUSED", "1") != "0"


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    num_labels: int = 2


class _LN(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))
        self.eps = eps

    def forward(self, x, resid=None):
        return layer_norm(x, self.weight, self.bias, self.eps, resid)


def _init_linear(lin: Linear, std):
    with torch.no_grad():
        lin.weight.zero_()
        lin.weight[: lin.out_features].normal_(0.0, std)
        if lin.bias is not None:
            lin.bias.zero_()


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        d = c.hidden_size
        self.heads = c.num_attention_heads
        self.qkv = Linear(d, 3 * d)
        self.attn_out = Linear(d, d)
        self.ln1 = _LN(d, c.layer_norm_eps)
        self.ffn1 = Linear(d, c.intermediate_size)
        self.ffn2 = Linear(c.intermediate_size, d)
        self.ln2 = _LN(d, c.layer_norm_eps)
        self.p_attn = c.attention_probs_dropout_prob
        self.drop = Dropout(c.hidden_dropout_prob)
        for lin in (self.qkv, self.attn_out, self.ffn1, self.ffn2):
            _init_linear(lin, c.initializer_range)

    def forward(self, h, ids, B, S):
        if _FUSED:
            return self.forward_fused(h, ids, B, S)
        qkv = self.qkv(h)
        ctx = attention(qkv, ids, B, S, self.heads, self.p_attn if self.training else 0.0)
        a = self.drop(self.attn_out(ctx))
        h1 = self.ln1(a, h)
        f = self.drop(self.ffn2(gelu(self.ffn1(h1))))
        return self.ln2(f, h1)

    def forward_fused(self, h, ids, B, S):
        """Same math as the op-by-op path, as two fused autograd nodes (ops/transformer.py)."""
        p_attn = self.p_attn if self.training else 0.0
        p_hid = self.drop.p if self.training else 0.0
        h1 = BertAttentionBlockFn.apply(h, ids, self.qkv.weight, self.qkv.bias, self.attn_out.weight,
                                        self.attn_out.bias, self.ln1.weight, self.ln1.bias, B, S, self.heads,
                                        p_attn, p_hid, self.ln1.eps)
        return BertFFNBlockFn.apply(h1, self.ffn1.weight, self.ffn1.bias, self.ffn2.weight, self.ffn2.bias,
                                    self.ln2.weight, self.ln2.bias, p_hid, self.ln2.eps)


class BertForSequenceClassification(nn.Module):
    def __init__(self, config: BertConfig | None = None, compute_dtype=None):
        super().__init__()
        c = config or BertConfig()
        self.config = c
        d = c.hidden_size
        std = c.initializer_range
        self.word = nn.Parameter(torch.randn(c.vocab_size, d) * std)
        self.position = nn.Parameter(torch.randn(c.max_position_embeddings, d) * std)
        self.token_type = nn.Parameter(torch.randn(c.type_vocab_size, d) * std)
        with torch.no_grad():
            self.word[0].zero_()  # padding_idx 0
        self.emb_ln = _LN(d, c.layer_norm_eps)
        self.emb_drop = Dropout(c.hidden_dropout_prob)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])
        self.pooler = Linear(d, d)
        self.cls_drop = Dropout(c.hidden_dropout_prob)
        self.classifier = Linear(d, c.num_labels)
        _init_linear(self.pooler, std)
        _init_linear(self.classifier, std)
        self.compute_dtype = compute_dtype

    def _cdtype(self, device):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return _lib.default_compute_dtype(device)

    def forward_logits(self, input_ids, attention_mask=None, token_type_ids=None):
        B, S = input_ids.shape
        dt = self._cdtype(input_ids.device)
        d = self.config.hidden_size
        # key mask: attention_mask if given (reference passes ids>0), else ids > 0
        mask_ids = input_ids if attention_mask is None else attention_mask.long()
        w = EmbeddingFn.apply(input_ids, self.word, 0, dt).reshape(B * S, d)
        if token_type_ids is None and _EMB_FUSED:
            # word + position + token-type-0 rows summed inside the LayerNorm kernel
            h = EmbedLayerNormFn.apply(w, self.position, self.token_type, self.emb_ln.weight, self.emb_ln.bias,
                                       self.emb_ln.eps, S)
        else:   # eager torch broadcast (PCMP_BERT_EMB_FUSED=0: the round-3 form, for A/B runs)
            tt = self.token_type[0] if token_type_ids is None else self.token_type[token_type_ids]
            pt = (self.position[:S].unsqueeze(0) + tt).to(dt).expand(B, S, d).reshape(B * S, d)
            h = self.emb_ln(w, pt.contiguous())
        h = self.emb_drop(h)
        for layer in self.layers:
            h = layer(h, mask_ids, B, S)
        cls = h.reshape(B, S, d)[:, 0].contiguous()
        pooled = tanh(self.pooler(cls))
        return self.classifier(self.cls_drop(pooled))

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None):
        logits = self.forward_logits(input_ids, attention_mask, token_type_ids)
        if labels is not None:
            return cross_entropy(logits, labels), logits
        return (logits,)

    @torch.no_grad()
    def load_hf(self, hf):
        """Copy weights from a transformers BertForSequenceClassification (module or its state_dict)."""
        sd = hf if isinstance(hf, dict) else hf.state_dict()
        self.word.copy_(sd["bert.embeddings.word_embeddings.weight"])
        self.position.copy_(sd["bert.embeddings.position_embeddings.weight"])
        self.token_type.copy_(sd["bert.embeddings.token_type_embeddings.weight"])
        self.emb_ln.weight.copy_(sd["bert.embeddings.LayerNorm.weight"])
        self.emb_ln.bias.copy_(sd["bert.embeddings.LayerNorm.bias"])
        for i, L in enumerate(self.layers):
            p = f"bert.encoder.layer.{i}."
            wq = torch.cat([sd[p + f"attention.self.{n}.weight"] for n in ("query", "key", "value")])
            bq = torch.cat([sd[p + f"attention.self.{n}.bias"] for n in ("query", "key", "value")])
            L.qkv.load_torch(wq, bq)
            L.attn_out.load_torch(sd[p + "attention.output.dense.weight"], sd[p + "attention.output.dense.bias"])
            L.ln1.weight.copy_(sd[p + "attention.output.LayerNorm.weight"])
            L.ln1.bias.copy_(sd[p + "attention.output.LayerNorm.bias"])
            L.ffn1.load_torch(sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"])
            L.ffn2.load_torch(sd[p + "output.dense.weight"], sd[p + "output.dense.bias"])
            L.ln2.weight.copy_(sd[p + "output.LayerNorm.weight"])
            L.ln2.bias.copy_(sd[p + "output.LayerNorm.bias"])
        self.pooler.load_torch(sd["bert.pooler.dense.weight"], sd["bert.pooler.dense.bias"])
        self.classifier.load_torch(sd["classifier.weight"], sd["classifier.bias"])
        return self


def bert_base(num_labels=2, **kw):
    return BertForSequenceClassification(BertConfig(num_labels=num_labels), **kw)
