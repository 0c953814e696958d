"""FaCodec timbre transformer (drop-in for reference flamed/models/facodec/transformer.py).

Used only on the prompt-encoding path: `FACodecDecoder.forward(vq=True)`
(reference facodec.py:509-530) runs `timbre_encoder` over the encoder output and averages over time
to get the speaker embedding.  Module/attribute names match the reference so checkpoints load.

Reference behaviour kept on purpose:
  * `PositionalEncoding.forward` adds `pe[:x.size(0)]` to a batch-first (B, T, d) input, i.e. the
    *batch index* selects the position vector, broadcast over T (reference transformer.py:49-51);
  * pre-LN layers, `nn.MultiheadAttention(batch_first=True)`, FFN = Conv1d(k=5) -> ReLU -> Linear
    (reference :54-151); dropout is inactive in eval.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed.utils.conv import GemmConv1d


class StyleAdaptiveLayerNorm(nn.Module):
    """LN(x)·γ + β with (γ, β) = Linear(mean_T(condition)) (reference transformer.py:13-32)."""

    def __init__(self, normalized_shape, eps=1e-5):
        super().__init__()
        self.in_dim = normalized_shape
        self.norm = nn.LayerNorm(self.in_dim, eps=eps, elementwise_affine=False)
        self.style = nn.Linear(self.in_dim, self.in_dim * 2)
        with torch.no_grad():
            self.style.bias[: self.in_dim] = 1
            self.style.bias[self.in_dim:] = 0

    def forward(self, x, condition):
        gamma, beta = self.style(condition.mean(dim=1, keepdim=True)).chunk(2, -1)
        return gamma * self.norm(x) + beta


class PositionalEncoding(nn.Module):
    """Sinusoid table `pe` (max_len, 1, d) registered as a buffer (reference transformer.py:35-51)."""

    def __init__(self, d_model, dropout, max_len=5000):
        super().__init__()
        self.dropout = dropout
        pos = torch.arange(max_len, dtype=torch.float32).unsqueeze(1)
        freq = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
        pe = torch.zeros(max_len, 1, d_model)
        pe[:, 0, 0::2] = torch.sin(pos * freq)
        pe[:, 0, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", pe)

    def forward(self, x):
        return F.dropout(x + self.pe[: x.size(0)], self.dropout, training=self.training)


class TransformerFFNLayer(nn.Module):
    """Conv1d(d -> filter, k) -> ReLU -> Linear(filter -> d) on (B, T, d) (reference :54-83)."""

    def __init__(self, encoder_hidden, conv_filter_size, conv_kernel_size, encoder_dropout):
        super().__init__()
        self.encoder_hidden = encoder_hidden
        self.conv_filter_size = conv_filter_size
        self.conv_kernel_size = conv_kernel_size
        self.encoder_dropout = encoder_dropout
        self.ffn_1 = GemmConv1d(encoder_hidden, conv_filter_size, conv_kernel_size, padding=conv_kernel_size // 2)
        self.ffn_2 = nn.Linear(conv_filter_size, encoder_hidden)
        with torch.no_grad():
            self.ffn_1.weight.normal_(0.0, 0.02)
            self.ffn_2.weight.normal_(0.0, 0.02)

    def forward(self, x):
        h = F.relu(self.ffn_1(x.transpose(1, 2)).transpose(1, 2))
        h = F.dropout(h, self.encoder_dropout, training=self.training)
        return self.ffn_2(h)


class TransformerEncoderLayer(nn.Module):
    """Pre-LN self-attention + FFN block (reference transformer.py:86-151)."""

    def __init__(self, encoder_hidden, encoder_head, conv_filter_size, conv_kernel_size, encoder_dropout, use_cln):
        super().__init__()
        self.encoder_hidden = encoder_hidden
        self.encoder_head = encoder_head
        self.conv_filter_size = conv_filter_size
        self.conv_kernel_size = conv_kernel_size
        self.encoder_dropout = encoder_dropout
        self.use_cln = use_cln
        norm = StyleAdaptiveLayerNorm if use_cln else nn.LayerNorm
        self.ln_1 = norm(encoder_hidden)
        self.ln_2 = norm(encoder_hidden)
        self.self_attn = nn.MultiheadAttention(encoder_hidden, encoder_head, batch_first=True)
        self.ffn = TransformerFFNLayer(encoder_hidden, conv_filter_size, conv_kernel_size, encoder_dropout)

    def _ln(self, ln, x, condition):
        return ln(x, condition) if self.use_cln else ln(x)

    def forward(self, x, key_padding_mask, conditon=None):
        kpm = None if key_padding_mask is None else ~(key_padding_mask.bool())
        h = self._ln(self.ln_1, x, conditon)
        h, _ = self.self_attn(query=h, key=h, value=h, key_padding_mask=kpm)
        x = x + F.dropout(h, self.encoder_dropout, training=self.training)
        return x + self.ffn(self._ln(self.ln_2, x, conditon))


class TransformerEncoder(nn.Module):
    """Positional encoding -> N encoder layers -> final LN (reference transformer.py:154-234)."""

    def __init__(self, enc_emb_tokens=None, encoder_layer=4, encoder_hidden=256, encoder_head=4,
                 conv_filter_size=1024, conv_kernel_size=5, encoder_dropout=0.1, use_cln=False, cfg=None):
        super().__init__()
        pick = lambda v, name: v if v is not None else getattr(cfg, name)  # noqa: E731
        self.encoder_layer = pick(encoder_layer, "encoder_layer")
        self.encoder_hidden = pick(encoder_hidden, "encoder_hidden")
        self.encoder_head = pick(encoder_head, "encoder_head")
        self.conv_filter_size = pick(conv_filter_size, "conv_filter_size")
        self.conv_kernel_size = pick(conv_kernel_size, "conv_kernel_size")
        self.encoder_dropout = pick(encoder_dropout, "encoder_dropout")
        self.use_cln = pick(use_cln, "use_cln")
        self.use_enc_emb = enc_emb_tokens is not None
        if self.use_enc_emb:
            self.enc_emb_tokens = enc_emb_tokens
        self.position_emb = PositionalEncoding(self.encoder_hidden, self.encoder_dropout)
        self.layers = nn.ModuleList([
            TransformerEncoderLayer(self.encoder_hidden, self.encoder_head, self.conv_filter_size,
                                    self.conv_kernel_size, self.encoder_dropout, self.use_cln)
            for _ in range(self.encoder_layer)])
        self.last_ln = StyleAdaptiveLayerNorm(self.encoder_hidden) if self.use_cln else nn.LayerNorm(self.encoder_hidden)

    def forward(self, x, key_padding_mask, condition=None):
        if x.dim() == 2 and self.use_enc_emb:
            x = self.enc_emb_tokens(x)
        x = self.position_emb(x)
        for layer in self.layers:
            x = layer(x, key_padding_mask, condition)
        return self.last_ln(x, condition) if self.use_cln else self.last_ln(x)
