"""FastSpeech2-style FFT transformer used by the prior generator (drop-in for reference
flamed/models/module/transformer/{Models,Layers,SubLayers,Modules}.py; same state-dict keys).
Runs on PyTorch ops (out of the HIP kernel scope: SURVEY.md §8(f) f2)."""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed.utils.conv import GemmConv1d

PAD = 0


def get_sinusoid_encoding_table(n_position, d_hid, padding_idx=None):
    """(n_position, d_hid) table: angle = pos / 10000^(2*(j//2)/d_hid), sin on even j, cos on odd j
    (float64 then float32, reference Models.py:10-30)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)[None, :]
    table = pos / np.power(10000, 2 * (j // 2) / d_hid)
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    if padding_idx is not None:
        table[padding_idx] = 0.0
    return torch.FloatTensor(table)


class ScaledDotProductAttention(nn.Module):
    def __init__(self, temperature):
        super().__init__()
        self.temperature = temperature
        self.softmax = nn.Softmax(dim=2)

    def forward(self, q, k, v, mask=None):
        attn = torch.bmm(q, k.transpose(1, 2)) / self.temperature
        if mask is not None:
            attn = attn.masked_fill(mask, -np.inf)
        attn = self.softmax(attn)
        return torch.bmm(attn, v), attn


class MultiHeadAttention(nn.Module):
    """Post-norm multi-head self attention (reference SubLayers.py:8-57)."""

    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        self.attention = ScaledDotProductAttention(temperature=np.power(d_k, 0.5))
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        self.dropout = nn.Dropout(dropout)

    def forward(self, q, k, v, mask=None):
        h, dk, dv = self.n_head, self.d_k, self.d_v
        b, lq, _ = q.shape
        lk = k.shape[1]
        residual = q

        def split(x, lin, d, n):
            return lin(x).view(b, n, h, d).permute(2, 0, 1, 3).reshape(h * b, n, d)

        qh, kh, vh = split(q, self.w_qs, dk, lq), split(k, self.w_ks, dk, lk), split(v, self.w_vs, dv, lk)
        out, attn = self.attention(qh, kh, vh, mask=mask.repeat(h, 1, 1) if mask is not None else None)
        out = out.view(h, b, lq, dv).permute(1, 2, 0, 3).reshape(b, lq, h * dv)
        return self.layer_norm(self.dropout(self.fc(out)) + residual), attn


class PositionwiseFeedForward(nn.Module):
    """conv(k0) -> ReLU -> conv(k1), post-norm residual (reference SubLayers.py:60-95)."""

    def __init__(self, d_in, d_hid, kernel_size, dropout=0.1):
        super().__init__()
        self.w_1 = GemmConv1d(d_in, d_hid, kernel_size=kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = GemmConv1d(d_hid, d_in, kernel_size=kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        y = self.w_2(F.relu(self.w_1(x.transpose(1, 2)))).transpose(1, 2)
        return self.layer_norm(self.dropout(y) + x)


class FFTBlock(nn.Module):
    """reference Layers.py:11-30"""

    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)

    def forward(self, enc_input, mask=None, slf_attn_mask=None):
        out, attn = self.slf_attn(enc_input, enc_input, enc_input, mask=slf_attn_mask)
        out = out.masked_fill(mask.unsqueeze(-1), 0)
        out = self.pos_ffn(out).masked_fill(mask.unsqueeze(-1), 0)
        return out, attn


def _stack(tc, prefix, n_layers):
    d = tc[f"{prefix}_hidden"]
    h = tc[f"{prefix}_head"]
    return nn.ModuleList([FFTBlock(d, h, d // h, d // h, tc[f"{prefix}_conv_filter_size"],
                                   tc[f"{prefix}_conv_kernel_size"], dropout=tc[f"{prefix}_dropout"])
                          for _ in range(n_layers)])


class Encoder(nn.Module):
    """Phoneme embedding + sinusoid positions + FFT blocks (reference Models.py:33-100)."""

    def __init__(self, config, n_symbols=None):
        super().__init__()
        tc = config["transformer"]
        if n_symbols is None:
            from flamed.text.symbols import symbols
            n_symbols = len(symbols)
        self.max_seq_len = tc["encoder_max_seq_len"]
        self.d_model = tc["encoder_hidden"]
        self.src_word_emb = nn.Embedding(n_symbols + 1, self.d_model, padding_idx=PAD)
        self.position_enc = nn.Parameter(get_sinusoid_encoding_table(self.max_seq_len + 1, self.d_model).unsqueeze(0),
                                         requires_grad=False)
        self.layer_stack = _stack(tc, "encoder", tc["encoder_layer"])

    def forward(self, src_seq, mask, return_attns=False):
        b, n = src_seq.shape
        attn_mask = mask.unsqueeze(1).expand(-1, n, -1)
        if not self.training and n > self.max_seq_len:
            pos = get_sinusoid_encoding_table(n, self.d_model)[:n].unsqueeze(0).to(src_seq.device)
        else:
            pos = self.position_enc[:, :n, :]
        x = self.src_word_emb(src_seq) + pos.expand(b, -1, -1)
        for layer in self.layer_stack:
            x, _ = layer(x, mask=mask, slf_attn_mask=attn_mask)
        return x


class Decoder(nn.Module):
    """Sinusoid positions + FFT blocks over an embedded sequence (reference Models.py:103-171)."""

    def __init__(self, config, n_layers):
        super().__init__()
        tc = config["transformer"]
        self.max_seq_len = tc["decoder_max_seq_len"]
        self.d_model = tc["decoder_hidden"]
        self.position_enc = nn.Parameter(get_sinusoid_encoding_table(self.max_seq_len + 1, self.d_model).unsqueeze(0),
                                         requires_grad=False)
        self.layer_stack = _stack(tc, "decoder", n_layers)

    def forward(self, enc_seq, mask, return_attns=False):
        b, n = enc_seq.shape[0], enc_seq.shape[1]
        if not self.training and n > self.max_seq_len:
            attn_mask = mask.unsqueeze(1).expand(-1, n, -1)
            x = enc_seq + get_sinusoid_encoding_table(n, self.d_model)[:n].unsqueeze(0).expand(b, -1, -1).to(enc_seq.device)
        else:
            n = min(n, self.max_seq_len)
            x = enc_seq[:, :n, :] + self.position_enc[:, :n, :].expand(b, -1, -1)
            mask = mask[:, :n]
            attn_mask = mask.unsqueeze(1).expand(-1, n, -1)
        for layer in self.layer_stack:
            x, _ = layer(x, mask=mask, slf_attn_mask=attn_mask)
        return x, mask
