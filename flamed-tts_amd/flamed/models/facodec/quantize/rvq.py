"""Residual VQ over factorized quantizers (drop-in for reference quantize/rvq.py:12-87).

Eval path: residual -= quantized after every layer; the summed output, stacked indices
(n_q, B, T), per-layer losses and per-layer quantized tensors (n_q, B, D, T) are returned.  The
training-time quantizer dropout is kept for API parity.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .fvq import FactorizedVectorQuantize


class ResidualVQ(nn.Module):

    def __init__(self, *, num_quantizers, codebook_size, **kwargs):
        super().__init__()
        sizes = [codebook_size] * num_quantizers if isinstance(codebook_size, int) else list(codebook_size)
        self.layers = nn.ModuleList([FactorizedVectorQuantize(codebook_size=2 ** s, **kwargs) for s in sizes])
        self.num_quantizers = num_quantizers
        self.quantizer_dropout = kwargs.get("quantizer_dropout", 0.0)
        self.dropout_type = kwargs.get("dropout_type", None)

    def _train_n_quantizers(self, x):
        B = x.shape[0]
        n_q = torch.ones((B,)) * self.num_quantizers + 1
        if self.dropout_type == "linear":
            drop = torch.randint(1, self.num_quantizers + 1, (B,))
        else:
            drop = torch.pow(2, torch.randint(1, int(math.log2(self.num_quantizers)), (B,)))
        n_drop = int(B * self.quantizer_dropout)
        n_q[:n_drop] = drop[:n_drop]
        return n_q.to(x.device)

    def forward(self, x, n_quantizers=None):
        if n_quantizers is None:
            n_quantizers = self.num_quantizers
        if self.training:
            n_quantizers = self._train_n_quantizers(x)
        out, residual = 0.0, x
        losses, indices, quantized_all = [], [], []
        for idx, layer in enumerate(self.layers):
            if not self.training and idx >= n_quantizers:
                break
            q, ind, loss = layer(residual)
            keep = torch.full((x.shape[0],), fill_value=idx, device=x.device) < n_quantizers
            residual = residual - q
            out = out + q * keep[:, None, None]
            losses.append((loss * keep).mean())
            indices.append(ind)
            quantized_all.append(q)
        return out, torch.stack(indices), torch.stack(losses), torch.stack(quantized_all)

    def vq2emb(self, vq):
        out = 0.0
        for idx, layer in enumerate(self.layers):
            out += layer.vq2emb(vq[idx])
        return out

    def get_emb(self):
        return [layer.get_emb() for layer in self.layers]
