"""Factorized vector quantizer (drop-in for reference flamed/models/facodec/quantize/fvq.py).

Adapted from Amphion's FACodec `fvq.py` (Copyright (c) 2023 Amphion; MIT license, as the reference file
carries it): the constructor, `vq2emb`, `get_emb`, `embed_code` and `decode_code` keep Amphion's structure
because the state-dict schema and the code ids are fixed by released checkpoints.

Per frame: z_e = in_proj(z) (weight-norm Linear dim -> codebook_dim), nearest code by the
L2-normalised euclidean distance |e|^2 - 2 e.c + |c|^2 (reference fvq.py:102-116), z_q = raw codebook
row, straight-through `z_e + (z_q - z_e)` kept in that order (it is not bit-identical to z_q in fp32,
reference :74-76), then out_proj (codebook_dim -> dim).  Layout (B, D, T) in and out.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils import weight_norm


class FactorizedVectorQuantize(nn.Module):

    def __init__(self, dim, codebook_size, codebook_dim, commitment, **kwargs):
        super().__init__()
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.commitment = commitment
        if dim != codebook_dim:
            self.in_proj = weight_norm(nn.Linear(dim, codebook_dim))
            self.out_proj = weight_norm(nn.Linear(codebook_dim, dim))
        else:
            self.in_proj = nn.Identity()
            self.out_proj = nn.Identity()
        self._codebook = nn.Embedding(codebook_size, codebook_dim)

    @property
    def codebook(self):
        return self._codebook

    def forward(self, z):
        z_e = self.in_proj(z.transpose(1, 2)).transpose(1, 2)           # (B, d, T)
        z_q, indices = self.decode_latents(z_e)
        if self.training:
            commitment_loss = F.mse_loss(z_e, z_q.detach(), reduction="none").mean([1, 2]) * self.commitment
            codebook_loss = F.mse_loss(z_q, z_e.detach(), reduction="none").mean([1, 2])
            commit_loss = commitment_loss + codebook_loss
        else:
            commit_loss = torch.zeros(z.shape[0], device=z.device)
        z_q = z_e + (z_q - z_e).detach()
        z_q = self.out_proj(z_q.transpose(1, 2)).transpose(1, 2)
        return z_q, indices, commit_loss

    def vq2emb(self, vq, proj=True):
        emb = self.embed_code(vq)
        if proj:
            emb = self.out_proj(emb)
        return emb.transpose(1, 2)

    def get_emb(self):
        return self.codebook.weight

    def embed_code(self, embed_id):
        return F.embedding(embed_id, self.codebook.weight)

    def decode_code(self, embed_id):
        return self.embed_code(embed_id).transpose(1, 2)

    def decode_latents(self, latents):
        B = latents.size(0)
        enc = F.normalize(latents.transpose(1, 2).reshape(-1, latents.size(1)))
        cb = F.normalize(self.codebook.weight)
        dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cb.t() + cb.pow(2).sum(1, keepdim=True).t()
        indices = (-dist).max(1)[1].reshape(B, -1)
        return self.decode_code(indices), indices
