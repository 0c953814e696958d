"""Conv1d as a plain GEMM on ROCm devices.

`GemmConv1d` is an `nn.Conv1d` (same parameters, same state-dict keys, same init) whose forward on a
CUDA (ROCm) tensor runs the convolution as im2col + one matmul (hipBLASLt) instead of MIOpen.  MIOpen
compiles / searches a solver per problem shape, and in TTS inference every utterance brings a new
sequence length: on a fresh box that cost ~50 ms per new length in the prior decoders' k=3 FFN convs
(tools/e2e_profile.py, fixed vs varying T).  A GEMM has no per-shape compile.  fp32 throughout (same
math as F.conv1d; only the summation order differs).  CPU tensors use F.conv1d unchanged.
Used on the paths that stay on PyTorch ops (prior transformer, condition fold, timbre transformer);
the hot path (denoiser, PVA, FaCodec decoder) runs in the HIP library.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv1d_gemm(x: torch.Tensor, weight: torch.Tensor, bias, stride: int = 1, padding: int = 0,
                dilation: int = 1) -> torch.Tensor:
    """x (B, Cin, T), weight (Cout, Cin, k) -> (B, Cout, T_out); groups = 1, zero padding."""
    B, Cin, T = x.shape
    Cout, _, k = weight.shape
    if k == 1 and stride == 1 and padding == 0:
        y = torch.matmul(weight[:, :, 0], x)                                   # (B, Cout, T)
        return y if bias is None else y + bias[:, None]
    xp = F.pad(x, (padding, padding)) if padding else x
    span = (k - 1) * dilation + 1
    cols = xp.unfold(2, span, stride)                                          # (B, Cin, T_out, span)
    if dilation > 1:
        cols = cols[..., ::dilation]
    T_out = cols.shape[2]
    cols = cols.permute(0, 2, 1, 3).reshape(B * T_out, Cin * k)
    y = torch.addmm(bias, cols, weight.reshape(Cout, Cin * k).t()) if bias is not None \
        else cols @ weight.reshape(Cout, Cin * k).t()
    return y.view(B, T_out, Cout).transpose(1, 2)


class GemmConv1d(nn.Conv1d):
    """nn.Conv1d with a GEMM forward on ROCm devices (groups = 1, zero padding)."""

    def forward(self, x):
        if x.is_cuda and self.groups == 1 and self.padding_mode == "zeros" and isinstance(self.padding, tuple):
            return conv1d_gemm(x, self.weight, self.bias, self.stride[0], self.padding[0], self.dilation[0])
        return super().forward(x)
