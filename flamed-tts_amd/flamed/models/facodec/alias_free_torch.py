# Adapted from https://github.com/junjun3518/alias-free-torch under the Apache License 2.0
# (via the reference's flamed/models/facodec/alias_free_torch/, which carries the same notice).
"""Alias-free activation (drop-in for reference flamed/models/facodec/alias_free_torch/{act,filter,
resample}.py): replicate-pad + 2x kaiser-sinc upsample -> activation -> 2x lowpass downsample.
The filters are state-dict buffers (`upsample.filter`, `downsample.lowpass.filter`)."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def kaiser_sinc_filter1d(cutoff, half_width, kernel_size):
    """Kaiser-windowed sinc lowpass, normalised to unit DC gain -> (1, 1, kernel_size)
    (reference filter.py:27-58)."""
    half = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    time = (torch.arange(-half, half) + 0.5) if kernel_size % 2 == 0 else (torch.arange(kernel_size) - half)
    if cutoff == 0:
        filt = torch.zeros_like(time)
    else:
        filt = 2 * cutoff * window * torch.sinc(2 * cutoff * time)
        filt = filt / filt.sum()
    return filt.view(1, 1, kernel_size)


class LowPassFilter1d(nn.Module):
    """reference filter.py:61-96"""

    def __init__(self, cutoff=0.5, half_width=0.6, stride: int = 1, padding: bool = True,
                 padding_mode: str = "replicate", kernel_size: int = 12):
        super().__init__()
        if cutoff < -0.0:
            raise ValueError("Minimum cutoff must be larger than zero.")
        if cutoff > 0.5:
            raise ValueError("A cutoff above 0.5 does not make sense.")
        self.kernel_size = kernel_size
        self.even = kernel_size % 2 == 0
        self.pad_left = kernel_size // 2 - int(self.even)
        self.pad_right = kernel_size // 2
        self.stride = stride
        self.padding = padding
        self.padding_mode = padding_mode
        self.register_buffer("filter", kaiser_sinc_filter1d(cutoff, half_width, kernel_size))

    def forward(self, x):
        C = x.shape[1]
        if self.padding:
            x = F.pad(x, (self.pad_left, self.pad_right), mode=self.padding_mode)
        return F.conv1d(x, self.filter.expand(C, -1, -1), stride=self.stride, groups=C)


class UpSample1d(nn.Module):
    """reference resample.py:9-37"""

    def __init__(self, ratio=2, kernel_size=None):
        super().__init__()
        self.ratio = ratio
        self.kernel_size = int(6 * ratio // 2) * 2 if kernel_size is None else kernel_size
        self.stride = ratio
        self.pad = self.kernel_size // ratio - 1
        self.pad_left = self.pad * self.stride + (self.kernel_size - self.stride) // 2
        self.pad_right = self.pad * self.stride + (self.kernel_size - self.stride + 1) // 2
        self.register_buffer("filter", kaiser_sinc_filter1d(0.5 / ratio, 0.6 / ratio, self.kernel_size))

    def forward(self, x):
        C = x.shape[1]
        y = F.pad(x, (self.pad, self.pad), mode="replicate")
        y = self.ratio * F.conv_transpose1d(y, self.filter.expand(C, -1, -1), stride=self.stride, groups=C)
        return y[..., self.pad_left:-self.pad_right]


class DownSample1d(nn.Module):
    """reference resample.py:40-57"""

    def __init__(self, ratio=2, kernel_size=None):
        super().__init__()
        self.ratio = ratio
        self.kernel_size = int(6 * ratio // 2) * 2 if kernel_size is None else kernel_size
        self.lowpass = LowPassFilter1d(cutoff=0.5 / ratio, half_width=0.6 / ratio, stride=ratio,
                                       kernel_size=self.kernel_size)

    def forward(self, x):
        return self.lowpass(x)


class Activation1d(nn.Module):
    """reference act.py:7-29"""

    def __init__(self, activation, up_ratio: int = 2, down_ratio: int = 2, up_kernel_size: int = 12,
                 down_kernel_size: int = 12):
        super().__init__()
        self.up_ratio = up_ratio
        self.down_ratio = down_ratio
        self.act = activation
        self.upsample = UpSample1d(up_ratio, up_kernel_size)
        self.downsample = DownSample1d(down_ratio, down_kernel_size)

    def forward(self, x):
        return self.downsample(self.act(self.upsample(x)))
