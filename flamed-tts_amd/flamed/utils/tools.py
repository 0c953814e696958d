"""Mask / padding helpers used by the PVA and prior generator (reference flamed/utils/tools.py)."""
import torch
import torch.nn.functional as F


def get_mask_from_lengths(lengths, max_len=None):
    """(B,) lengths -> (B, max_len) bool, True = padding (reference tools.py:91-99)."""
    if max_len is None:
        max_len = int(torch.max(lengths).item())
    ids = torch.arange(0, max_len, device=lengths.device).unsqueeze(0)
    return ids >= lengths.unsqueeze(1)


def pad(input_ele, mel_max_length=None):
    """Zero-pad a list of 1-D / 2-D tensors to a common length and stack (reference :299-317).
    A falsy mel_max_length means 'longest item'; longer items are truncated."""
    max_len = mel_max_length if mel_max_length else max(e.size(0) for e in input_ele)
    out = []
    for e in input_ele:
        if e.dim() == 1:
            out.append(F.pad(e, (0, max_len - e.size(0)), "constant", 0.0))
        else:
            out.append(F.pad(e, (0, 0, 0, max_len - e.size(0)), "constant", 0.0))
    return torch.stack(out)
