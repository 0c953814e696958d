"""Seeded, order-independent random initialisation of Flamed / FaCodec state dicts.

The released Flamed and FaCodec checkpoints are not available offline, so every
parity fixture, test and benchmark runs on *seeded random* weights.  The reference's own init is
degenerate for the hot path: `SimpleMLPAdaLN.initialize_weights` zeroes every AdaLN projection and
`final_layer.conv_out` (reference `flamed/models/synthesizer/prob_generator.py:338-347`), so an
as-initialised denoiser returns exactly 0.  This filler replaces *every* parameter by a value that
depends only on (seed, key, shape) — never on dict order — so the reference model (fixture
generation in this container) and this package's modules (GPU box) get bit-identical weights.

Rules (by key, applied to a template state dict whose keys/shapes define the model):
  * buffers that are deterministic constants are kept from the template: alias-free resampling
    filters (`*.filter`, reference `alias_free_torch/filter.py:27-58`) and sinusoid position tables
    (`position_enc`, FaCodec `position_emb.pe`, reference `facodec/transformer.py:35-51`);
  * SnakeBeta `alpha` / `beta` (log-scale) -> 0.1·N(0,1);
  * other 1-D `weight` (norm gains) -> 1 + 0.1·N(0,1); 1-D `bias` / `*_bias` -> 0.05·N(0,1);
  * weight-norm `weight_g` -> ||weight_v|| over all dims but 0 (effective weight = weight_v);
  * everything else -> N(0,1)/sqrt(numel/shape[0]).
Pure torch on CPU; no GPU, no reference code.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Mapping

import torch

_KEEP_SUBSTRINGS = ("position_enc", "position_emb.pe")


def _gen(seed: int, key: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((int(seed) * 1_000_003 + zlib.crc32(key.encode("utf-8"))) & 0x7FFF_FFFF_FFFF)
    return g


def _is_kept(key: str) -> bool:
    return key.endswith(".filter") or any(s in key for s in _KEEP_SUBSTRINGS) \
        or key.endswith("num_batches_tracked")


def seeded_value(key: str, template: torch.Tensor, seed: int) -> torch.Tensor:
    shape = tuple(template.shape)
    if not template.is_floating_point():
        return template.clone()
    g = _gen(seed, key)
    leaf = key.rsplit(".", 1)[-1]
    if leaf in ("alpha", "beta") and len(shape) == 1:
        return 0.1 * torch.randn(shape, generator=g)
    if len(shape) <= 1:
        if leaf == "bias" or leaf.endswith("_bias"):
            return 0.05 * torch.randn(shape, generator=g)
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    fan_in = max(1, math.prod(shape[1:]))
    return torch.randn(shape, generator=g) / math.sqrt(fan_in)


def fill_state_dict(template: Mapping[str, torch.Tensor], seed: int) -> Dict[str, torch.Tensor]:
    """Return a new fp32 state dict with the template's keys, seeded as described above."""
    out: Dict[str, torch.Tensor] = {}
    for key, t in template.items():
        if _is_kept(key) or key.endswith(".weight_g"):
            out[key] = t.detach().clone().cpu()
        else:
            out[key] = seeded_value(key, t.detach().cpu(), seed).to(t.dtype)
    for key in list(out):
        if key.endswith(".weight_g"):
            v = out[key[: -len("_g")] + "_v"]
            dims = tuple(range(1, v.dim()))
            out[key] = torch.linalg.vector_norm(v, dim=dims, keepdim=True).to(out[key].dtype)
    return out


def scale_weight_norm_gains(sd: Mapping[str, torch.Tensor], gain: float) -> Dict[str, torch.Tensor]:
    """Scale every weight-norm gain (`*.weight_g`) by `gain`: effective conv weights x gain.  Used for
    the non-saturating FaCodec decoder fixture (tests/golden/make_golden.py, CALM_GAIN)."""
    return {k: (v * gain if k.endswith(".weight_g") else v) for k, v in sd.items()}


def randomize_module(module: torch.nn.Module, seed: int) -> torch.nn.Module:
    """Load seeded weights into `module` in place (keys from its own state_dict)."""
    sd = fill_state_dict(module.state_dict(), seed)
    module.load_state_dict(sd)
    return module
