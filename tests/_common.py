"""Shared test helpers: fixture loading and seeded state dicts (weights are never committed)."""
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "flamed-tts_amd")
GOLDEN = os.path.join(HERE, "golden")

from flamed.utils.seeded_init import fill_state_dict  # noqa: E402
from oracle import flamed_oracle as orc  # noqa: E402  (checker only)

SEED = 20251205


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def manifest(name):
    with open(os.path.join(GOLDEN, "state_dict_manifest.json")) as f:
        return json.load(f)[name]


def template(name):
    """Zero template with the reference's keys/shapes; constant buffers recomputed."""
    t = {}
    filt = orc.kaiser_sinc_filter(0.25, 0.3, 12).reshape(1, 1, 12)
    for k, shape in manifest(name).items():
        if k.endswith(".filter"):
            t[k] = filt.clone()
        elif k.endswith("position_emb.pe"):
            t[k] = orc.positional_table(shape[-1], shape[0])
        else:
            t[k] = torch.zeros(shape)
    return t


def seeded(name, seed=SEED, prefix=""):
    sd = fill_state_dict(template(name), seed)
    return {prefix + k: v for k, v in sd.items()} if prefix else sd


def t32(a):
    return torch.from_numpy(np.asarray(a))


def rel_l2(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b).clamp_min(1e-30))
