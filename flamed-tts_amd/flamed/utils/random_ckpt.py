"""Write a seeded random-init Flamed checkpoint, its config.yaml and FaCodec encoder/decoder weights.

The released checkpoints are not reachable offline; BASELINE config 0 (the CPU
plumbing run of synthesize.py) uses random-init weights.  The files have the reference layout:
  <out>/flamed.pt                   the Flamed state dict (reference keys; load with --weights-only true,
                                    synthesize.py's default)
  <out>/config.yaml                 {prior_generator, prob_generator, codec_cfg} as train.py:60-65 saves
  <out>/ns3_facodec_encoder.bin     FaCodec encoder state dict
  <out>/ns3_facodec_decoder.bin     FaCodec decoder state dict (inference keys; no predictor heads)
Weights come from flamed.utils.seeded_init (same values the parity fixtures use for a given seed).

    python -m flamed.utils.random_ckpt --out-dir /tmp/flamed_rand [--seed 20251205]
"""
from __future__ import annotations

import argparse
import os

import torch
import yaml

from flamed.utils.seeded_init import fill_state_dict

CFG_DIR = os.path.join(os.path.dirname(__file__), "..", "..", "configs")


def load_yaml(name):
    with open(os.path.join(CFG_DIR, name)) as f:
        return yaml.safe_load(f)


def codec_models(codec_cfg):
    from flamed.models.facodec import FACodecDecoder, FACodecEncoder
    e, d = codec_cfg["encoder"], codec_cfg["decoder"]
    enc = FACodecEncoder(ngf=e["ngf"], up_ratios=e["up_ratios"], out_channels=e["out_channels"])
    dec = FACodecDecoder(**{k: v for k, v in d.items() if k not in ("ckpt_filename", "device")})
    return enc, dec


def write(out_dir: str, seed: int = 20251205) -> dict:
    from flamed import Flamed
    os.makedirs(out_dir, exist_ok=True)
    cfg = {"prior_generator": load_yaml("prior.yaml"), "prob_generator": load_yaml("prob.yaml"),
           "codec_cfg": load_yaml("codec.yaml")}
    model = Flamed({"prior_generator": cfg["prior_generator"], "prob_generator": cfg["prob_generator"]})
    torch.save(fill_state_dict(model.state_dict(), seed), os.path.join(out_dir, "flamed.pt"))
    enc, dec = codec_models(cfg["codec_cfg"])
    paths = {"ckpt": os.path.join(out_dir, "flamed.pt"), "cfg": os.path.join(out_dir, "config.yaml"),
             "encoder": os.path.join(out_dir, "ns3_facodec_encoder.bin"),
             "decoder": os.path.join(out_dir, "ns3_facodec_decoder.bin")}
    torch.save(fill_state_dict(enc.state_dict(), seed), paths["encoder"])
    torch.save(fill_state_dict(dec.state_dict(), seed), paths["decoder"])
    with open(paths["cfg"], "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    return paths


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--seed", type=int, default=20251205)
    a = ap.parse_args()
    for k, v in write(a.out_dir, a.seed).items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    main()
