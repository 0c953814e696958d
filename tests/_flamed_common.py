"""Build the drop-in Flamed + FaCodec decoder with the fixtures' seeded weights."""
import os

import yaml

from _common import PKG, SEED, seeded
from flamed.utils.seeded_init import fill_state_dict


def build_flamed(device="cpu", dtype="f32"):
    from flamed import Flamed
    from flamed.models.facodec import FACodecDecoder
    prior = yaml.safe_load(open(os.path.join(PKG, "configs", "prior.yaml")))
    prob = yaml.safe_load(open(os.path.join(PKG, "configs", "prob.yaml")))
    m = Flamed({"prior_generator": prior, "prob_generator": prob}).eval()
    m.load_state_dict(fill_state_dict(m.state_dict(), SEED))
    dec = FACodecDecoder(in_channels=256, upsample_initial_channel=1024, up_ratios=[5, 5, 4, 2], vq_dim=256).eval()
    dec.load_state_dict(seeded("facodec_decoder"))
    m.prob_generator.denoiser.hip_dtype = dtype
    m.prior_generator.hip_dec_dtype = dtype  # decoder-side prior GEMMs (the prior encoder is always fp32)
    dec.hip_dtype = dtype
    return m.to(device), dec.to(device)


def build_codec_encoder(device="cpu"):
    from flamed.models.facodec import FACodecEncoder
    e = FACodecEncoder(ngf=32, up_ratios=[2, 4, 5, 5], out_channels=256).eval()
    e.load_state_dict(seeded("facodec_encoder"))
    return e.to(device)
