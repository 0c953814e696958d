"""Drop-in Flamed on CPU (the `--device cpu` path) vs the reference's end-to-end fixture:
PriorGenerator.sample and Flamed.sample_batch (prior -> PVA -> denoiser -> decoder), same global-RNG
draw order.  Also the text frontend and the sample() argument contract."""
import numpy as np
import pytest
import torch

from _common import golden, t32, rel_l2
from _flamed_common import build_flamed, build_codec_encoder


@pytest.fixture(scope="module")
def models():
    torch.set_num_threads(8)
    return build_flamed("cpu")


def test_prior_sample(models):
    m, _ = models
    g = golden("flamed_sample")
    with torch.inference_mode():
        torch.manual_seed(int(g["rng_seed"]))
        pe, pl, tm = m.prior_generator.sample(texts=t32(g["phonemes"]), src_lens=t32(g["src_lens"]), max_src_len=12,
                                              prompts=t32(g["prompts"]), prompts_len=20, nfe=4, temperature=0.3)
    assert np.array_equal(tm.numpy(), g["tgt_mask"])
    assert rel_l2(pe, g["prior_embs"]) < 1e-4
    assert rel_l2(pl.sum(dim=1), g["prior_logits_sum"]) < 1e-4


def test_sample_batch(models):
    m, dec = models
    g = golden("flamed_sample")
    with torch.inference_mode():
        torch.manual_seed(int(g["rng_seed"]))
        out = m.sample_batch(phonemes=t32(g["phonemes"]), src_lens=t32(g["src_lens"]), prompts=t32(g["prompts"]),
                             timbres=t32(g["timbres"]), codec_decoder=dec, temp_durgen=0.3, temp_denoiser=0.3,
                             nsteps_durgen=4, nsteps_denoiser=4)
    assert set(out) == {"prior_embs", "prior_logits", "tgt_mask", "latents", "time", "wav"}
    assert np.array_equal(out["tgt_mask"].numpy(), g["sb_tgt_mask"])
    assert rel_l2(out["latents"], g["sb_latents"]) < 1e-4
    assert out["wav"].shape == g["sb_wav"].shape
    assert rel_l2(out["wav"], g["sb_wav"]) < 1e-3


def test_sample_raw_prompt(models):
    """Flamed.sample with a raw waveform prompt: prompt encode (encoder + RVQ + timbre) -> sample_batch
    -> decode, vs the reference (flamed.py:89-166)."""
    m, dec = models
    enc = build_codec_encoder("cpu")
    g = golden("flamed_sample_raw")
    torch.manual_seed(int(g["rng_seed"]))
    res = m.sample(phonemes=t32(g["phonemes"]), prompt_raw=g["prompt"], sr=16000, codec_encoder=enc,
                   codec_decoder=dec, temp_durgen=0.3, temp_denoiser=0.3, nsteps_durgen=4, nsteps_denoiser=4)
    assert set(res) == {"wav", "time"}
    assert res["wav"].shape == g["wav"].shape
    assert rel_l2(res["wav"], g["wav"]) < 1e-3


def test_sample_argument_contract(models):
    m, dec = models
    with pytest.raises(ValueError, match="mutually exclusive"):
        m.sample(text="hi", phonemes=torch.zeros(3, dtype=torch.long), prompt_processed=torch.zeros(6, 4),
                 timbre=torch.zeros(256), codec_decoder=dec, codec_encoder=object())
    with pytest.raises(ValueError, match="timbre"):
        m.sample(text="hi", prompt_processed=torch.zeros(6, 4, dtype=torch.long), codec_decoder=dec,
                 codec_encoder=object())
    with pytest.raises(ValueError, match="codec_cfg"):
        m.sample(text="hi", prompt_processed=torch.zeros(6, 4, dtype=torch.long), timbre=torch.zeros(256))


def test_text_frontend():
    from flamed.text import text_to_sequence, sequence_to_text
    from flamed.text.symbols import symbols
    assert len(symbols) == 360
    seq = text_to_sequence("{sp HH AH0 L OW1} world 42.", ["english_cleaners"])
    assert sequence_to_text(seq) == "{sp HH AH0 L OW1} world forty two."
    m = build_flamed("cpu")[0]
    ids, _, phones = m._preprocess_english("Hello, world 12!")
    assert ids.dim() == 2 and ids.shape[1] > 5 and phones.startswith("{sp ")
