"""GPU end to end: Flamed.sample_batch with every hot-path piece on the HIP library (PVA flow +
length regulator, AdaLN + Euler solve, FaCodec decode) vs the reference's fixture.
Tolerances: f32 mode tgt_mask bit-exact, prior embeddings and latents rel-L2 <= 1e-4, waveform rel-L2
<= 2e-3 (chaotic random-weight decoder amplifies fp32 reassociation noise); bf16 mode (bf16 denoiser,
decoder-side prior GEMMs and FaCodec convs) tgt_mask exact (the prior encoder and the duration flow stay
fp32), prior embeddings <= 2e-2, latents <= 2e-2."""
import numpy as np
import pytest
import torch

from _common import golden, t32, rel_l2
from _flamed_common import build_flamed, build_codec_encoder

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("dtype,lat_tol,emb_tol", [("f32", 1e-4, 1e-4), ("bf16", 2e-2, 2e-2)])
def test_sample_batch_gpu(dtype, lat_tol, emb_tol):
    m, dec = build_flamed(DEV, dtype)
    g = golden("flamed_sample")
    with torch.inference_mode():
        torch.manual_seed(int(g["rng_seed"]))
        out = m.sample_batch(phonemes=t32(g["phonemes"]), src_lens=t32(g["src_lens"]), prompts=t32(g["prompts"]),
                             timbres=t32(g["timbres"]), codec_decoder=dec, temp_durgen=0.3, temp_denoiser=0.3,
                             nsteps_durgen=4, nsteps_denoiser=4)
    assert np.array_equal(out["tgt_mask"].cpu().numpy(), g["sb_tgt_mask"])
    e = rel_l2(out["prior_embs"].cpu(), g["sb_prior_embs"])
    print(f"{dtype}: prior_embs rel-L2 {e:.3e}")
    assert e < emb_tol
    assert rel_l2(out["latents"].cpu(), g["sb_latents"]) < lat_tol
    assert out["wav"].shape == g["sb_wav"].shape
    if dtype == "f32":
        assert rel_l2(out["wav"].cpu(), g["sb_wav"]) < 2e-3
    assert out["time"] > 0


def test_prompt_encode_gpu():
    """FaCodec encoder + RVQ codes + timbre on the GPU vs the reference fixture (codes bit-exact; the
    fixture's smallest top-2 code-distance gap is recorded as vq_gap_min)."""
    _, dec = build_flamed(DEV, "f32")
    enc = build_codec_encoder(DEV)
    g = golden("facodec_encode")
    with torch.inference_mode():
        z = enc(t32(g["wav"]).to(DEV))
        _, codes, _, _, spk = dec(t32(g["enc_out"]).to(DEV), eval_vq=False, vq=True)
    assert rel_l2(z.cpu(), g["enc_out"]) < 1e-4
    assert np.array_equal(codes.cpu().numpy(), g["codes"])
    assert rel_l2(spk.cpu(), g["spk"]) < 1e-4


def test_sample_raw_prompt_gpu():
    """Flamed.sample with a raw prompt (encode -> prior/PVA -> denoiser -> decode) on the GPU."""
    m, dec = build_flamed(DEV, "f32")
    enc = build_codec_encoder(DEV)
    g = golden("flamed_sample_raw")
    torch.manual_seed(int(g["rng_seed"]))
    res = m.sample(phonemes=t32(g["phonemes"]), prompt_raw=g["prompt"], sr=16000, codec_encoder=enc,
                   codec_decoder=dec, temp_durgen=0.3, temp_denoiser=0.3, nsteps_durgen=4, nsteps_denoiser=4)
    assert res["wav"].shape == g["wav"].shape
    assert rel_l2(res["wav"], g["wav"]) < 2e-3


def test_end_to_end_duration_flips_vs_oracle():
    """the integer durations of an end-to-end run at the bench's 5 s utterance size
    (L = 285 phonemes, --nsteps-durgen 64) from the HIP prior encoder's output: the HIP PVA flow against
    the oracle's restatement of PVA.sample's Euler loop (pva.py:97-109) on the same encoder output and the
    same CPU-RNG noise.  Zero frame flips away from .5 rounding boundaries (pva.py:111-112); log-durations
    rel-L2 <= 1e-5."""
    from _common import orc
    m, _ = build_flamed(DEV, "bf16")
    pr = m.prior_generator
    L, nfe = 285, 64
    phon = torch.randint(1, 300, (1, L), generator=torch.Generator().manual_seed(1234)).to(DEV)
    smask = torch.zeros(1, L, dtype=torch.bool, device=DEV)
    with torch.inference_mode():
        enc = pr.hip().encode(phon, smask)
        torch.manual_seed(0)
        d_g, s_g = pr.pva.flow(enc, smask, nfe, 0.3)
    sd = {"prior_generator.pva." + k: v.detach().float().cpu() for k, v in pr.pva.state_dict().items()}
    torch.manual_seed(0)
    d_c, s_c = orc.pva_flow(sd, enc.float().cpu(), smask.cpu(), nfe, 0.3)
    assert rel_l2(d_g.cpu(), d_c) < 1e-5 and rel_l2(s_g.cpu(), s_c) < 1e-5
    near, flips = 0, 0
    for got, ref in ((d_g.cpu(), d_c), (s_g.cpu(), s_c)):
        e = torch.exp(ref) - 1
        safe = (e - e.floor() - 0.5).abs() > 1e-4
        near += int((~safe).sum())
        flips += int((orc.log_to_frames(got)[safe] != orc.log_to_frames(ref)[safe]).sum())
    print(f"end-to-end L=285 nfe=64: duration flips {flips} of {2 * L}, near a .5 boundary {near}")
    assert flips == 0
