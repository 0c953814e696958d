"""GPU parity: HIP FaCodec decoder (FACodecDecoder.inference) vs reference golden waveforms and the
oracle.

* Seeded unit-gain weights (golden `facodec`): the decoder is chaotic there (~85-90 % of samples
  saturate the tanh); f32 mode per-sample max |diff| <= 5e-4; bf16 SNR no worse than the reference's
  own bf16 behaviour (oracle under torch.autocast(cpu, bfloat16)) minus 1 dB.
* Non-saturating weights (golden `facodec_calm`, weight-norm gains x 0.6; output std 0.04, no
  saturation): SURVEY.md §8(c)'s absolute bars — f32 max |diff| <= 5e-3 (measured far below), bf16
  SNR >= 30 dB — at T = 64 against the reference fixture and at the bench length T = 400 (80,000
  samples, the bench's bf16 decode) against the oracle."""
import math

import numpy as np
import pytest
import torch

from _common import golden, seeded, t32, rel_l2, orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _dec(dtype):
    from flamed.models.facodec import FACodecDecoder
    d = FACodecDecoder(in_channels=256, upsample_initial_channel=1024, ngf=32, up_ratios=[5, 5, 4, 2],
                       vq_num_q_c=2, vq_num_q_p=1, vq_num_q_r=3, vq_dim=256, codebook_dim=8,
                       use_gr_x_timbre=True, use_gr_residual_f0=True, use_gr_residual_phone=True).eval()
    sd = seeded("facodec_decoder")
    d.load_state_dict(sd)
    d.hip_dtype = dtype
    return d.to(DEV), sd


@pytest.fixture(scope="module")
def dec_f32():
    return _dec("f32")


@pytest.fixture(scope="module")
def dec_bf16():
    return _dec("bf16")


def snr_db(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    return 10 * math.log10(np.sum(ref ** 2) / max(np.sum((x - ref) ** 2), 1e-30))


def ref_bf16_snr(sd, lat, spk, ref):
    with torch.autocast("cpu", dtype=torch.bfloat16):
        w = orc.facodec_decode(sd, t32(lat), t32(spk)).float().numpy()
    return snr_db(w, ref)


def _run(dec, lat, spk):
    with torch.inference_mode():
        return dec.inference(t32(lat).to(DEV), t32(spk).to(DEV)).cpu().numpy()


def test_state_dict_schema_and_extra_keys(dec_f32):
    d, sd = dec_f32
    assert set(d.state_dict().keys()) <= set(sd.keys())
    assert all(k.split(".")[0] in ("model", "timbre_linear", "timbre_encoder", "quantizer") for k in d.state_dict())
    assert len(d.unused_state) == len(sd) - len(d.state_dict())
    assert all(k.split(".")[0].endswith("_predictor") for k in d.unused_state)


@pytest.mark.parametrize("case", ["1", "2"])
def test_decode_golden_f32(case, dec_f32):
    d, _ = dec_f32
    g = golden("facodec")
    wav = _run(d, g["lat" + case], g["spk" + case])
    assert wav.shape == g["wav" + case].shape
    assert np.max(np.abs(wav - g["wav" + case])) < 5e-4


@pytest.mark.parametrize("case", ["1", "2"])
def test_decode_golden_bf16_snr(case, dec_bf16):
    d, sd = dec_bf16
    g = golden("facodec")
    wav = _run(d, g["lat" + case], g["spk" + case])
    floor = ref_bf16_snr(sd, g["lat" + case], g["spk" + case], g["wav" + case])
    assert snr_db(wav, g["wav" + case]) > floor - 1.0


def test_decode_longer_vs_oracle(dec_f32, dec_bf16):
    gen = torch.Generator().manual_seed(12)
    lat = torch.randn(2, 256, 37, generator=gen)
    spk = torch.randn(2, 256, generator=gen)
    _, sd = dec_f32
    ref = orc.facodec_decode(sd, lat, spk).numpy()
    w32 = _run(dec_f32[0], lat, spk)
    assert np.max(np.abs(w32 - ref)) < 5e-4
    assert snr_db(_run(dec_bf16[0], lat, spk), ref) > ref_bf16_snr(sd, lat, spk, ref) - 1.0


def _calm(dtype):
    from flamed.utils.seeded_init import scale_weight_norm_gains
    d, sd = _dec(dtype)
    sd = scale_weight_norm_gains(sd, float(golden("facodec_calm")["gain"]))
    with torch.inference_mode():
        d.load_state_dict({k: v.to(DEV) for k, v in sd.items()}, strict=False)
    return d, sd


@pytest.fixture(scope="module")
def calm():
    return {"f32": _calm("f32"), "bf16": _calm("bf16")}


def test_decode_calm_golden(calm):
    g = golden("facodec_calm")
    w32 = _run(calm["f32"][0], g["lat"], g["spk"])
    wbf = _run(calm["bf16"][0], g["lat"], g["spk"])
    d32, sbf = float(np.max(np.abs(w32 - g["wav"]))), snr_db(wbf, g["wav"])
    print(f"calm T=64: f32 max|d| {d32:.2e}, bf16 SNR {sbf:.1f} dB")
    assert d32 < 5e-3 and sbf >= 30.0


def test_decode_calm_bench_length(calm):
    """The bench's decode shape (T = 400 frames -> 80,000 samples) vs the oracle."""
    gen = torch.Generator().manual_seed(40)
    lat = torch.randn(1, 256, 400, generator=gen)
    spk = torch.randn(1, 256, generator=gen)
    ref = orc.facodec_decode(calm["f32"][1], lat, spk).numpy()
    w32 = _run(calm["f32"][0], lat, spk)
    wbf = _run(calm["bf16"][0], lat, spk)
    d32, sbf = float(np.max(np.abs(w32 - ref))), snr_db(wbf, ref)
    print(f"calm T=400: f32 max|d| {d32:.2e}, bf16 SNR {sbf:.1f} dB")
    assert wbf.shape == (1, 1, 80000)
    assert d32 < 5e-3 and sbf >= 30.0


def test_graph_equals_eager(dec_f32):
    d, _ = dec_f32
    gen = torch.Generator().manual_seed(4)
    lat = torch.randn(1, 256, 11, generator=gen)
    spk = torch.randn(1, 256, generator=gen)
    d.hip_graph = True
    a = _run(d, lat, spk)
    b = _run(d, lat, spk)
    d.hip_graph = False
    c = _run(d, lat, spk)
    d.hip_graph = True
    assert np.array_equal(a, b) and np.array_equal(a, c)
