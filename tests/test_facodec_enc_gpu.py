"""HIP FaCodec encoder (prompt encoding) vs the reference fixture and the oracle.
Tolerances: exact-fp32 MFMA mode rel-L2 <= 2e-5 (reassociation only) and the RVQ codes computed from
it bit-identical to the reference's; bf16 mode: error vs the fp32 reference within 1 dB of what the
reference itself reaches under CPU bf16 autocast (rel-L2 <= 1.122 x, as the decoder test); graph
replay == eager bitwise."""
import numpy as np
import pytest
import torch

from _common import golden, seeded, t32, rel_l2, orc
from _flamed_common import build_codec_encoder

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def enc():
    return build_codec_encoder(DEV)


def test_encode_golden_f32(enc):
    g = golden("facodec_encode")
    enc.hip_dtype = "f32"
    with torch.inference_mode():
        z = enc(t32(g["wav"]).to(DEV))
    assert enc._hip is not None and enc._hip.dtype_name == "f32"  # the HIP path ran
    assert z.shape == g["enc_out"].shape
    assert rel_l2(z.cpu(), g["enc_out"]) < 2e-5


def test_codes_from_hip_encoder_match_reference(enc):
    from _flamed_common import build_flamed
    _, dec = build_flamed(DEV, "f32")
    g = golden("facodec_encode")
    enc.hip_dtype = "f32"
    with torch.inference_mode():
        _, codes, _, _, spk = dec(enc(t32(g["wav"]).to(DEV)), eval_vq=False, vq=True)
    assert np.array_equal(codes.cpu().numpy(), g["codes"])
    assert rel_l2(spk.cpu(), g["spk"]) < 1e-4


@pytest.mark.parametrize("n", [8137, 1000, 16003])
def test_encode_odd_lengths_vs_oracle(enc, n):
    gen = torch.Generator().manual_seed(n)
    wav = 0.1 * torch.randn(1, 1, n, generator=gen)
    ref = orc.facodec_encode(seeded("facodec_encoder"), wav)
    enc.hip_dtype = "f32"
    with torch.inference_mode():
        z = enc(wav.to(DEV))
    assert z.shape == ref.shape
    assert rel_l2(z.cpu(), ref) < 2e-5


def test_encode_bf16_and_graph(enc):
    g = golden("facodec_encode")
    x = t32(g["wav"]).to(DEV)
    enc.hip_dtype = "bf16"
    try:
        with torch.inference_mode():
            enc.hip_graph = False
            z_eager = enc(x)
            enc.hip_graph = True
            z_graph = enc(x)
            z_graph2 = enc(x)
    finally:
        enc.hip_dtype = "f32"
        enc.hip_graph = True
    assert torch.equal(z_eager, z_graph) and torch.equal(z_graph, z_graph2)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ref_bf16 = orc.facodec_encode(seeded("facodec_encoder"), t32(g["wav"])).float()
    e_ref = rel_l2(ref_bf16, g["enc_out"])
    assert rel_l2(z_graph.cpu(), g["enc_out"]) < 1.122 * max(e_ref, 1e-3)


@pytest.mark.parametrize("B,T", [(2, 240), (1, 37)])
def test_vq_timbre_vs_oracle(B, T):
    """Prompt-side RVQ codes + timbre speaker embedding on HIP (flamed_vq_encode) vs the oracle
    (decoder_vq: facodec.py:470-533) on random encoder outputs.  Codes bit-exact except where the
    oracle's top-2 distance gap is below 1e-5 (counted; fp32 summation-order ties), spk rel-L2 <= 1e-4;
    quantized sums vs the module's own torch path on CPU."""
    from _flamed_common import build_flamed
    _, dec = build_flamed(DEV, "f32")
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    x = torch.randn(B, 256, T, generator=torch.Generator().manual_seed(11))
    with torch.inference_mode():
        outs, codes, _, qb, spk = dec(x.to(DEV), eval_vq=False, vq=True)
        gaps = []
        rc, rspk = orc.decoder_vq(sd, x, gaps=gaps)
        dec_cpu = dec.to("cpu")
        couts, ccodes, _, cqb, cspk = dec_cpu(x, eval_vq=False, vq=True)
        dec.to(DEV)
    assert dec._vq_hip is not None and dec._vq_hip.handle is not None  # the HIP path ran
    codes = codes.cpu()
    assert codes.shape == rc.shape
    near = torch.stack(gaps) < 1e-5  # (n_q, B, T) near-ties of the oracle's own distances
    neq = codes != rc
    # a mismatch in one layer changes every later residual of that group: only frames whose first
    # mismatch sits on a near-tie are excused
    first = neq.float().cumsum(0) == 1
    assert bool((near | ~(neq & first)).all()), "code mismatch away from a near-tie"
    assert rel_l2(spk.cpu(), rspk) < 1e-4
    if not bool(neq.any()):
        assert rel_l2(outs.cpu(), couts) < 1e-4
        for a, b in zip(qb, cqb):
            assert rel_l2(a.cpu(), b) < 1e-4
