"""Pin the oracle (CPU restatement) against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import torch

from _common import golden, seeded, t32, rel_l2, orc

torch.set_num_threads(min(8, torch.get_num_threads()))
TOL = 2e-5  # fp32 restatement vs reference: same ops, only summation-order differences


def test_rng_stream():
    g = golden("rng")
    torch.manual_seed(0)
    assert torch.equal(torch.randn((2, 5)), t32(g["r1"]))
    assert torch.equal(torch.randn((2, 5)), t32(g["r2"]))
    assert torch.equal(torch.randn((2, 3, 4)), t32(g["r3"]))


def test_kaiser_filters_match_reference_buffers():
    g = golden("act1d")
    f = orc.kaiser_sinc_filter(0.25, 0.3, 12)
    assert torch.allclose(f, t32(g["up_filter"]).flatten(), atol=1e-7)
    assert torch.allclose(f, t32(g["down_filter"]).flatten(), atol=1e-7)


def test_denoiser_tiny():
    g = golden("den_tiny")
    sd = seeded("den_tiny", prefix="den.")
    kw = dict(p="den", n_blocks=2, k=31)
    v1 = orc.denoiser_forward(sd, t32(g["x"]), t32(g["t1"]), t32(g["c"]), **kw)
    assert rel_l2(v1, g["v1"]) < TOL
    vB = orc.denoiser_forward(sd, t32(g["x"]), t32(g["tB"]), t32(g["c"]), **kw)
    assert rel_l2(vB, g["vB"]) < TOL
    xt = t32(g["x"])
    ts = torch.linspace(0, 1, 5)
    for i in range(4):
        xt = xt + 0.25 * orc.denoiser_forward(sd, xt, ts[i].reshape(1, 1), t32(g["c"]), **kw)
        assert rel_l2(xt, g["traj"][i]) < TOL


def test_denoiser_full():
    g = golden("den_full")
    sd = seeded("prob_generator")
    v1 = orc.denoiser_forward(sd, t32(g["x"]), t32(g["t1"]), t32(g["c"]))
    assert rel_l2(v1, g["v1"]) < TOL
    vB = orc.denoiser_forward(sd, t32(g["xB"]), t32(g["tB"]), t32(g["cB"]))
    assert rel_l2(vB, g["vB"]) < TOL
    vB1 = orc.denoiser_forward(sd, t32(g["xB"]), t32(g["t_mid"]), t32(g["cB"]))
    assert rel_l2(vB1, g["vB1"]) < TOL


def test_prob_sample():
    g = golden("prob_sample")
    sd = seeded("prob_generator")
    lens = t32(g["lens"])
    T = g["cond"].shape[2]
    mask = ~(torch.arange(T)[None, :] >= lens[:, None]).unsqueeze(-1)
    cf = orc.cond_fold(sd, t32(g["cond"]), mask)
    assert rel_l2(cf, g["cond_fold"]) < TOL
    torch.manual_seed(int(g["rng_seed"]))
    lat = orc.prob_sample(sd, t32(g["cond"]), t32(g["spk"]), mask, nfe=int(g["nfe"]),
                          temperature=float(g["temperature"]))
    assert rel_l2(lat, g["latents"]) < TOL


def test_pva_module_and_flow():
    g = golden("pva")
    sd = seeded("pva")
    src_len = t32(g["src_len"])
    L = g["enc"].shape[1]
    mask = torch.arange(L)[None, :] >= src_len[:, None]
    p = "prior_generator.pva"
    v = orc.prob_module_forward(sd, p + ".duration_generator", t32(g["xt"]), t32(g["enc"]), torch.tensor(0.5), mask)
    assert rel_l2(v, g["v_dur"]) < TOL
    v = orc.prob_module_forward(sd, p + ".sil_generator", t32(g["xt"]), t32(g["enc"]), torch.tensor(0.125), mask)
    assert rel_l2(v, g["v_sil"]) < TOL
    torch.manual_seed(int(g["rng_seed"]))
    d, s = orc.pva_flow(sd, t32(g["enc"]), mask, int(g["nfe"]), float(g["temperature"]))
    assert rel_l2(d, g["dur_final"]) < TOL and rel_l2(s, g["sil_final"]) < TOL
    pd = orc.log_to_frames(d).numpy()
    sdur = orc.log_to_frames(s).numpy()
    x_lr, tl = orc.length_regulate(g["enc"], pd, sdur, g["src_len"])
    assert np.array_equal(tl, g["tgt_len"])
    assert x_lr.shape == g["x_lr"].shape and np.array_equal(x_lr, g["x_lr"])


def test_length_regulator_cases_bit_exact():
    g = golden("lr_cases")
    for ci in range(int(g["n"])):
        mx = int(g[f"c{ci}_max"])
        out, tl = orc.length_regulate(g[f"c{ci}_x"], g[f"c{ci}_pd"], g[f"c{ci}_sd"], g[f"c{ci}_sl"],
                                      None if mx < 0 else mx)
        assert np.array_equal(tl, g[f"c{ci}_tl"]), ci
        assert out.shape == g[f"c{ci}_out"].shape and np.array_equal(out, g[f"c{ci}_out"]), ci
        # the gather-index form used by the LR kernel reproduces the same output
        rep = orc.lr_repeats(g[f"c{ci}_pd"], g[f"c{ci}_sd"], g[f"c{ci}_sl"])
        idx = orc.lr_gather_index(rep, out.shape[1])
        x = g[f"c{ci}_x"]
        alt = np.where(idx[..., None] >= 0, np.take_along_axis(x, np.maximum(idx, 0)[..., None], 1), 0)
        assert np.array_equal(alt, out), ci


def test_act1d():
    g = golden("act1d")
    sd = {"a.upsample.filter": t32(g["up_filter"]), "a.downsample.lowpass.filter": t32(g["down_filter"]),
          "a.act.alpha": t32(g["alpha"]), "a.act.beta": t32(g["beta"])}
    y = orc.activation1d(sd, "a", t32(g["x"]))
    assert rel_l2(y, g["y"]) < 1e-6


def test_facodec_decode():
    g = golden("facodec")
    sd = seeded("facodec_decoder")
    w1 = orc.facodec_decode(sd, t32(g["lat1"]), t32(g["spk1"]))
    assert rel_l2(w1, g["wav1"]) < 1e-4
    w2 = orc.facodec_decode(sd, t32(g["lat2"]), t32(g["spk2"]))
    assert rel_l2(w2, g["wav2"]) < 1e-4


def test_facodec_decode_calm():
    """Oracle vs the reference on the non-saturating decoder fixture (weight-norm gains x 0.6, T = 64)."""
    from flamed.utils.seeded_init import scale_weight_norm_gains
    g = golden("facodec_calm")
    sd = scale_weight_norm_gains(seeded("facodec_decoder"), float(g["gain"]))
    w = orc.facodec_decode(sd, t32(g["lat"]), t32(g["spk"]))
    assert w.shape == g["wav"].shape
    assert float((w - t32(g["wav"])).abs().max()) < 1e-6
    assert float(t32(g["wav"]).abs().max()) < 0.9  # not saturated


def test_facodec_encode_and_vq():
    """Encoder, factorized RVQ codes (bit-exact) and timbre embedding vs the reference (§8(f) f3)."""
    g = golden("facodec_encode")
    esd = seeded("facodec_encoder")
    dsd = seeded("facodec_decoder")
    enc = orc.facodec_encode(esd, t32(g["wav"]))
    assert rel_l2(enc, g["enc_out"]) < TOL
    codes, spk = orc.decoder_vq(dsd, t32(g["enc_out"]))
    assert torch.equal(codes, t32(g["codes"]))
    assert rel_l2(spk, g["spk"]) < TOL
    assert orc.positional_table(256).shape == (5000, 1, 256)


def test_prior_sample():
    """Prior transformer restatement (encoder -> PVA -> LR -> bridge/shared/6 decoders -> head) vs the
    reference's PriorGenerator.sample fixture (global-RNG draw order as the reference)."""
    from _flamed_common import build_flamed
    m, _ = build_flamed("cpu")
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    g = golden("flamed_sample")
    torch.manual_seed(int(g["rng_seed"]))
    with torch.inference_mode():
        pe, pl, tm = orc.prior_sample(sd, t32(g["phonemes"]), t32(g["src_lens"]), t32(g["prompts"]), nfe=4,
                                      temperature=0.3)
    assert np.array_equal(tm.numpy(), g["tgt_mask"])
    assert rel_l2(pe, g["prior_embs"]) < TOL
    assert rel_l2(pl.sum(dim=1), g["prior_logits_sum"]) < TOL
