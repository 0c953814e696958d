"""Prior transformer stack on the HIP library (flamed_prior_encode / flamed_prior_decode; SURVEY.md
§8(f) f2) vs the reference's PriorGenerator.sample fixture and vs the oracle restatement
(oracle/flamed_oracle.py prior_encoder / prior_decode, itself pinned to the reference fixture by
test_oracle_golden.py::test_prior_sample).  Exact-fp32 path: tolerances are summation-order noise —
embeddings / logits rel-L2 <= 1e-4 after 22 FFT blocks, tgt_mask bit-exact, padded logits exactly 0."""
import numpy as np
import pytest
import torch

from _common import golden, t32, rel_l2, orc
from _flamed_common import build_flamed

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def model():
    m, _ = build_flamed(DEV, "f32")
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    return m.prior_generator, sd


def test_prior_sample_golden(model):
    pg, _ = model
    g = golden("flamed_sample")
    with torch.inference_mode():
        torch.manual_seed(int(g["rng_seed"]))
        pe, pl, tm = pg.sample(texts=t32(g["phonemes"]).to(DEV), src_lens=t32(g["src_lens"]).to(DEV), max_src_len=12,
                               prompts=t32(g["prompts"]).to(DEV), prompts_len=20, nfe=4, temperature=0.3)
    assert pg._hip is not None and pg._hip.handle is not None  # the HIP path ran
    assert np.array_equal(tm.cpu().numpy(), g["tgt_mask"])
    assert rel_l2(pe.cpu(), g["prior_embs"]) < 1e-4
    assert rel_l2(pl.sum(dim=1).cpu(), g["prior_logits_sum"]) < 1e-4


def _ids(B, L, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(1, 361, (B, L), generator=g)


@pytest.mark.parametrize("lens", [[97, 60, 33], [1], [130], [250, 247, 200, 180, 150, 99, 64, 12]])
def test_encode_vs_oracle(model, lens):
    pg, sd = model
    B, L = len(lens), max(lens)
    ids = _ids(B, L, 1)
    sl = torch.tensor(lens)
    mask = orc.mask_from_lengths(sl, L)
    with torch.inference_mode():
        out = pg.hip().encode(ids.to(DEV), mask.to(DEV)).cpu()
        ref = orc.prior_encoder(sd, ids, mask)
    valid = ~mask
    assert rel_l2(out[valid], ref[valid]) < 2e-5
    assert torch.all(out[mask] == 0)


def test_encode_beyond_position_table(model):
    """L > encoder_max_seq_len (4096): the sinusoid table is built for L, as Models.py:83-86 does."""
    pg, sd = model
    L = 4100
    ids = _ids(1, L, 2)
    mask = torch.zeros(1, L, dtype=torch.bool)
    with torch.inference_mode():
        out = pg.hip().encode(ids.to(DEV), mask.to(DEV)).cpu()
        ref = orc.prior_encoder(sd, ids, mask)
    assert rel_l2(out, ref) < 2e-5


@pytest.mark.parametrize("B,T,P,tl", [(1, 400, 240, [400]), (2, 96, 20, [96, 61]), (3, 37, 0, [37, 5, 30]),
                                      (8, 420, 160, [420, 400, 377, 350, 301, 256, 199, 64])])
def test_decode_vs_oracle(model, B, T, P, tl):
    """bridge -> shared decoder -> six prompt-prefixed decoders -> head at the bench shape (T=400 target
    frames behind a 3 s prompt) and ragged / prompt-less batches."""
    pg, sd = model
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, T, 192, generator=g)
    tgt = torch.tensor(tl)
    prompts = torch.randint(0, 1025, (B, 6, P), generator=g)
    mask = orc.mask_from_lengths(tgt, T)
    x = x.masked_fill(mask.unsqueeze(-1), 0)  # the length regulator zero-pads
    with torch.inference_mode():
        pe, pl = pg.hip().decode(x.to(DEV), mask.to(DEV), prompts.to(DEV), P)
        re, rl, rm = orc.prior_decode(sd, x, tgt, prompts)
    pe, pl = pe.cpu(), pl.cpu()
    assert pe.shape == re.shape and pl.shape == rl.shape
    assert rel_l2(pe, re) < 1e-4
    assert rel_l2(pl, rl) < 1e-4
    assert torch.all(pl.permute(0, 2, 3, 1)[mask.unsqueeze(1).expand(-1, 6, -1)] == 0)


def test_graph_equals_eager(model):
    pg, _ = model
    B, T, P = 2, 80, 30
    g = torch.Generator().manual_seed(4)
    x = torch.randn(B, T, 192, generator=g).to(DEV)
    mask = orc.mask_from_lengths(torch.tensor([80, 50]), T).to(DEV)
    prompts = torch.randint(0, 1025, (B, 6, P), generator=g).to(DEV)
    ids = _ids(B, 40, 5).to(DEV)
    smask = orc.mask_from_lengths(torch.tensor([40, 22]), 40).to(DEV)
    outs = []
    with torch.inference_mode():
        for graph in (True, False, True):
            pg.hip_graph = graph
            outs.append((pg.hip().encode(ids, smask), *pg.hip().decode(x, mask, prompts, P)))
    pg.hip_graph = True
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[0], outs[2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T,P,tl", [(1, 400, 240, [400]), (3, 37, 0, [37, 5, 30])])
def test_decode_bf16_vs_oracle(model, B, T, P, tl):
    """Decoder-side GEMMs on bf16 operands (PriorGenerator.hip_dec_dtype = "bf16", the package default; fp32
    accumulation, LayerNorm / softmax / residuals fp32) against the fp32 oracle: embeddings rel-L2 <= 1e-2
    and logits rel-L2 <= 1e-2 after 22 FFT blocks (measured 5.0-5.7e-3); the masked-logit zeros stay exact.  The fp32 handle is
    restored after (the module fixture runs the exact path)."""
    pg, sd = model
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, T, 192, generator=g)
    tgt = torch.tensor(tl)
    prompts = torch.randint(0, 1025, (B, 6, P), generator=g)
    mask = orc.mask_from_lengths(tgt, T)
    x = x.masked_fill(mask.unsqueeze(-1), 0)
    try:
        pg.hip_dec_dtype = "bf16"
        with torch.inference_mode():
            pe, pl = pg.hip().decode(x.to(DEV), mask.to(DEV), prompts.to(DEV), P)
    finally:
        pg.hip_dec_dtype = "f32"
    with torch.inference_mode():
        re, rl, _ = orc.prior_decode(sd, x, tgt, prompts)
        pe32, _ = pg.hip().decode(x.to(DEV), mask.to(DEV), prompts.to(DEV), P)
    pe, pl = pe.cpu(), pl.cpu()
    ee, el = rel_l2(pe, re), rel_l2(pl, rl)
    print(f"bf16 decoders B={B} T={T} P={P}: embs rel-L2 {ee:.3e}, logits rel-L2 {el:.3e}")
    assert ee < 1e-2 and el < 1e-2  # measured 5.0-5.7e-3
    assert torch.all(pl.permute(0, 2, 3, 1)[mask.unsqueeze(1).expand(-1, 6, -1)] == 0)
    assert rel_l2(pe32.cpu(), re) < 1e-4  # switching back re-runs the exact path


def test_attention_mfma_matches_fma_kernel(model):
    """The fp32-MFMA attention (flamed_tune attn_mfma = 1, default; xfmr.hpp attn_mfma_kernel) against the
    LDS-broadcast FMA kernel (attn_mfma = 0) on the encoder (48-wide heads, key-padding mask) and the
    decoders (32-wide heads, prompt-prefixed masks): both exact fp32, so they agree to summation order
    (rel-L2 <= 1e-5)."""
    from flamed import _native as nat
    pg, _ = model
    g = torch.Generator().manual_seed(9)
    B, T, P = 2, 150, 70
    x = torch.randn(B, T, 192, generator=g).to(DEV)
    mask = orc.mask_from_lengths(torch.tensor([150, 97]), T).to(DEV)
    prompts = torch.randint(0, 1025, (B, 6, P), generator=g).to(DEV)
    ids = _ids(B, 131, 6).to(DEV)
    smask = orc.mask_from_lengths(torch.tensor([131, 64]), 131).to(DEV)
    outs = []
    L = nat.lib()
    try:
        for v in (1, 0):
            nat.check(L.flamed_tune(b"attn_mfma", v), "flamed_tune")
            with torch.inference_mode():
                outs.append((pg.hip().encode(ids, smask), *pg.hip().decode(x, mask, prompts, P)))
    finally:
        nat.check(L.flamed_tune(b"attn_mfma", 1), "flamed_tune")
    for a, b in zip(outs[0], outs[1]):
        valid = torch.isfinite(b)
        assert torch.equal(torch.isfinite(a), valid)
        assert rel_l2(a[valid].cpu(), b[valid].cpu()) < 1e-5
