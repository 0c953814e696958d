"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement (fp32, torch eager on CPU, functional form over a state dict) of the Flamed-TTS
flow-matching inference hot path, following the reference op order.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may use this module, and only as the
checker / CPU baseline.

Pinned against golden vectors produced by importing the reference itself in the build container
(`tests/golden/make_golden.py` -> `tests/golden/*.npz`; checked by `tests/test_oracle_golden.py`).

Every function cites the reference file:line it restates (paths relative to the reference root).
Weights are looked up by the reference's own state-dict keys.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


# --------------------------------------------------------------------------------------------
# ProbGenerator / SimpleMLPAdaLN   (flamed/models/synthesizer/prob_generator.py)
# --------------------------------------------------------------------------------------------

def _lin(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def timestep_freq(t: torch.Tensor, dim: int = 256, max_period: float = 10000.0) -> torch.Tensor:
    """prob_generator.py:49-67 — [cos(t f), sin(t f)], f_j = exp(-ln(P) j / half); t is 2-D."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[:, :, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def _layer_norm(x: torch.Tensor, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def convnext(sd: SD, p: str, x: torch.Tensor, k: int) -> torch.Tensor:
    """prob_generator.py:75-111 — x (B,T,H): dwconv(k, pad k//2) -> GroupNorm(H,H) -> 1x1 -> GELU
    -> 1x1, plus the block's own residual."""
    H = x.shape[-1]
    h = x.transpose(1, -1)
    y = F.conv1d(h, sd[p + ".conv_1.weight"], sd[p + ".conv_1.bias"], padding=k // 2, groups=H)
    y = F.group_norm(y, H, sd[p + ".ln_1.weight"], sd[p + ".ln_1.bias"], 1e-5)
    y = F.conv1d(y, sd[p + ".conv_2.weight"], sd[p + ".conv_2.bias"])
    y = F.gelu(y)
    y = F.conv1d(y, sd[p + ".conv_3.weight"], sd[p + ".conv_3.bias"])
    return (h + y).transpose(1, -1)


def resblock(sd: SD, p: str, x: torch.Tensor, y: torch.Tensor, k: int) -> torch.Tensor:
    """prob_generator.py:114-164 (modulate :7-8)."""
    m = _lin(sd, p + ".adaLN_modulation.1", F.silu(y))
    sh_c, sc_c, g_c, sh_m, sc_m, g_m = m.chunk(6, dim=-1)
    h = _layer_norm(x, sd[p + ".ln_conv.weight"], sd[p + ".ln_conv.bias"], 1e-6)
    x = x + g_c * convnext(sd, p + ".conv_in", h * (1 + sc_c) + sh_c, k)
    h = _layer_norm(x, sd[p + ".ln_mlp.weight"], sd[p + ".ln_mlp.bias"], 1e-6)
    h = h * (1 + sc_m) + sh_m
    h = _lin(sd, p + ".mlp.2", F.silu(_lin(sd, p + ".mlp.0", h)))
    return x + g_m * h


def final_layer(sd: SD, p: str, x: torch.Tensor, y: torch.Tensor, k: int) -> torch.Tensor:
    """prob_generator.py:208-264."""
    m = _lin(sd, p + ".adaLN_modulation.1", F.silu(y))
    sh_c, sc_c, g_c, sh_o, sc_o = m.chunk(5, dim=-1)
    h = _layer_norm(x, None, None, 1e-6)
    x = x + g_c * convnext(sd, p + ".conv_in", h * (1 + sc_c) + sh_c, k)
    x = _layer_norm(x, None, None, 1e-6) * (1 + sc_o) + sh_o
    x = F.conv1d(x.transpose(1, -1), sd[p + ".conv_out.weight"], sd[p + ".conv_out.bias"], padding=1)
    return x.transpose(1, -1)


def denoiser_forward(sd: SD, x: torch.Tensor, t: torch.Tensor, c: torch.Tensor,
                     p: str = "prob_generator.denoiser", n_blocks: int = 4, k: int = 31) -> torch.Tensor:
    """SimpleMLPAdaLN.forward, prob_generator.py:349-365.  x (B,T,C), t (1,1) or (B,T), c (B,S)."""
    te = _lin(sd, p + ".time_embed.mlp.2", F.silu(_lin(sd, p + ".time_embed.mlp.0", timestep_freq(t))))
    ce = _lin(sd, p + ".cond_embed", c)
    y = te + ce.unsqueeze(1)
    h = _lin(sd, p + ".proj_in", x)
    for i in range(n_blocks):
        h = resblock(sd, f"{p}.res_blocks.{i}", h, y, k)
    return final_layer(sd, p + ".final_layer", h, y, k)


def cond_fold(sd: SD, cond: torch.Tensor, mask: torch.Tensor, p: str = "prob_generator",
              n_stages: int = 1) -> torch.Tensor:
    """QuantizerEncoding (prob_generator.py:368-381) + ConditionDownSampler (:167-205).
    cond (B,Q,T,D) -> (B,T,target_dim); mask (B,T,1) float/bool (True = valid)."""
    b, q, l, d = cond.shape
    ident = sd[p + ".quantizer_encoding.quantizer_emb.weight"][:q]
    x = cond + ident[None, :, None, :]
    x = x.permute(0, 2, 1, 3).reshape(b, l, q * d)
    m = mask.to(x.dtype).transpose(1, -1)
    x = x.transpose(1, -1)
    dp = p + ".cond_downsampling"
    for s in range(n_stages):
        rp = f"{dp}.resblocks.{s}.block.block"
        h = F.conv1d(x * m, sd[rp + ".0.weight"], sd[rp + ".0.bias"])
        h = F.group_norm(h, 8, sd[rp + ".1.weight"], sd[rp + ".1.bias"], 1e-5)
        h = F.mish(h) * m
        x = x + h
        bp = f"{dp}.downblocks.{s}"
        x = F.conv1d(x, sd[bp + ".0.weight"], sd[bp + ".0.bias"])
        x = F.group_norm(x, 8, sd[bp + ".1.weight"], sd[bp + ".1.bias"], 1e-5)
        x = F.relu(x)
    x = x.transpose(1, -1)
    return F.relu(_lin(sd, dp + ".proj_out.0", x))


def prob_sample(sd: SD, cond: torch.Tensor, spk: torch.Tensor, mask: torch.Tensor, nfe: int = 4,
                temperature: float = 1.0, target_dim: int = 256, n_blocks: int = 4, k: int = 31,
                noise: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ProbGenerator.sample, prob_generator.py:434-447.  Noise is drawn from the global CPU RNG
    exactly as the reference does (:440) unless `noise` is given.  Returns (B, target_dim, T)."""
    c = cond_fold(sd, cond, mask)
    b, l, _ = c.shape
    ts = torch.linspace(0, 1, nfe + 1)
    if noise is None:
        noise = torch.randn((b, l, target_dim))
    xt = noise * temperature + c
    dt = 1 / nfe
    for i in range(1, len(ts)):
        vt = denoiser_forward(sd, xt, ts[i - 1].unsqueeze(0).unsqueeze(1), spk, n_blocks=n_blocks, k=k)
        xt = xt + dt * vt
    return xt.transpose(1, -1)


def euler_solve(sd: SD, xt: torch.Tensor, spk: torch.Tensor, nfe: int, n_blocks: int = 4, k: int = 31,
                steps: Optional[int] = None) -> torch.Tensor:
    """The denoiser Euler loop alone (prob_generator.py:439-445) starting from xt (B,T,C).
    `steps` < nfe runs only the first `steps` steps (bounded CPU baselines)."""
    ts = torch.linspace(0, 1, nfe + 1)
    dt = 1 / nfe
    for i in range(1, (steps if steps is not None else nfe) + 1):
        xt = xt + dt * denoiser_forward(sd, xt, ts[i - 1].unsqueeze(0).unsqueeze(1), spk, n_blocks=n_blocks, k=k)
    return xt


# --------------------------------------------------------------------------------------------
# PVA duration / silence generator   (flamed/models/synthesizer/pva.py)
# --------------------------------------------------------------------------------------------

def sinusoidal_pos_emb(x: torch.Tensor, dim: int, scale: float = 1000.0) -> torch.Tensor:
    """pva.py:9-22 — [sin, cos] with denominator (half-1)."""
    half = dim // 2
    e = math.log(10000) / (half - 1)
    freqs = torch.exp(torch.arange(half).float() * -e)
    if x.ndim < 1:
        x = x.unsqueeze(0)
    emb = scale * x.unsqueeze(1) * freqs.unsqueeze(0)
    return torch.cat((emb.sin(), emb.cos()), dim=-1)


def prob_module_forward(sd: SD, p: str, xt: torch.Tensor, enc: torch.Tensor, t: torch.Tensor,
                        mask: Optional[torch.Tensor], dim: int = 192) -> torch.Tensor:
    """ProbabilisticModule.forward, pva.py:221-238 (Conv :241-284, TimeEmbedding :25-41)."""
    out = _lin(sd, p + ".proj", torch.cat([xt.unsqueeze(-1), enc], dim=-1))
    te = sinusoidal_pos_emb(t, dim)
    te = _lin(sd, p + ".time_emb.time_emb.3", F.silu(_lin(sd, p + ".time_emb.time_emb.1", te)))
    out = out + te.unsqueeze(1).expand(-1, out.size(1), -1)
    cp = p + ".conv_layer"
    h = F.conv1d(out.transpose(1, 2), sd[cp + ".conv1d_1.conv.weight"], sd[cp + ".conv1d_1.conv.bias"], padding=1)
    h = F.relu(h.transpose(1, 2))
    h = F.layer_norm(h, (h.shape[-1],), sd[cp + ".layer_norm_1.weight"], sd[cp + ".layer_norm_1.bias"], 1e-5)
    h = F.conv1d(h.transpose(1, 2), sd[cp + ".conv1d_2.conv.weight"], sd[cp + ".conv1d_2.conv.bias"], padding=1)
    h = F.relu(h.transpose(1, 2))
    h = F.layer_norm(h, (h.shape[-1],), sd[cp + ".layer_norm_2.weight"], sd[cp + ".layer_norm_2.bias"], 1e-5)
    v = _lin(sd, p + ".linear_layer", h).squeeze(-1)
    if mask is not None:
        v = v.masked_fill(mask, 0.0)
    return v


def pva_flow(sd: SD, x: torch.Tensor, src_mask: torch.Tensor, nfe: int, temperature: float,
             p: str = "prior_generator.pva", noise: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """The Euler loop of PVA.sample, pva.py:97-109.  Returns the final (dur_t, sil_t) in log space.
    Noise order: dur then sil from the global CPU RNG (:101-102)."""
    b, l, _ = x.shape
    ts = torch.linspace(0, 1, nfe + 1)
    dt = 1 / nfe
    if noise is None:
        dur = torch.randn((b, l)) * temperature
        sil = torch.randn((b, l)) * temperature
    else:
        dur, sil = noise[0] * temperature, noise[1] * temperature
    for i in range(1, len(ts)):
        dur = dur + dt * prob_module_forward(sd, p + ".duration_generator", dur, x, ts[i - 1], src_mask)
        sil = sil + dt * prob_module_forward(sd, p + ".sil_generator", sil, x, ts[i - 1], src_mask)
    return dur, sil


def log_to_frames(d: torch.Tensor) -> torch.Tensor:
    """pva.py:111-112 — clamp(round(exp(d) - 1), min=0) (float tensor, integral values)."""
    return torch.clamp(torch.round(torch.exp(d) - 1), min=0)


def lr_repeats(phone_dur: np.ndarray, sil_dur: np.ndarray, src_lens: np.ndarray) -> np.ndarray:
    """LengthRegulator.LR repeat counts, pva.py:133-145 (integer part, numpy).
    Returns repeats (B, 2L) int64 interleaved [phone_0, sil_0, phone_1, sil_1, ...]; padded phonemes
    (index >= src_len) repeat exactly 1 frame and 0 silence frames."""
    B, L = phone_dur.shape
    valid = np.arange(L)[None, :] < np.asarray(src_lens)[:, None]
    pr = np.where(valid, np.rint(phone_dur.astype(np.float64)), 0).astype(np.int64)
    pr = np.maximum(pr, 1)
    sr = np.where(valid, np.rint(sil_dur.astype(np.float64)), 0).astype(np.int64)
    sr = np.maximum(sr, 0)
    rep = np.empty((B, 2 * L), dtype=np.int64)
    rep[:, 0::2] = pr
    rep[:, 1::2] = sr
    return rep


def length_regulate(x: np.ndarray, phone_dur: np.ndarray, sil_dur: np.ndarray, src_lens: np.ndarray,
                    max_len: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """LengthRegulator.LR, pva.py:125-166 (+ tools.pad :299-317): interleave phone / silence segments
    (silence frame = x[:, 0]), repeat, split per item, zero-pad to max_len (or the longest), truncating
    longer items to max_len as F.pad with a negative amount does."""
    B, L, H = x.shape
    rep = lr_repeats(phone_dur, sil_dur, src_lens)
    tgt = rep.sum(axis=1)
    T = int(max_len) if max_len else int(tgt.max())
    out = np.zeros((B, T, H), dtype=x.dtype)
    for b in range(B):
        rows: List[int] = []
        for j in range(2 * L):
            src = j // 2 if j % 2 == 0 else 0
            rows.extend([src] * int(rep[b, j]))
        rows = rows[:T]
        if rows:
            out[b, : len(rows)] = x[b, rows]
    return out, tgt


def lr_gather_index(rep: np.ndarray, T: int) -> np.ndarray:
    """Per output frame the source phoneme index (or -1 for zero padding): the integer map the LR
    kernel builds (prefix sum over the interleaved repeats).  (B, T) int64."""
    B, L2 = rep.shape
    idx = np.full((B, T), -1, dtype=np.int64)
    for b in range(B):
        pos = 0
        for j in range(L2):
            n = int(rep[b, j])
            src = j // 2 if j % 2 == 0 else 0
            end = min(pos + n, T)
            if end > pos:
                idx[b, pos:end] = src
            pos += n
            if pos >= T:
                break
    return idx


def mask_from_lengths(lengths: torch.Tensor, max_len: Optional[int] = None) -> torch.Tensor:
    """tools.get_mask_from_lengths, tools.py:91-99 (True = padding)."""
    if max_len is None:
        max_len = int(lengths.max().item())
    ids = torch.arange(0, max_len).unsqueeze(0).expand(lengths.shape[0], -1)
    return ids >= lengths.unsqueeze(1)


# --------------------------------------------------------------------------------------------
# FaCodec decoder   (flamed/models/facodec/facodec.py, alias_free_torch/*.py)
# --------------------------------------------------------------------------------------------

def kaiser_sinc_filter(cutoff: float, half_width: float, kernel_size: int) -> torch.Tensor:
    """alias_free_torch/filter.py:27-58 (even kernel) -> (kernel_size,)."""
    half = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    win = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    if kernel_size % 2 == 0:
        time = torch.arange(-half, half) + 0.5
    else:
        time = torch.arange(kernel_size) - half
    f = 2 * cutoff * win * torch.sinc(2 * cutoff * time)
    return f / f.sum()


def snake_beta(x: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
    """facodec.py:57-118 with alpha_logscale=True."""
    a = torch.exp(alpha)[None, :, None]
    b = torch.exp(beta)[None, :, None]
    return x + (1.0 / (b + 1e-9)) * torch.pow(torch.sin(x * a), 2)


def activation1d(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """Activation1d, act.py:7-29; UpSample1d resample.py:9-37; DownSample1d/LowPassFilter1d
    resample.py:40-57, filter.py:61-96.  ratio 2, 12-tap filters taken from the state dict."""
    C = x.shape[1]
    fu = sd[p + ".upsample.filter"].reshape(1, 1, -1)
    fd = sd[p + ".downsample.lowpass.filter"].reshape(1, 1, -1)
    K = fu.shape[-1]
    pad = K // 2 - 1
    pl = pad * 2 + (K - 2) // 2
    pr = pad * 2 + (K - 2 + 1) // 2
    y = F.pad(x, (pad, pad), mode="replicate")
    y = 2 * F.conv_transpose1d(y, fu.expand(C, -1, -1), stride=2, groups=C)
    y = y[..., pl:-pr]
    y = snake_beta(y, sd[p + ".act.alpha"], sd[p + ".act.beta"])
    y = F.pad(y, (K // 2 - 1, K // 2), mode="replicate")
    return F.conv1d(y, fd.expand(C, -1, -1), stride=2, groups=C)


def wn_weight(sd: SD, p: str) -> torch.Tensor:
    """torch weight_norm (dim=0): w = g * v / ||v|| (norm over all dims but 0); facodec.py:27-32."""
    v = sd[p + ".weight_v"]
    g = sd[p + ".weight_g"]
    n = torch.linalg.vector_norm(v, dim=tuple(range(1, v.dim())), keepdim=True)
    return g * v / n


def residual_unit(sd: SD, p: str, x: torch.Tensor, dilation: int) -> torch.Tensor:
    """ResidualUnit, facodec.py:121-133."""
    y = activation1d(sd, p + ".block.0", x)
    y = F.conv1d(y, wn_weight(sd, p + ".block.1"), sd[p + ".block.1.bias"], padding=3 * dilation, dilation=dilation)
    y = activation1d(sd, p + ".block.2", y)
    y = F.conv1d(y, wn_weight(sd, p + ".block.3"), sd[p + ".block.3.bias"])
    return x + y


def decoder_block(sd: SD, p: str, x: torch.Tensor, stride: int) -> torch.Tensor:
    """DecoderBlock, facodec.py:246-265."""
    y = activation1d(sd, p + ".block.0", x)
    y = F.conv_transpose1d(y, wn_weight(sd, p + ".block.1"), sd[p + ".block.1.bias"], stride=stride,
                           padding=stride // 2 + stride % 2, output_padding=stride % 2)
    for j, d in enumerate((1, 3, 9)):
        y = residual_unit(sd, f"{p}.block.{j + 2}", y, d)
    return y


def facodec_decode(sd: SD, x: torch.Tensor, spk: torch.Tensor, up_ratios: Sequence[int] = (5, 5, 4, 2),
                   p: str = "") -> torch.Tensor:
    """FACodecDecoder.inference, facodec.py:630-638 (model stack :398-415).  x (B,256,T) -> (B,1,hop*T)."""
    style = _lin(sd, p + "timbre_linear", spk).unsqueeze(2)
    gamma, beta = style.chunk(2, 1)
    h = F.layer_norm(x.transpose(1, 2), (x.shape[1],), None, None, 1e-5).transpose(1, 2)
    h = h * gamma + beta
    h = F.conv1d(h, wn_weight(sd, p + "model.0"), sd[p + "model.0.bias"], padding=3)
    for i, s in enumerate(up_ratios):
        h = decoder_block(sd, f"{p}model.{i + 1}", h, s)
    n = len(up_ratios) + 1
    h = activation1d(sd, f"{p}model.{n}", h)
    h = F.conv1d(h, wn_weight(sd, f"{p}model.{n + 1}"), sd[f"{p}model.{n + 1}.bias"], padding=3)
    return torch.tanh(h)


# ============================ FaCodec prompt encoding ==========================

def encoder_block(sd: SD, p: str, x: torch.Tensor, stride: int) -> torch.Tensor:
    """EncoderBlock, facodec.py:136-155: 3 residual units (dil 1,3,9) -> Act1d -> strided WNConv1d."""
    for j, d in enumerate((1, 3, 9)):
        x = residual_unit(sd, f"{p}.block.{j}", x, d)
    x = activation1d(sd, p + ".block.3", x)
    return F.conv1d(x, wn_weight(sd, p + ".block.4"), sd[p + ".block.4.bias"], stride=stride,
                    padding=stride // 2 + stride % 2)


def facodec_encode(sd: SD, wav: torch.Tensor, up_ratios: Sequence[int] = (2, 4, 5, 5), p: str = "") -> torch.Tensor:
    """FACodecEncoder.forward, facodec.py:183-216.  wav (B,1,n) -> (B,out_channels,n/hop)."""
    h = F.conv1d(wav, wn_weight(sd, p + "block.0"), sd[p + "block.0.bias"], padding=3)
    for i, s in enumerate(up_ratios):
        h = encoder_block(sd, f"{p}block.{i + 1}", h, s)
    n = len(up_ratios) + 1
    h = activation1d(sd, f"{p}block.{n}", h)
    return F.conv1d(h, wn_weight(sd, f"{p}block.{n + 1}"), sd[f"{p}block.{n + 1}.bias"], padding=1)


def _wn_linear(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    return F.linear(x, wn_weight(sd, p), sd[p + ".bias"])


def fvq_quantize(sd: SD, p: str, z: torch.Tensor, gaps: Optional[list] = None):
    """FactorizedVectorQuantize.forward (eval), fvq.py:35-87 + decode_latents :102-116.
    z (B,D,T) -> (z_q (B,D,T), indices (B,T) int64).  Nearest code under L2-normalised euclidean
    distance (first index on ties, as torch.max), straight-through `z_e + (z_q - z_e)` kept."""
    B, D, T = z.shape
    z_e = _wn_linear(sd, p + ".in_proj", z.transpose(1, 2))                       # (B,T,d)
    e = F.normalize(z_e.reshape(B * T, -1))
    cb_raw = sd[p + "._codebook.weight"]
    cb = F.normalize(cb_raw)
    dist = e.pow(2).sum(1, keepdim=True) - 2 * e @ cb.t() + cb.pow(2).sum(1, keepdim=True).t()
    idx = (-dist).max(1)[1].reshape(B, T)
    if gaps is not None:  # top-2 distance gap per frame (test diagnostics: near-ties)
        top2 = torch.topk(-dist, 2, dim=1).values
        gaps.append((top2[:, 0] - top2[:, 1]).reshape(B, T))
    z_q = cb_raw[idx]                                                               # (B,T,d)
    z_q = z_e + (z_q - z_e)
    return _wn_linear(sd, p + ".out_proj", z_q).transpose(1, 2), idx


def rvq_quantize(sd: SD, p: str, x: torch.Tensor, n_layers: int, gaps: Optional[list] = None):
    """ResidualVQ.forward (eval), rvq.py:27-76.  Returns (sum, indices (n,B,T), quantized (n,B,D,T))."""
    out, res, idx, qs = 0.0, x, [], []
    for i in range(n_layers):
        q, ind = fvq_quantize(sd, f"{p}.layers.{i}", res, gaps)
        res = res - q
        out = out + q
        idx.append(ind)
        qs.append(q)
    return out, torch.stack(idx), torch.stack(qs)


def positional_table(d: int, max_len: int = 5000) -> torch.Tensor:
    """PositionalEncoding buffer `pe` (max_len, 1, d), facodec/transformer.py:35-47."""
    pos = torch.arange(max_len).unsqueeze(1)
    freq = torch.exp(torch.arange(0, d, 2) * (-math.log(10000.0) / d))
    pe = torch.zeros(max_len, 1, d)
    pe[:, 0, 0::2] = torch.sin(pos * freq)
    pe[:, 0, 1::2] = torch.cos(pos * freq)
    return pe


def timbre_encoder(sd: SD, x: torch.Tensor, p: str = "timbre_encoder", n_layers: int = 4, heads: int = 4) -> torch.Tensor:
    """TransformerEncoder.forward (use_cln False, no padding mask), transformer.py:154-234, with
    nn.MultiheadAttention restated (scaled dot-product, softmax over keys).  x (B,T,d) -> (B,T,d).
    PositionalEncoding adds pe[:B] — the batch index picks the position vector (:49-51)."""
    B, T, d = x.shape
    x = x + sd[p + ".position_emb.pe"][:B]
    hd = d // heads
    for i in range(n_layers):
        q = f"{p}.layers.{i}"
        h = F.layer_norm(x, (d,), sd[q + ".ln_1.weight"], sd[q + ".ln_1.bias"], 1e-5)
        qkv = F.linear(h, sd[q + ".self_attn.in_proj_weight"], sd[q + ".self_attn.in_proj_bias"])
        qq, kk, vv = (t.reshape(B, T, heads, hd).transpose(1, 2) for t in qkv.split(d, dim=-1))
        att = torch.softmax((qq / math.sqrt(hd)) @ kk.transpose(-1, -2), dim=-1)
        a = (att @ vv).transpose(1, 2).reshape(B, T, d)
        x = x + F.linear(a, sd[q + ".self_attn.out_proj.weight"], sd[q + ".self_attn.out_proj.bias"])
        h = F.layer_norm(x, (d,), sd[q + ".ln_2.weight"], sd[q + ".ln_2.bias"], 1e-5)
        h = F.conv1d(h.transpose(1, 2), sd[q + ".ffn.ffn_1.weight"], sd[q + ".ffn.ffn_1.bias"],
                     padding=sd[q + ".ffn.ffn_1.weight"].shape[-1] // 2).transpose(1, 2)
        x = x + F.linear(F.relu(h), sd[q + ".ffn.ffn_2.weight"], sd[q + ".ffn.ffn_2.bias"])
    return F.layer_norm(x, (d,), sd[p + ".last_ln.weight"], sd[p + ".last_ln.bias"], 1e-5)


def decoder_vq(sd: SD, x: torch.Tensor, n_q=(1, 2, 3), gaps: Optional[list] = None):
    """FACodecDecoder.forward(vq=True) (eval), facodec.py:470-530.  x (B,C,T) encoder output ->
    (codes (sum n_q, B, T) int64 in [prosody, content, residual] order, spk (B,C)).  The residual RVQ
    sees x - (sum of prosody layers + sum of content layers) (:495-497)."""
    _, ip, qp = rvq_quantize(sd, "quantizer.0", x, n_q[0], gaps)
    _, ic, qc = rvq_quantize(sd, "quantizer.1", x, n_q[1], gaps)
    codes = [ip, ic]
    if n_q[2] > 0:
        _, ir, _ = rvq_quantize(sd, "quantizer.2", x - (qp.sum(0) + qc.sum(0)), n_q[2], gaps)
        codes.append(ir)
    spk = timbre_encoder(sd, x.transpose(1, 2)).transpose(1, 2).mean(dim=2)
    return torch.cat(codes, dim=0), spk


# --------------------------------------------------------------------------------------------
# Prior transformer stack   (flamed/models/synthesizer/prior_generator.py, module/transformer/*.py)
# --------------------------------------------------------------------------------------------

def sinusoid_table(n_position: int, d_hid: int) -> torch.Tensor:
    """Models.py:10-30 — angle pos / 10000^(2*(j//2)/d) in float64, sin on even j, cos on odd j, then
    float32.  (n_position, d_hid)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)[None, :]
    t = pos / np.power(10000, 2 * (j // 2) / d_hid)
    t[:, 0::2] = np.sin(t[:, 0::2])
    t[:, 1::2] = np.cos(t[:, 1::2])
    return torch.from_numpy(t).float()


def fft_block(sd: SD, p: str, x: torch.Tensor, mask: torch.Tensor, n_head: int) -> torch.Tensor:
    """FFTBlock.forward, Layers.py:21-30: post-norm MultiHeadAttention (SubLayers.py:29-57; scaled
    dot product with the key-padding mask set to -inf, Modules.py:14-25), masked_fill, then the conv
    FFN (SubLayers.py:85-95: Conv1d k0 -> ReLU -> Conv1d k1, + residual, LayerNorm), masked_fill.
    x (B, n, D), mask (B, n) True = padding."""
    B, n, D = x.shape
    dk = D // n_head
    a = p + ".slf_attn."

    def heads(name):
        return F.linear(x, sd[a + name + ".weight"], sd[a + name + ".bias"]).view(B, n, n_head, dk) \
            .permute(2, 0, 1, 3).reshape(n_head * B, n, dk)

    q, k, v = heads("w_qs"), heads("w_ks"), heads("w_vs")
    att = torch.bmm(q, k.transpose(1, 2)) / float(np.power(dk, 0.5))
    att = att.masked_fill(mask.unsqueeze(1).expand(-1, n, -1).repeat(n_head, 1, 1), -np.inf)
    o = torch.bmm(torch.softmax(att, dim=2), v).view(n_head, B, n, dk).permute(1, 2, 0, 3).reshape(B, n, D)
    o = F.linear(o, sd[a + "fc.weight"], sd[a + "fc.bias"])
    x = F.layer_norm(o + x, (D,), sd[a + "layer_norm.weight"], sd[a + "layer_norm.bias"], 1e-5)
    x = x.masked_fill(mask.unsqueeze(-1), 0)
    f = p + ".pos_ffn."
    w1, w2 = sd[f + "w_1.weight"], sd[f + "w_2.weight"]
    h = F.conv1d(x.transpose(1, 2), w1, sd[f + "w_1.bias"], padding=(w1.shape[-1] - 1) // 2)
    h = F.conv1d(F.relu(h), w2, sd[f + "w_2.bias"], padding=(w2.shape[-1] - 1) // 2).transpose(1, 2)
    x = F.layer_norm(h + x, (D,), sd[f + "layer_norm.weight"], sd[f + "layer_norm.bias"], 1e-5)
    return x.masked_fill(mask.unsqueeze(-1), 0)


def _n_layers(sd: SD, p: str) -> int:
    n = 0
    while f"{p}.layer_stack.{n}.slf_attn.fc.weight" in sd:
        n += 1
    return n


def prior_encoder(sd: SD, texts: torch.Tensor, src_mask: torch.Tensor, p: str = "prior_generator.encoder",
                  n_head: int = 4) -> torch.Tensor:
    """Encoder.forward (eval), Models.py:73-100: src_word_emb(ids) + position table, FFT blocks."""
    B, n = texts.shape
    pe = sd[p + ".position_enc"][0]
    pos = sinusoid_table(n, pe.shape[-1]) if n > pe.shape[0] - 1 else pe[:n]
    x = F.embedding(texts, sd[p + ".src_word_emb.weight"]) + pos.unsqueeze(0).expand(B, -1, -1)
    for i in range(_n_layers(sd, p)):
        x = fft_block(sd, f"{p}.layer_stack.{i}", x, src_mask, n_head)
    return x


def prior_decoder_stack(sd: SD, p: str, x: torch.Tensor, mask: torch.Tensor, n_head: int) -> torch.Tensor:
    """Decoder.forward (eval), Models.py:139-171: + position table, FFT blocks."""
    B, n, _ = x.shape
    pe = sd[p + ".position_enc"][0]
    pos = sinusoid_table(n, pe.shape[-1]) if n > pe.shape[0] - 1 else pe[:n]
    x = x + pos.unsqueeze(0).expand(B, -1, -1)
    for i in range(_n_layers(sd, p)):
        x = fft_block(sd, f"{p}.layer_stack.{i}", x, mask, n_head)
    return x


def prior_decode(sd: SD, x_lr: torch.Tensor, tgt_lens: torch.Tensor, prompts: torch.Tensor,
                 p: str = "prior_generator", n_head: int = 12):
    """PriorGenerator.sample after the PVA, prior_generator.py:165-188: bridge -> shared decoder ->
    six prompt-prefixed decoders chained through their target slices (PreEncoding :20-26 adds the
    segment and quantizer embeddings) -> head, masked and permuted.  x_lr (B, T, 192), prompts
    (B, nq, P) -> (prior_embs (B, nq, T, 384), logits (B, V+1, nq, T), tgt_mask (B, T))."""
    B, T, _ = x_lr.shape
    P = prompts.shape[-1]
    tgt_mask = mask_from_lengths(tgt_lens, T)
    out = prior_decoder_stack(sd, p + ".shared_decoder",
                              F.linear(x_lr, sd[p + ".bridge.weight"], sd[p + ".bridge.bias"]), tgt_mask, n_head)
    dec_mask = mask_from_lengths(P + tgt_lens, P + T)
    pemb = F.embedding(prompts, sd[p + ".code_embedding.weight"])
    hid = []
    nq = prompts.shape[1]
    for q in range(nq):
        z = torch.cat([pemb[:, q], out], dim=1)
        z = torch.cat([z[:, :P] + sd[p + ".pre_encode.prompt_emb"], z[:, P:] + sd[p + ".pre_encode.target_emb"]], 1)
        z = z + sd[p + ".pre_encode.quantizer_emb.weight"][q]
        out = prior_decoder_stack(sd, f"{p}.prior_decoder.{q}", z, dec_mask, n_head)[:, P:]
        hid.append(out.unsqueeze(1))
    embs = torch.cat(hid, dim=1)
    logits = F.linear(embs, sd[p + ".head.weight"], sd[p + ".head.bias"])
    logits = logits * ~tgt_mask.unsqueeze(1).expand(-1, nq, -1).unsqueeze(3)
    return embs, logits.permute(0, 3, 1, 2).contiguous(), tgt_mask


def prior_sample(sd: SD, texts: torch.Tensor, src_lens: torch.Tensor, prompts: torch.Tensor, nfe: int,
                 temperature: float, p: str = "prior_generator"):
    """PriorGenerator.sample, prior_generator.py:141-196: encoder -> PVA flow (global-RNG noise) ->
    length regulator -> decode."""
    B, L = texts.shape
    src_mask = mask_from_lengths(src_lens, L)
    enc = prior_encoder(sd, texts, src_mask, p + ".encoder")
    d, s = pva_flow(sd, enc, src_mask, nfe, temperature, p + ".pva")
    x_lr, tl = length_regulate(enc.numpy(), log_to_frames(d).numpy(), log_to_frames(s).numpy(), src_lens.numpy())
    return prior_decode(sd, torch.from_numpy(x_lr), torch.from_numpy(tl), prompts, p)
