"""ProbGenerator — flow-matching latent generator (drop-in for reference
flamed/models/synthesizer/prob_generator.py).

Module/parameter names match the reference state dict exactly
(e.g. `denoiser.res_blocks.{i}.adaLN_modulation.1.weight`), and the public signatures are kept:
  * SimpleMLPAdaLN.forward(x, t, c)                       (reference :349-365)
  * ProbGenerator.sample(cond, spk, mask, nfe, temperature) (reference :434-447)
  * ProbGenerator.compute_loss(x1, cond, spk, mask)         (reference :414-432)

Execution: on a CUDA (ROCm) device at inference time the denoiser and the whole Euler loop run in
the gfx950 HIP library (`flamed/_native`, see include/flamed_hip.h) — GEMMs on MFMA, AdaLN hoisted
out of the loop, the nfe steps captured into one hipGraph.  The library is mandatory there: a
missing extension raises.  CPU tensors (the `--device cpu` plumbing config) and autograd training
use the module's own torch ops.  `hip_dtype` ("bf16" default, "f32" exact-fp32 MFMA parity mode)
selects the GEMM operand precision; residual stream, norms, AdaLN and the Euler state stay fp32.
"""
from __future__ import annotations

import ctypes
import math
import warnings
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed import _native as nat
from flamed import ops
from flamed.utils.conv import GemmConv1d


def modulate(x, shift, scale):
    """reference :7-8"""
    return x * (1 + scale) + shift


# ------------------------------------------------------------------ condition fold (once/utt)

class Block1D(nn.Module):
    """1x1 conv -> GroupNorm(8) -> Mish on masked input (reference :11-22)."""

    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.block = nn.Sequential(GemmConv1d(dim, dim_out, 1), nn.GroupNorm(groups, dim_out), nn.Mish())

    def forward(self, x, mask):
        return self.block(x * mask) * mask


class ResnetBlock1D(nn.Module):
    """reference :25-32"""

    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.block = Block1D(dim, dim_out, groups=groups)

    def forward(self, x, mask):
        return x + self.block(x, mask)


class ConditionDownSampler(nn.Module):
    """(B,T,Cin) -> (B,T,Cout): n_stages x [masked res 1x1 block, 1x1 halving conv + GN + ReLU],
    then Linear + ReLU (reference :167-205)."""

    def __init__(self, in_channel, out_channel, n_stages=1, n_groups=8):
        super().__init__()
        self.n_stages = n_stages
        self.resblocks = nn.ModuleList()
        self.downblocks = nn.ModuleList()
        ch = in_channel
        for _ in range(n_stages):
            self.resblocks.append(ResnetBlock1D(dim=ch, dim_out=ch))
            self.downblocks.append(nn.Sequential(GemmConv1d(ch, ch // 2, 1), nn.GroupNorm(n_groups, ch // 2), nn.ReLU()))
            ch //= 2
        self.proj_out = nn.Sequential(nn.Linear(ch, out_channel), nn.ReLU())

    def forward(self, x, mask):
        m = mask.transpose(1, -1)
        h = x.transpose(1, -1)
        for res, down in zip(self.resblocks, self.downblocks):
            h = down(res(h, m))
        return self.proj_out(h.transpose(1, -1))


class QuantizerEncoding(nn.Module):
    """Adds a learned per-quantizer embedding and folds (B,Q,T,D) -> (B,T,Q*D) (reference :368-381)."""

    def __init__(self, n_quantizers, hidden_dim):
        super().__init__()
        self.quantizer_ids = torch.arange(n_quantizers).expand((1, -1))
        self.quantizer_emb = nn.Embedding(n_quantizers, hidden_dim)

    def forward(self, x):
        b, q, l, d = x.shape
        ident = self.quantizer_emb(self.quantizer_ids.to(x.device))  # (1, Q, D)
        x = x + ident.unsqueeze(2)
        return x.permute(0, 2, 1, 3).reshape(b, l, q * d)


# ------------------------------------------------------------------ denoiser modules

class TimestepEmbedder(nn.Module):
    """Sinusoid [cos, sin] (max period 1e4, fp32) -> Linear -> SiLU -> Linear (reference :35-72)."""

    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(frequency_embedding_size, hidden_size, bias=True), nn.SiLU(),
                                 nn.Linear(hidden_size, hidden_size, bias=True))
        self.frequency_embedding_size = frequency_embedding_size

    @staticmethod
    def timestep_embedding(t, dim, max_period=10000):
        half = dim // 2
        k = torch.arange(start=0, end=half, dtype=torch.float32)
        freqs = torch.exp(-math.log(max_period) * k / half).to(device=t.device)
        args = t[:, :, None].float() * freqs[None]
        out = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
        if dim % 2:
            out = F.pad(out, (0, 1))
        return out

    def forward(self, t):
        return self.mlp(self.timestep_embedding(t, self.frequency_embedding_size))


class ConvNeXtBlock(nn.Module):
    """(B,T,C): depthwise conv -> GroupNorm(C,C) over T -> 1x1 -> GELU -> 1x1, residual
    (reference :75-111)."""

    def __init__(self, channels, kernel=31, stride=1, padding=15, expand=1, groups=None):
        super().__init__()
        groups = channels if groups is None else groups
        self.conv_1 = nn.Conv1d(channels, channels, kernel_size=kernel, stride=stride, padding=padding, groups=groups)
        self.ln_1 = nn.GroupNorm(channels, channels)
        self.conv_2 = nn.Conv1d(channels, channels * expand, kernel_size=1)
        self.conv_3 = nn.Conv1d(channels * expand, channels, kernel_size=1)

    def forward(self, x):
        h = x.transpose(1, -1)
        y = self.conv_3(F.gelu(self.conv_2(self.ln_1(self.conv_1(h)))))
        return (h + y).transpose(1, -1)


class ResBlock(nn.Module):
    """AdaLN(6) + gated ConvNeXt branch + gated MLP branch (reference :114-164)."""

    def __init__(self, channels, convnext_kernel=31, convnext_stride=1, convnext_padding=15, convnext_expand=1,
                 convnext_groups=None):
        super().__init__()
        self.channels = channels
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(channels, 6 * channels, bias=True))
        self.ln_conv = nn.LayerNorm(channels, eps=1e-6)
        self.conv_in = ConvNeXtBlock(channels, kernel=convnext_kernel, stride=convnext_stride,
                                     padding=convnext_padding, expand=convnext_expand, groups=convnext_groups)
        self.ln_mlp = nn.LayerNorm(channels, eps=1e-6)
        self.mlp = nn.Sequential(nn.Linear(channels, channels, bias=True), nn.SiLU(),
                                 nn.Linear(channels, channels, bias=True))

    def forward(self, x, y):
        sh_c, sc_c, g_c, sh_m, sc_m, g_m = self.adaLN_modulation(y).chunk(6, dim=-1)
        x = x + g_c * self.conv_in(modulate(self.ln_conv(x), sh_c, sc_c))
        return x + g_m * self.mlp(modulate(self.ln_mlp(x), sh_m, sc_m))


class FinalLayer(nn.Module):
    """AdaLN(5) + gated ConvNeXt + LN/modulate + Conv1d(k3) to the latent (reference :208-264)."""

    def __init__(self, model_channels, out_channels, convnext_kernel, convnext_stride, convnext_padding,
                 convnext_expand, convnext_groups):
        super().__init__()
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(model_channels, 5 * model_channels, bias=True))
        self.norm_in = nn.LayerNorm(model_channels, elementwise_affine=False, eps=1e-6)
        self.conv_in = ConvNeXtBlock(model_channels, kernel=convnext_kernel, stride=convnext_stride,
                                     padding=convnext_padding, expand=convnext_expand, groups=convnext_groups)
        self.norm_out = nn.LayerNorm(model_channels, elementwise_affine=False, eps=1e-6)
        self.conv_out = nn.Conv1d(model_channels, out_channels, kernel_size=3, stride=1, padding=1)

    def forward(self, x, c):
        sh_c, sc_c, g_c, sh_o, sc_o = self.adaLN_modulation(c).chunk(5, dim=-1)
        x = x + g_c * self.conv_in(modulate(self.norm_in(x), sh_c, sc_c))
        x = modulate(self.norm_out(x), sh_o, sc_o)
        return self.conv_out(x.transpose(1, -1)).transpose(1, -1)


class SimpleMLPAdaLN(nn.Module):
    """The attention-free denoiser (reference :267-365).  forward(x (B,T,C), t (1,1)|(B,T), c (B,S))."""

    def __init__(self, in_channels, model_channels, out_channels, spk_dim, num_res_blocks, convnext_kernel,
                 convnext_stride, convnext_padding, convnext_expand, convnext_groups):
        super().__init__()
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.spk_dim = spk_dim
        self.kernel_size = convnext_kernel
        self._convnext_plain = (convnext_stride == 1 and convnext_padding == convnext_kernel // 2 and convnext_expand == 1
                                and convnext_groups in (None, model_channels))
        self.time_embed = TimestepEmbedder(model_channels)
        self.cond_embed = nn.Linear(spk_dim, model_channels)
        self.proj_in = nn.Linear(in_channels, model_channels)
        self.res_blocks = nn.ModuleList([
            ResBlock(model_channels, convnext_kernel, convnext_stride, convnext_padding, convnext_expand,
                     convnext_groups) for _ in range(num_res_blocks)])
        self.final_layer = FinalLayer(model_channels, out_channels, convnext_kernel, convnext_stride,
                                      convnext_padding, convnext_expand, convnext_groups)
        self.hip_dtype = "bf16"
        self.hip_graph = True
        self._hip = None
        self.initialize_weights()

    def initialize_weights(self):
        """Same init recipe as the reference (:326-347): xavier Linear, N(0,0.02) time MLP, zeroed
        AdaLN projections and conv_out."""
        for mod in self.modules():
            if isinstance(mod, nn.Linear):
                nn.init.xavier_uniform_(mod.weight)
                if mod.bias is not None:
                    nn.init.zeros_(mod.bias)
        for lin in (self.time_embed.mlp[0], self.time_embed.mlp[2]):
            nn.init.normal_(lin.weight, std=0.02)
        zero = [blk.adaLN_modulation[-1] for blk in self.res_blocks]
        zero += [self.final_layer.adaLN_modulation[-1], self.final_layer.conv_out]
        for mod in zero:
            nn.init.zeros_(mod.weight)
            nn.init.zeros_(mod.bias)

    # -- dispatch
    def _use_hip(self, x: torch.Tensor) -> bool:
        if not x.is_cuda:
            return False
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return False  # autograd training: the HIP path is inference-only
        return self.hip_dims_ok()

    def hip_dims_ok(self) -> bool:
        """The library specialises these dims (flamed_den_create accepts them; stride-1 'same' depthwise
        ConvNeXt); otherwise the module keeps its torch ops on ROCm."""
        return self._convnext_plain and nat.supported("den", self.in_channels, self.model_channels, self.num_res_blocks,
                                                      self.kernel_size, self.spk_dim, nat.dtype_code(self.hip_dtype))

    def hip(self) -> "DenoiserHIP":
        if self._hip is None or self._hip.dtype_name != self.hip_dtype:
            self._hip = DenoiserHIP(self, self.hip_dtype)
        return self._hip

    def hip_invalidate(self):
        """Force the next HIP call to re-pack the weights.  load_state_dict does this by itself (below);
        call it after writing parameters in place under inference_mode, where tensors carry no
        version counter."""
        if self._hip is not None:
            self._hip._sig = None

    def _load_from_state_dict(self, *args, **kwargs):
        self.hip_invalidate()  # load_state_dict copies in place: same pointers, maybe no version bump
        super()._load_from_state_dict(*args, **kwargs)

    def forward(self, x, t, c):
        if self._use_hip(x):
            return ops.den_velocity(self.hip().oid, x, t, c)
        y = self.time_embed(t) + self.cond_embed(c).unsqueeze(1)
        h = self.proj_in(x)
        for blk in self.res_blocks:
            h = blk(h, y)
        return self.final_layer(h, y)


class ProbGenerator(nn.Module):
    """Condition fold + flow-matching Euler sampler over SimpleMLPAdaLN (reference :384-447)."""

    def __init__(self, config):
        super().__init__()
        self.target_dim = config["target_dim"]
        self.sigma_min = float(config["sigma_min"])
        self.quantizer_encoding = QuantizerEncoding(n_quantizers=config["n_quantizers"], hidden_dim=config["cond_dim"])
        self.cond_downsampling = ConditionDownSampler(in_channel=config["n_quantizers"] * config["cond_dim"],
                                                      out_channel=config["target_dim"],
                                                      n_stages=config["downsampling_stages"])
        self.n_stages = config["downsampling_stages"]
        cx = config["convnext"]
        self.denoiser = SimpleMLPAdaLN(in_channels=config["target_dim"], model_channels=config["hidden_dim"],
                                       out_channels=config["target_dim"], spk_dim=config["spk_dim"],
                                       num_res_blocks=config["n_layers"], convnext_kernel=cx["kernel_size"],
                                       convnext_stride=cx["stride"], convnext_padding=cx["padding"],
                                       convnext_expand=cx["expand"], convnext_groups=cx["groups"])
        self.cond_hip_dtype = "f32"  # condition fold GEMM operands on the HIP path ("f32" exact | "bf16")
        self._cond_hip = None

    def _cond_hip_ok(self, cond: torch.Tensor) -> bool:
        if not cond.is_cuda:
            return False
        mods = (self.quantizer_encoding, self.cond_downsampling)
        if torch.is_grad_enabled() and (cond.requires_grad or any(p.requires_grad for m in mods for p in m.parameters())):
            return False
        return self.cond_hip_dims_ok()

    def cond_hip_dims_ok(self) -> bool:
        q, d = self.quantizer_encoding.quantizer_emb.weight.shape
        return nat.supported("cond", q, d, self.target_dim, self.n_stages, nat.dtype_code(self.cond_hip_dtype))

    def fold_condition(self, cond, mask):
        """QuantizerEncoding + ConditionDownSampler (reference :435-436); on ROCm at inference one HIP
        call (flamed_cond_fold: three GEMMs with the quantizer encoding, GroupNorm/Mish/residual and
        GroupNorm/ReLU applied in their operand loaders)."""
        if self._cond_hip_ok(cond):
            if self._cond_hip is None or self._cond_hip.dtype_name != self.cond_hip_dtype:
                self._cond_hip = CondFoldHIP(self, self.cond_hip_dtype)
            return ops.cond_fold(self._cond_hip.oid, cond, mask)
        return self.cond_downsampling(self.quantizer_encoding(cond), mask)

    def _load_from_state_dict(self, *args, **kwargs):
        if self._cond_hip is not None:
            self._cond_hip._sig = None  # load_state_dict copies in place: re-pack at the next call
        super()._load_from_state_dict(*args, **kwargs)

    def compute_loss(self, x1, cond, spk, mask):
        """reference :414-432 (training objective; runs on torch ops under autograd)."""
        cond = self.fold_condition(cond, mask)
        t = torch.rand((cond.size(0), cond.size(1), 1), device=cond.device)
        x0 = torch.randn_like(cond, device=cond.device) + cond
        k = 1 - self.sigma_min
        xt = t * x1 + (1 - k * t) * x0
        dx = (x1 - k * x0) * mask
        vt = self.denoiser(xt, t.squeeze(), spk) * mask
        x1_est = (xt + (1 - k * t) * vt) * mask
        return {"fm_loss": F.mse_loss(vt, dx), "anchor_loss": F.mse_loss(x1_est, x1)}

    def sample(self, cond, spk, mask, nfe=4, temperature=1.0):
        """reference :434-447.  Noise is drawn from the global CPU RNG with the reference's shape and
        order, so seeded runs reproduce the reference trajectory."""
        cond = self.fold_condition(cond, mask)
        b, l, _ = cond.shape
        ts = torch.linspace(0, 1, nfe + 1, device=cond.device)
        xt = torch.randn((b, l, self.target_dim)).to(cond.device) * temperature + cond
        if self.denoiser._use_hip(xt):
            xt = ops.den_solve(self.denoiser.hip().oid, xt, ts, spk, nfe)
        else:
            delta_t = 1 / nfe
            for i in range(1, len(ts)):
                xt = xt + delta_t * self.denoiser(xt, ts[i - 1].unsqueeze(0).unsqueeze(1), spk)
        return xt.transpose(1, -1)


# ------------------------------------------------------------------ HIP backend

def denoiser_weight_list(den: SimpleMLPAdaLN) -> List[torch.Tensor]:
    """Weights in the order flamed_den_load expects (include/flamed_hip.h)."""
    te, fl = den.time_embed.mlp, den.final_layer
    w = [te[0].weight, te[0].bias, te[2].weight, te[2].bias, den.cond_embed.weight, den.cond_embed.bias,
         den.proj_in.weight, den.proj_in.bias]
    for blk in den.res_blocks:
        cv = blk.conv_in
        w += [blk.adaLN_modulation[1].weight, blk.adaLN_modulation[1].bias, blk.ln_conv.weight, blk.ln_conv.bias,
              cv.conv_1.weight, cv.conv_1.bias, cv.ln_1.weight, cv.ln_1.bias, cv.conv_2.weight, cv.conv_2.bias,
              cv.conv_3.weight, cv.conv_3.bias, blk.ln_mlp.weight, blk.ln_mlp.bias, blk.mlp[0].weight,
              blk.mlp[0].bias, blk.mlp[2].weight, blk.mlp[2].bias]
    cv = fl.conv_in
    w += [fl.adaLN_modulation[1].weight, fl.adaLN_modulation[1].bias, cv.conv_1.weight, cv.conv_1.bias,
          cv.ln_1.weight, cv.ln_1.bias, cv.conv_2.weight, cv.conv_2.bias, cv.conv_3.weight, cv.conv_3.bias,
          fl.conv_out.weight, fl.conv_out.bias]
    return w


class DenoiserHIP:
    """Owns one flamed_den_t handle for a SimpleMLPAdaLN module on one device."""

    def __init__(self, den: SimpleMLPAdaLN, dtype_name: str = "bf16"):
        self.den = den
        self.dtype_name = dtype_name
        self.code = nat.dtype_code(dtype_name)
        self.handle = None
        self._sig = None
        self._keep: List[torch.Tensor] = []
        self.ws = nat.Workspace()
        self.ada_ws = nat.Workspace()
        self._solve_bufs = {}
        # a solve that ran as an uncaptured persistent launch (B = 1 .. 8, bf16) is checked WITHOUT waiting for
        # it: its outcome (flamed_den_persist_query) is looked at by this handle's next call, or by settle() at
        # the caller's own sync point (Flamed.sample_batch), and a failed launch (NaN-poisoned x) is then re-run
        # on the graph of launches into the same output tensor, so a failure never survives to the caller's
        # host copy; skipped inside a stream capture (the caller then owns the check: persist_status)
        self.check_persist = True
        self._pending = []  # (launch seq, output, input x, ts, spk, nfe) of solves not yet known to have succeeded
        self.oid = ops.register(self)  # torch.ops.flamed_hip.den_* carry this id

    def __del__(self):
        try:
            if self.handle is not None:
                nat.destroy(self.handle, "flamed_den_destroy")
        except Exception:
            pass

    def _ensure(self, device):
        params = denoiser_weight_list(self.den)
        sig = tuple((p.data_ptr(), nat.tensor_version(p)) for p in params) + (str(device),)
        if sig == self._sig and self.handle is not None:
            return
        L = nat.lib()
        if self.handle is None:
            h = ctypes.c_void_p()
            d = self.den
            nat.check(L.flamed_den_create(d.in_channels, d.model_channels, d.num_res_blocks, d.kernel_size,
                                          d.spk_dim, self.code, ctypes.byref(h)), "flamed_den_create")
            self.handle = h
            nat.track(h, "flamed_den_destroy")
        keep = [p.detach().to(device=device, dtype=torch.float32).contiguous() for p in params]
        arr = (ctypes.c_void_p * len(keep))(*[t.data_ptr() for t in keep])
        nat.check(L.flamed_den_load(self.handle, arr, len(keep), nat.stream_ptr(device)), "flamed_den_load")
        self._keep = keep
        self._sig = sig
        self._solve_bufs = {}

    def adaln(self, t_vals: torch.Tensor, spk: torch.Tensor, tidx: torch.Tensor, sidx: torch.Tensor,
              out: torch.Tensor | None = None) -> torch.Tensor:
        dev = spk.device
        L = nat.lib()
        t_vals = t_vals.to(device=dev, dtype=torch.float32).contiguous()
        spk = spk.to(dtype=torch.float32).contiguous()
        tidx = tidx.to(device=dev, dtype=torch.int32).contiguous()
        sidx = sidx.to(device=dev, dtype=torch.int32).contiguous()
        R = tidx.numel()
        ms = L.flamed_den_mods_stride(self.handle)  # modulation floats (+ LayerNorm-fold tables, bf16)
        if out is not None:
            # the solve's persistent table (its pointer is baked into the captured graph): a mismatch is a
            # caller bug, never silently replaced by a fresh table the solve would not read
            if out.shape != (R, ms) or out.device != dev or out.dtype != torch.float32 or not out.is_contiguous():
                raise ValueError(f"adaln: out must be a contiguous float32 ({R}, {ms}) tensor on {dev}; got "
                                 f"{tuple(out.shape)} {out.dtype} on {out.device}")
            mods = out
        else:
            mods = torch.empty((R, ms), dtype=torch.float32, device=dev)
        nbytes = L.flamed_den_adaln_workspace_size(self.handle, t_vals.numel(), spk.shape[0])
        ws = self.ada_ws.get(nbytes, dev)
        nat.check(L.flamed_den_adaln(self.handle, nat.ptr(t_vals), t_vals.numel(), nat.ptr(spk), spk.shape[0],
                                     nat.ptr(tidx), nat.ptr(sidx), R, nat.ptr(mods), nat.ptr(ws), ws.numel(),
                                     nat.stream_ptr(dev)), "flamed_den_adaln")
        return mods

    def _check_groupnorm(self, B: int, T: int):
        """The reference's GroupNorm(H, H) over T (F.group_norm's batch-size check) rejects a single
        value per channel; the HIP path raises the same ValueError instead of normalising it."""
        if B * T == 1:
            raise ValueError(f"Expected more than 1 value per channel when training, got input size "
                             f"{[1, self.den.model_channels, 1]}")

    def velocity(self, x: torch.Tensor, t: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
        dev = x.device
        self._ensure(dev)
        B, T, C = x.shape
        self._check_groupnorm(B, T)
        if t.dim() != 2:
            raise ValueError(f"t must be 2-D ((1,1), (B,1) or (B,T)); got shape {tuple(t.shape)}")
        tb, tt = t.shape
        if tb not in (1, B) or tt not in (1, T):
            raise ValueError(f"t shape {tuple(t.shape)} does not broadcast with x {tuple(x.shape)}")
        if tt == 1:
            R, mod_div = B, T
            tidx = torch.arange(B, device=dev) if tb == B else torch.zeros(B, dtype=torch.long, device=dev)
            sidx = torch.arange(B, device=dev)
        else:
            R, mod_div = B * T, 1
            r = torch.arange(R, device=dev)
            tidx = r if tb == B else r % T
            sidx = r // T
        mods = self.adaln(t.reshape(-1), c, tidx, sidx)
        xin = x.to(torch.float32).contiguous()
        v = torch.empty((B, T, self.den.out_channels), dtype=torch.float32, device=dev)
        L = nat.lib()
        ws = self.ws.get(L.flamed_den_workspace_size(self.handle, B, T), dev)
        nat.check(L.flamed_den_velocity(self.handle, nat.ptr(xin), nat.ptr(mods), mod_div, B, T, nat.ptr(v),
                                        nat.ptr(ws), ws.numel(), nat.stream_ptr(dev)), "flamed_den_velocity")
        return v.to(x.dtype)

    def persist_info(self, with_ms: bool = False):
        """(persistent launches enqueued, broken[, device ms of the last uncaptured launch]) of this handle:
        whether B = 1 solves ran as one persistent launch (flamed_den_persist_info; waits for that launch)."""
        runs, broken, ms = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_float(0.0)
        nat.check(nat.lib().flamed_den_persist_info(self.handle, ctypes.byref(runs), ctypes.byref(broken), ctypes.byref(ms)),
                  "flamed_den_persist_info")
        if with_ms:
            return runs.value, bool(broken.value), float(ms.value)
        return runs.value, bool(broken.value)

    def persist_fails(self) -> int:
        """Failed (NaN-poisoned) persistent launches so far on this handle (diagnostic: waits for the device)."""
        f = ctypes.c_int(0)
        nat.check(nat.lib().flamed_den_persist_fails(self.handle, ctypes.byref(f)), "flamed_den_persist_fails")
        return f.value

    def persist_times(self, n: int) -> List[float]:
        """Device ms of the up to n most recent uncaptured persistent launches, oldest first (HIP events
        around each kernel on its launch stream; flamed_den_persist_times)."""
        buf = (ctypes.c_float * max(n, 1))()
        k = nat.lib().flamed_den_persist_times(self.handle, buf, n)
        if k < 0:
            nat.check(-1, "flamed_den_persist_times")
        return [float(buf[i]) for i in range(k)]

    def solve(self, xt: torch.Tensor, ts: torch.Tensor, spk: torch.Tensor, nfe: int) -> torch.Tensor:
        """Full Euler solve; returns a new (B,T,C) fp32 tensor.  Only enqueues work: a persistent launch is
        checked later (settle), and a failed one re-written in place before the caller's next sync point."""
        dev = xt.device
        self._ensure(dev)
        B, T, C = xt.shape
        self._check_groupnorm(B, T)
        capturing = torch.cuda.is_current_stream_capturing()
        if self._pending and not capturing:  # (event queries are not allowed while a stream captures)
            self.settle(block=False)
        runs0, _ = self.persist_status()
        x = self._launch(xt, ts, spk, nfe, 0)
        out = x.clone()
        if self.check_persist and not capturing and self.persist_status()[0] > runs0:
            seq = ctypes.c_longlong(-1)
            nat.check(nat.lib().flamed_den_persist_last(self.handle, ctypes.byref(seq)), "flamed_den_persist_last")
            self._pending.append((seq.value, out, xt.detach().clone(), ts.detach().clone(), spk.detach().clone(), nfe))
            if len(self._pending) > 32:  # the launch ring holds 64: settle the oldest before their slots are reused
                self.settle(block=True)
        return out

    def settle(self, block: bool = True) -> int:
        """Check this handle's pending persistent solves (flamed_den_persist_query, no wait per launch); a failed
        one is reported with a warning and re-run on the graph of launches (use_graph bit 2) into the tensor that
        solve returned, enqueued on the current stream.  block=True first waits for the device, so every pending
        solve is decided (the call Flamed.sample_batch makes at its own synchronisation); block=False leaves the
        unfinished ones pending.  Returns the number of re-runs."""
        if not self._pending or torch.cuda.is_current_stream_capturing():
            return 0
        L = nat.lib()
        if block:
            torch.cuda.synchronize(self._pending[0][1].device)
        keep, reruns = [], 0
        for rec in self._pending:
            seq, out, x0, ts, spk, nfe = rec
            st = ctypes.c_int(0)
            nat.check(L.flamed_den_persist_query(self.handle, seq, ctypes.byref(st)), "flamed_den_persist_query")
            state = st.value
            if state == 2:
                keep.append(rec)
                continue
            if state == 3:  # the launch's ring slot was reused: decide from the output itself
                state = 1 if bool(torch.isnan(out).any()) else 0
            if state == 1:
                warnings.warn("flamed: persistent solve failed (its output was NaN-poisoned); "
                              "re-running it on the graph of launches")
                out.copy_(self._launch(x0, ts, spk, nfe, 2))
                reruns += 1
        self._pending = keep
        return reruns

    def _launch(self, xt, ts, spk, nfe, extra_graph_bits):
        """AdaLN rows + flamed_den_solve into the handle's solve buffer (returned, not copied)."""
        dev = xt.device
        B, T, C = xt.shape
        L = nat.lib()
        key = (B, T, nfe)
        bufs = self._solve_bufs.get(key)
        if bufs is None:
            r = torch.arange(nfe * B, device=dev)
            bufs = {"x": torch.empty((B, T, C), dtype=torch.float32, device=dev),
                    "tidx": (r // B).to(torch.int32), "sidx": (r % B).to(torch.int32)}
            self._solve_bufs = {key: bufs}
        ws = self.ws.get(L.flamed_den_workspace_size(self.handle, B, T), dev)
        if "mods" not in bufs:
            bufs["mods"] = torch.empty((nfe * B, L.flamed_den_mods_stride(self.handle)), dtype=torch.float32, device=dev)
        # AdaLN rows of every step first (computing the later rows on a side stream while the first graph
        # chunk runs was measured slower: 34.8 -> 36.6 ms at B = 1, 352 -> 358 ms at B = 64)
        self.adaln(ts[:nfe], spk, bufs["tidx"], bufs["sidx"], out=bufs["mods"])
        bufs["x"].copy_(xt)
        use_graph = int(bool(self.den.hip_graph)) | extra_graph_bits
        nat.check(L.flamed_den_solve(self.handle, nat.ptr(bufs["x"]), nat.ptr(bufs["mods"]), nfe, B, T, nat.ptr(ws),
                                     ws.numel(), use_graph, nat.stream_ptr(dev)),
                  "flamed_den_solve" if not extra_graph_bits else "flamed_den_solve (re-run)")
        return bufs["x"]

    def persist_status(self):
        """(persistent launches enqueued, failed launches as of the last completed copy) of this handle; never
        waits (flamed_den_persist_status)."""
        runs, fails = ctypes.c_int(0), ctypes.c_int(0)
        nat.check(nat.lib().flamed_den_persist_status(self.handle, ctypes.byref(runs), ctypes.byref(fails)),
                  "flamed_den_persist_status")
        return runs.value, fails.value


def cond_weight_list(pg: "ProbGenerator") -> List[torch.Tensor]:
    """Weights in the order flamed_cond_load expects (include/flamed_hip.h)."""
    cd = pg.cond_downsampling
    rb = cd.resblocks[0].block.block
    db = cd.downblocks[0]
    return [pg.quantizer_encoding.quantizer_emb.weight, rb[0].weight, rb[0].bias, rb[1].weight, rb[1].bias,
            db[0].weight, db[0].bias, db[1].weight, db[1].bias, cd.proj_out[0].weight, cd.proj_out[0].bias]


class CondFoldHIP:
    """Owns one flamed_cond_t handle (condition fold of a ProbGenerator on one device)."""

    def __init__(self, pg: "ProbGenerator", dtype_name: str = "f32"):
        self.pg = pg
        self.dtype_name = dtype_name
        self.code = nat.dtype_code(dtype_name)
        self.handle = None
        self._sig = None
        self.ws = nat.Workspace()
        self.oid = ops.register(self)  # torch.ops.flamed_hip.cond_fold

    def __del__(self):
        try:
            if self.handle is not None:
                nat.destroy(self.handle, "flamed_cond_destroy")
        except Exception:
            pass

    def _ensure(self, device):
        params = cond_weight_list(self.pg)
        sig = tuple((p.data_ptr(), nat.tensor_version(p)) for p in params) + (str(device),)
        if sig == self._sig and self.handle is not None:
            return
        L = nat.lib()
        if self.handle is None:
            h = ctypes.c_void_p()
            q, d = self.pg.quantizer_encoding.quantizer_emb.weight.shape
            nat.check(L.flamed_cond_create(q, d, self.pg.target_dim, self.pg.n_stages, self.code, ctypes.byref(h)),
                      "flamed_cond_create")
            self.handle = h
            nat.track(h, "flamed_cond_destroy")
        keep = [p.detach().to(device=device, dtype=torch.float32).contiguous() for p in params]
        arr = (ctypes.c_void_p * len(keep))(*[t.data_ptr() for t in keep])
        nat.check(L.flamed_cond_load(self.handle, arr, len(keep), nat.stream_ptr(device)), "flamed_cond_load")
        self._keep = keep
        self._sig = sig

    def fold(self, cond: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """cond (B, Q, T, D), mask (B, T, 1) True = valid -> (B, T, target_dim) fp32."""
        dev = cond.device
        self._ensure(dev)
        B, Q, T, D = cond.shape
        c = cond.to(torch.float32).contiguous()
        m = mask.reshape(B, T).to(device=dev, dtype=torch.float32).contiguous()
        out = torch.empty((B, T, self.pg.target_dim), dtype=torch.float32, device=dev)
        L = nat.lib()
        ws = self.ws.get(L.flamed_cond_workspace_size(self.handle, B, T), dev)
        nat.check(L.flamed_cond_fold(self.handle, nat.ptr(c), nat.ptr(m), B, T, nat.ptr(out), nat.ptr(ws), ws.numel(),
                                     nat.stream_ptr(dev)), "flamed_cond_fold")
        return out
