"""PVA — probabilistic variance adaptor: flow-matching duration / silence generators and the integer
length regulator (drop-in for reference flamed/models/synthesizer/pva.py).

Parameter names match the reference state dict (`duration_generator.conv_layer.conv1d_1.conv.weight`,
...).  On a CUDA (ROCm) device at inference, PVA.sample runs the whole nfe-step flow of both
generators in the gfx950 HIP library (exact-fp32 MFMA GEMMs, graph-captured) and the length
regulator as two HIP kernels (prefix sums + gather, bit-exact); the library is mandatory there.
CPU tensors and autograd training use the modules' own torch ops.
"""
from __future__ import annotations

import ctypes
import warnings
import math
from collections import OrderedDict
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed import _native as nat
from flamed import ops
from flamed.utils.tools import pad


class SinusoidalPosEmb(nn.Module):
    """[sin, cos] of scale * t * exp(-k ln(1e4) / (half - 1)) (reference pva.py:9-22)."""

    def __init__(self, dim):
        super().__init__()
        if dim % 2:
            raise ValueError("SinusoidalPosEmb requires an even dim")
        half = dim // 2
        self.emb = torch.exp(torch.arange(half).float() * -(math.log(10000) / (half - 1)))

    def forward(self, x, scale=1000):
        if x.ndim < 1:
            x = x.unsqueeze(0)
        a = scale * x.unsqueeze(1) * self.emb.unsqueeze(0).to(x.device)
        return torch.cat((a.sin(), a.cos()), dim=-1)


class TimeEmbedding(nn.Module):
    """reference pva.py:25-41"""

    def __init__(self, hidden_dim, time_emb_scale):
        super().__init__()
        self.time_emb = nn.Sequential(SinusoidalPosEmb(hidden_dim), nn.Linear(hidden_dim, hidden_dim * time_emb_scale),
                                      nn.SiLU(), nn.Linear(hidden_dim * time_emb_scale, hidden_dim))

    def forward(self, t):
        return self.time_emb(t)


class Conv(nn.Module):
    """Conv1d over a channels-last (B, L, C) sequence (reference pva.py:241-284)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, bias=True,
                 w_init="linear"):
        super().__init__()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=padding,
                              dilation=dilation, bias=bias)

    def forward(self, x):
        return self.conv(x.contiguous().transpose(1, 2)).contiguous().transpose(1, 2)


class ProbabilisticModule(nn.Module):
    """Velocity net of one log-duration flow: proj([xt, enc]) + time embedding -> 2 x (conv k3, ReLU,
    LayerNorm) -> Linear(->1), masked (reference pva.py:173-238)."""

    def __init__(self, model_config):
        super().__init__()
        self.input_size = model_config["input_size"]
        self.filter_size = model_config["filter_size"]
        self.kernel = model_config["kernel_size"]
        self.time_scale = model_config["time_scale"]
        self.conv_output_size = model_config["filter_size"]
        self.dropout = model_config["drop_out"]
        d, f, k = self.input_size, self.filter_size, self.kernel
        self.proj = nn.Linear(d + 1, d)
        self.time_emb = TimeEmbedding(d, self.time_scale)
        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", Conv(d, f, kernel_size=k, padding=(k - 1) // 2)),
            ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(f)),
            ("dropout_1", nn.Dropout(self.dropout)),
            ("conv1d_2", Conv(f, f, kernel_size=k, padding=1)),
            ("relu_2", nn.ReLU()),
            ("layer_norm_2", nn.LayerNorm(f)),
            ("dropout_2", nn.Dropout(self.dropout)),
        ]))
        self.linear_layer = nn.Linear(self.conv_output_size, 1)

    def forward(self, xt, encoder_output, t, mask):
        h = self.proj(torch.cat([xt.unsqueeze(-1), encoder_output], dim=-1))
        h = h + self.time_emb(t).unsqueeze(1).expand(-1, h.size(1), -1)
        v = self.linear_layer(self.conv_layer(h)).squeeze(-1)
        return v if mask is None else v.masked_fill(mask, 0.0)

    def hip_weights(self) -> List[torch.Tensor]:
        cl = self.conv_layer
        te = self.time_emb.time_emb
        return [self.proj.weight, self.proj.bias, te[1].weight, te[1].bias, te[3].weight, te[3].bias,
                cl.conv1d_1.conv.weight, cl.conv1d_1.conv.bias, cl.layer_norm_1.weight, cl.layer_norm_1.bias,
                cl.conv1d_2.conv.weight, cl.conv1d_2.conv.bias, cl.layer_norm_2.weight, cl.layer_norm_2.bias,
                self.linear_layer.weight, self.linear_layer.bias]


def _hip_ok(t: torch.Tensor, module: nn.Module) -> bool:
    if not t.is_cuda:
        return False
    if torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters()):
        return False
    return module.hip_dims_ok()


def _lr_hip_ok(x: torch.Tensor) -> bool:
    """The HIP length regulator writes a fresh buffer (no autograd graph): it serves inference only.
    Under autograd (training, PVA.compute_loss -> Flamed.forward) the differentiable repeat_interleave
    path runs, as in the reference (pva.py:125-166)."""
    return x.is_cuda and not (torch.is_grad_enabled() and x.requires_grad)


class LengthRegulator(nn.Module):
    """Interleaved phone/silence length regulation (reference pva.py:119-170)."""

    def LR(self, x, phone_duration, sil_duration, src_lens, max_len, log_domain=False):
        if _lr_hip_ok(x):
            return hip_length_regulate(x, phone_duration, sil_duration, src_lens, max_len, log_domain)
        if log_domain:
            phone_duration = torch.clamp(torch.round(torch.exp(phone_duration) - 1), min=0)
            sil_duration = torch.clamp(torch.round(torch.exp(sil_duration) - 1), min=0)
        B, L, H = x.shape
        valid = torch.arange(L, device=x.device).unsqueeze(0) < src_lens.to(x.device).unsqueeze(1)
        zero = torch.zeros_like(phone_duration, dtype=torch.float32)
        pr = torch.clamp(torch.where(valid, phone_duration.float(), zero).round().long(), min=1)
        sr = torch.clamp(torch.where(valid, sil_duration.float(), zero).round().long(), min=0)
        seg = torch.stack((x, x[:, :1, :].expand(-1, L, -1)), dim=2).reshape(B, 2 * L, H)
        rep = torch.stack((pr, sr), dim=2).reshape(B, 2 * L)
        tgt_len = rep.sum(dim=1)
        out = [torch.repeat_interleave(seg[b], rep[b], dim=0) for b in range(B)]
        return pad(out, max_len), tgt_len

    def forward(self, x, phone_duration, sil_duration, src_lens, max_len):
        return self.LR(x, phone_duration, sil_duration, src_lens, max_len)


def hip_length_regulate(x, phone, sil, src_lens, max_len, log_domain=False):
    """torch.ops.flamed_hip.length_regulate (max_len None/0 = the batch's longest utterance)."""
    return ops.length_regulate(x, phone, sil, src_lens, int(max_len) if max_len else 0, bool(log_domain))


def hip_length_regulate_impl(x, phone, sil, src_lens, max_len, log_domain=False):
    """HIP length regulator: phase 1 (repeats + prefix sums), one host read of the lengths (the
    reference's .tolist() sync, pva.py:158), phase 2 (gather)."""
    L_ = nat.lib()
    dev = x.device
    B, L, H = x.shape
    xf = x.to(torch.float32).contiguous()
    pf = phone.to(device=dev, dtype=torch.float32).contiguous()
    sf = sil.to(device=dev, dtype=torch.float32).contiguous()
    sl = src_lens.to(device=dev, dtype=torch.int64).contiguous()
    cum = torch.empty((B, 2 * L + 1), dtype=torch.int64, device=dev)
    tgt = torch.empty((B,), dtype=torch.int64, device=dev)
    st = nat.stream_ptr(dev)
    nat.check(L_.flamed_lr_lengths(nat.ptr(pf), nat.ptr(sf), nat.ptr(sl), B, L, int(bool(log_domain)), nat.ptr(cum),
                                   nat.ptr(tgt), st), "flamed_lr_lengths")
    T = int(max_len) if max_len else int(tgt.max().item())
    out = torch.empty((B, T, H), dtype=torch.float32, device=dev)
    nat.check(L_.flamed_lr_expand(nat.ptr(xf), nat.ptr(cum), B, L, H, T, nat.ptr(out), st), "flamed_lr_expand")
    return out.to(x.dtype), tgt


class PVA(nn.Module):
    """Probabilistic variance adaptor (reference pva.py:44-116)."""

    def __init__(self, model_config):
        super().__init__()
        self.sigma_min = float(model_config["sigma_min"])
        self.duration_generator = ProbabilisticModule(model_config["duration_generator"])
        self.sil_generator = ProbabilisticModule(model_config["sil_generator"])
        self.length_regulator = LengthRegulator()
        self.hip_graph = True
        self._hip = None

    def compute_loss(self, x, src_len, src_mask, max_tgt_len, phone_duration, sil_duration):
        """reference pva.py:54-86 (training objective, torch ops)."""
        t = torch.rand((x.shape[0], 1)).to(x.device)
        k = 1 - self.sigma_min
        losses = {}
        for name, gen, dur in (("dur_loss", self.duration_generator, phone_duration),
                               ("sil_loss", self.sil_generator, sil_duration)):
            d1 = torch.log(dur.float() + 1)
            d0 = torch.randn_like(d1)
            dt_ = t * d1 + (1 - k * t) * d0
            u = (d1 - k * d0) * ~src_mask
            losses[name] = F.mse_loss(gen(dt_, x, t.squeeze(), src_mask), u)
        x, _ = self.length_regulator(x, phone_duration, sil_duration, src_len, max_tgt_len)
        return x, losses

    def flow(self, x, src_mask, nfe, temperature):
        """Euler loop of both generators (pva.py:97-109); returns final log-durations (dur, sil).
        Noise: dur then sil from the global CPU RNG, as the reference draws it."""
        b, l, _ = x.size()
        ts = torch.linspace(0, 1, nfe + 1, device=x.device)
        dur_t = torch.randn((b, l)).to(x.device) * temperature
        sil_t = torch.randn((b, l)).to(x.device) * temperature
        if _hip_ok(x, self):
            return ops.pva_flow(self.hip().oid, x, src_mask, dur_t, sil_t, ts, nfe)
        delta_t = 1 / nfe
        for i in range(1, len(ts)):
            dur_t = dur_t + delta_t * self.duration_generator(dur_t, x, ts[i - 1], src_mask)
            sil_t = sil_t + delta_t * self.sil_generator(sil_t, x, ts[i - 1], src_mask)
        return dur_t, sil_t

    def sample(self, x, src_len, src_mask, max_tgt_len=None, nfe=32, temperature=1.0):
        """reference pva.py:88-116"""
        dur_t, sil_t = self.flow(x, src_mask, nfe, temperature)
        if _lr_hip_ok(x):
            return self.length_regulator.LR(x, dur_t, sil_t, src_len, max_tgt_len, log_domain=True)
        phone_duration = torch.clamp(torch.round(torch.exp(dur_t) - 1), min=0)
        sil_duration = torch.clamp(torch.round(torch.exp(sil_t) - 1), min=0)
        return self.length_regulator(x, phone_duration, sil_duration, src_len, max_tgt_len)

    def hip_dims_ok(self) -> bool:
        """flamed_dur_create specialises both generators' dims; otherwise the torch ops run."""
        return all(nat.supported("dur", g.input_size, g.filter_size, g.kernel)
                   for g in (self.duration_generator, self.sil_generator))

    def hip(self) -> "PvaHIP":
        if self._hip is None:
            self._hip = PvaHIP(self)
        return self._hip

    def hip_invalidate(self):
        """Force the next HIP call to re-pack the weights (after an in-place weight update that
        load_state_dict does not cover)."""
        if self._hip is not None:
            self._hip._sig = None

    def _load_from_state_dict(self, *args, **kwargs):
        self.hip_invalidate()  # load_state_dict copies in place: same pointers, maybe no version bump
        super()._load_from_state_dict(*args, **kwargs)


class PvaHIP:
    """Owns the two flamed_dur_t handles of a PVA module."""

    def __init__(self, pva: PVA):
        self.pva = pva
        self.handles = [None, None]
        self._sig = None
        self._keep = []
        self.ws = nat.Workspace()
        self._bufs = {}
        # after a persistent flow: wait for it and re-run it on the graph path if the kernel reported a failure
        # (NaN states), so a failed launch never reaches the length regulator; skipped inside a stream capture
        # (the caller then owns the check: persist_status).  The length regulator reads max(tgt_len) on the
        # host right after the flow anyway (pva.py:158), so the wait costs little.
        self.check_persist = True
        self._fails_seen = 0
        self.oid = ops.register(self)  # torch.ops.flamed_hip.pva_flow

    def __del__(self):
        try:
            for h in self.handles:
                if h is not None:
                    nat.destroy(h, "flamed_dur_destroy")
        except Exception:
            pass

    def _ensure(self, dev):
        gens = (self.pva.duration_generator, self.pva.sil_generator)
        params = [w for g in gens for w in g.hip_weights()]
        sig = tuple((p.data_ptr(), nat.tensor_version(p)) for p in params) + (str(dev),)
        if sig == self._sig:
            return
        L = nat.lib()
        keep = []
        for i, g in enumerate(gens):
            if self.handles[i] is None:
                h = ctypes.c_void_p()
                nat.check(L.flamed_dur_create(g.input_size, g.filter_size, g.kernel, ctypes.byref(h)), "flamed_dur_create")
                self.handles[i] = h
                nat.track(h, "flamed_dur_destroy")
            ws = [w.detach().to(device=dev, dtype=torch.float32).contiguous() for w in g.hip_weights()]
            arr = (ctypes.c_void_p * len(ws))(*[t.data_ptr() for t in ws])
            nat.check(L.flamed_dur_load(self.handles[i], arr, len(ws), nat.stream_ptr(dev)), "flamed_dur_load")
            keep += ws
        self._keep = keep
        self._sig = sig
        self._bufs = {}

    def flow(self, x, src_mask, dur_t, sil_t, ts, nfe):
        dev = x.device
        self._ensure(dev)
        B, L, D = x.shape
        Lb = nat.lib()
        if self.pva.hip_graph and Lb.flamed_pva_persist_ready(self.handles[0], self.handles[1], B, L,
                                                              nat.stream_ptr(dev)) == 1:
            # one persistent launch, no captured graph keyed on buffer addresses: the caller's tensors go in
            # directly (the bool mask's bytes are the uint8 the kernel reads) and the states are flowed in
            # place in fresh copies (the op returns new tensors)
            enc = x.float().contiguous()
            mask = src_mask.contiguous()
            if mask.dtype not in (torch.bool, torch.uint8):
                mask = mask.to(torch.uint8)
            # contiguous copies: the kernel indexes the states flat (r = b L + l); clone() would keep the
            # strides of a dense non-contiguous input (preserve_format)
            d = dur_t.float().clone(memory_format=torch.contiguous_format)
            s = sil_t.float().clone(memory_format=torch.contiguous_format)
            tsc = ts.float().contiguous()
            ws = self.ws.get(Lb.flamed_pva_workspace_size(self.handles[0], B, L, nfe), dev)
            runs0, _ = self.persist_status()
            nat.check(Lb.flamed_pva_flow(self.handles[0], self.handles[1], nat.ptr(enc), nat.ptr(mask), nat.ptr(d),
                                         nat.ptr(s), nat.ptr(tsc), nfe, B, L, nat.ptr(ws), ws.numel(), 1,
                                         nat.stream_ptr(dev)), "flamed_pva_flow")
            if not (self.check_persist and not torch.cuda.is_current_stream_capturing()):
                return d, s
            runs1, _ = self.persist_status()
            if runs1 == runs0:  # the grid was refused: the call took the graph path
                return d, s
            torch.cuda.current_stream(dev).synchronize()  # also completes the failure count's copy
            _, fails = self.persist_status()
            if fails <= self._fails_seen:
                return d, s
            self._fails_seen = fails
            warnings.warn(f"flamed: persistent PVA flow failed ({fails} so far on this pair); "
                          "re-running it on the graph path")
            return self._graph_flow(x, src_mask, dur_t, sil_t, ts, nfe, 1 | 2)
        return self._graph_flow(x, src_mask, dur_t, sil_t, ts, nfe, int(bool(self.pva.hip_graph)))

    def _graph_flow(self, x, src_mask, dur_t, sil_t, ts, nfe, use_graph):
        dev = x.device
        self._ensure(dev)
        B, L, D = x.shape
        Lb = nat.lib()
        key = (B, L, nfe)
        bufs = self._bufs.get(key)
        if bufs is None:
            bufs = {"enc": torch.empty((B, L, D), dtype=torch.float32, device=dev),
                    "mask": torch.empty((B, L), dtype=torch.uint8, device=dev),
                    "dur": torch.empty((B, L), dtype=torch.float32, device=dev),
                    "sil": torch.empty((B, L), dtype=torch.float32, device=dev),
                    "ts": torch.empty((nfe + 1,), dtype=torch.float32, device=dev)}
            self._bufs = {key: bufs}
        bufs["enc"].copy_(x)
        bufs["mask"].copy_(src_mask)
        bufs["dur"].copy_(dur_t)
        bufs["sil"].copy_(sil_t)
        bufs["ts"].copy_(ts)
        ws = self.ws.get(Lb.flamed_pva_workspace_size(self.handles[0], B, L, nfe), dev)
        nat.check(Lb.flamed_pva_flow(self.handles[0], self.handles[1], nat.ptr(bufs["enc"]), nat.ptr(bufs["mask"]),
                                     nat.ptr(bufs["dur"]), nat.ptr(bufs["sil"]), nat.ptr(bufs["ts"]), nfe, B, L,
                                     nat.ptr(ws), ws.numel(), use_graph, nat.stream_ptr(dev)),
                  "flamed_pva_flow")
        return bufs["dur"].clone(), bufs["sil"].clone()

    def persist_status(self):
        """(persistent flows enqueued, failed launches as of the last completed copy) of this pair; never waits."""
        if self.handles[0] is None:
            return 0, 0
        runs, fails = ctypes.c_int(), ctypes.c_int()
        nat.check(nat.lib().flamed_pva_persist_status(self.handles[0], ctypes.byref(runs), ctypes.byref(fails)),
                  "flamed_pva_persist_status")
        return runs.value, fails.value

    def persist_info(self):
        """(persistent flows completed, timed out, device ms of the last one) on this pair (pvaflow.hip)."""
        if self.handles[0] is None:
            return 0, False, 0.0
        runs, broken, ms = ctypes.c_int(), ctypes.c_int(), ctypes.c_float()
        nat.check(nat.lib().flamed_pva_persist_info(self.handles[0], ctypes.byref(runs), ctypes.byref(broken),
                                                    ctypes.byref(ms)), "flamed_pva_persist_info")
        return runs.value, bool(broken.value), ms.value
