"""torch.library custom-op layer over the HIP library (`flamed_hip::den_step` & co.).

Every hot-path entry point the modules dispatch to on ROCm is registered as a PyTorch custom op in the
`flamed_hip` namespace, so the calls are visible to the dispatcher: `torch.compile` (dynamo traces them
as single opaque nodes instead of graph-breaking on ctypes), FakeTensor / meta shape propagation, and
`torch.library.opcheck`.  The ops are thin: the work is done by the per-module owner objects
(`DenoiserHIP`, `CondFoldHIP`, `PvaHIP`, `FacDecoderHIP`, `EncoderHIP`, `VqHIP`, `PriorHIP`), which own the native handles and
their device-resident weight arenas.  An owner is passed to an op by an integer id (custom-op schemas
take tensors and scalars only); the registry holds weak references, so a dropped module frees its handle.

  op                                    reference function it stands for
  flamed_hip::den_velocity(id, x, t, c)            SimpleMLPAdaLN.forward          prob_generator.py:349-365
  flamed_hip::den_solve(id, xt, ts, spk, nfe)      ProbGenerator.sample Euler loop prob_generator.py:439-445
  flamed_hip::cond_fold(id, cond, mask)            QuantizerEncoding + ConditionDownSampler :167-205, 435-436
  flamed_hip::pva_flow(id, x, mask, dur, sil, ts, nfe)  PVA.sample Euler loops       pva.py:97-109
  flamed_hip::length_regulate(x, pd, sd, lens, max_len, log_domain)  LengthRegulator.LR  pva.py:125-166
  flamed_hip::fac_decode(id, x, spk)               FACodecDecoder.inference        facodec.py:630-638
  flamed_hip::enc_encode(id, x)                    FACodecEncoder.forward          facodec.py:158-243
  flamed_hip::vq_encode(id, x)                     FACodecDecoder.forward(vq=True) facodec.py:470-533
  flamed_hip::prior_encode(id, texts, mask)        Encoder.forward (prior)         prior_generator.py:152-153
  flamed_hip::prior_decode(id, x, mask, prompts, P) bridge + decoders + head       prior_generator.py:165-188

None of the ops has an autograd formula: the modules route autograd (training) to their torch ops
before reaching here, exactly as the reference trains.  There is no CPU kernel: the ops are registered
for every device, and the owners raise if the HIP library is missing (no fallback).
"""
from __future__ import annotations

import itertools
import threading
import weakref
from typing import Tuple

import torch
from torch import Tensor

_ids = itertools.count(1)
_owners: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()
_lock = threading.Lock()


def register(owner) -> int:
    """Give a HIP owner object an id the custom ops can carry."""
    with _lock:
        i = next(_ids)
        _owners[i] = owner
    return i


def owner(i: int):
    o = _owners.get(int(i))
    if o is None:
        raise RuntimeError(f"flamed_hip: no live HIP owner with id {i}")
    return o


# ---------------------------------------------------------------- denoiser

@torch.library.custom_op("flamed_hip::den_velocity", mutates_args=())
def den_velocity(oid: int, x: Tensor, t: Tensor, c: Tensor) -> Tensor:
    return owner(oid).velocity(x, t, c)


@den_velocity.register_fake
def _(oid, x, t, c):
    return x.new_empty(x.shape, dtype=x.dtype)


@torch.library.custom_op("flamed_hip::den_solve", mutates_args=())
def den_solve(oid: int, xt: Tensor, ts: Tensor, spk: Tensor, nfe: int) -> Tensor:
    return owner(oid).solve(xt, ts, spk, nfe)


@den_solve.register_fake
def _(oid, xt, ts, spk, nfe):
    return xt.new_empty(xt.shape, dtype=torch.float32)


@torch.library.custom_op("flamed_hip::cond_fold", mutates_args=())
def cond_fold(oid: int, cond: Tensor, mask: Tensor) -> Tensor:
    return owner(oid).fold(cond, mask)


@cond_fold.register_fake
def _(oid, cond, mask):
    B, _, T, _ = cond.shape
    return cond.new_empty((B, T, owner(oid).pg.target_dim), dtype=torch.float32)


# ---------------------------------------------------------------- PVA + length regulator

@torch.library.custom_op("flamed_hip::pva_flow", mutates_args=())
def pva_flow(oid: int, x: Tensor, src_mask: Tensor, dur_t: Tensor, sil_t: Tensor, ts: Tensor,
             nfe: int) -> Tuple[Tensor, Tensor]:
    return owner(oid).flow(x, src_mask, dur_t, sil_t, ts, nfe)


@pva_flow.register_fake
def _(oid, x, src_mask, dur_t, sil_t, ts, nfe):
    return (dur_t.new_empty(dur_t.shape, dtype=torch.float32), sil_t.new_empty(sil_t.shape, dtype=torch.float32))


@torch.library.custom_op("flamed_hip::length_regulate", mutates_args=())
def length_regulate(x: Tensor, phone: Tensor, sil: Tensor, src_lens: Tensor, max_len: int,
                    log_domain: bool) -> Tuple[Tensor, Tensor]:
    from .models.synthesizer.pva import hip_length_regulate_impl
    return hip_length_regulate_impl(x, phone, sil, src_lens, max_len, log_domain)


@length_regulate.register_fake
def _(x, phone, sil, src_lens, max_len, log_domain):
    B, _, H = x.shape
    # the regulated length is data-dependent unless max_len pins it (the reference's `.tolist()` sync)
    T = max_len if max_len else torch.library.get_ctx().new_dynamic_size()
    return x.new_empty((B, T, H)), src_lens.new_empty((B,), dtype=torch.int64)


# ---------------------------------------------------------------- FaCodec

@torch.library.custom_op("flamed_hip::fac_decode", mutates_args=())
def fac_decode(oid: int, x: Tensor, spk: Tensor) -> Tensor:
    return owner(oid).decode(x, spk)


@fac_decode.register_fake
def _(oid, x, spk):
    B, _, T = x.shape
    return x.new_empty((B, 1, owner(oid).dec.hop_length * T), dtype=torch.float32)


@torch.library.custom_op("flamed_hip::enc_encode", mutates_args=())
def enc_encode(oid: int, x: Tensor) -> Tensor:
    return owner(oid).encode(x)


@enc_encode.register_fake
def _(oid, x):
    o = owner(oid)
    B, _, n = x.shape
    return x.new_empty((B, o.enc.out_channels, o.out_len(n)), dtype=torch.float32)


@torch.library.custom_op("flamed_hip::vq_encode", mutates_args=())
def vq_encode(oid: int, x: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    return owner(oid).encode(x)


@vq_encode.register_fake
def _(oid, x):
    B, C, T = x.shape
    q = owner(oid).dec.quantizer
    nq = sum(len(r.layers) for r in q)
    return (x.new_empty((B, C, T)), x.new_empty((nq, B, T), dtype=torch.int64), x.new_empty((len(q), B, C, T)),
            x.new_empty((B, C)))


# ---------------------------------------------------------------- prior transformer stack

@torch.library.custom_op("flamed_hip::prior_encode", mutates_args=())
def prior_encode(oid: int, texts: Tensor, src_mask: Tensor) -> Tensor:
    return owner(oid).encode(texts, src_mask)


@prior_encode.register_fake
def _(oid, texts, src_mask):
    B, n = texts.shape
    return texts.new_empty((B, n, owner(oid).pg.encoder.d_model), dtype=torch.float32)


@torch.library.custom_op("flamed_hip::prior_decode", mutates_args=())
def prior_decode(oid: int, x: Tensor, tgt_mask: Tensor, prompts: Tensor, prompts_len: int) -> Tuple[Tensor, Tensor]:
    return owner(oid).decode(x, tgt_mask, prompts, prompts_len)


@prior_decode.register_fake
def _(oid, x, tgt_mask, prompts, prompts_len):
    B, T, _ = x.shape
    pg = owner(oid).pg
    nq, D, V1 = len(pg.prior_decoder), pg.shared_decoder.d_model, pg.head.weight.shape[0]
    return x.new_empty((B, nq, T, D)), x.new_empty((B, V1, nq, T))


OPS = ("den_velocity", "den_solve", "cond_fold", "pva_flow", "length_regulate", "fac_decode", "enc_encode",
       "vq_encode", "prior_encode", "prior_decode")
