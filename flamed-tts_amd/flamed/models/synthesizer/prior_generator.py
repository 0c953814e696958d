"""PriorGenerator — text encoder, PVA (HIP duration flow + length regulator on GPU), shared and six
per-quantizer prompt-prefixed decoders, code head (drop-in for reference
flamed/models/synthesizer/prior_generator.py; same state-dict keys).

On ROCm tensors at inference the transformer parts run in the HIP library:
`flamed_prior_encode` (embedding + position + the encoder's FFT blocks) before the PVA and
`flamed_prior_decode` (bridge, shared decoder, six prompt-prefixed decoders, head, masked logits)
after it, each one graph-captured native call (`PriorHIP`, torch.ops.flamed_hip.prior_encode /
prior_decode).  CPU tensors and autograd training use the modules' own torch ops."""
from __future__ import annotations

import ctypes
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed import _native as nat
from flamed import ops
from flamed.models.module import Encoder, Decoder
from flamed.models.module.transformer import get_sinusoid_encoding_table
from flamed.utils.tools import get_mask_from_lengths
from .pva import PVA


class PreEncoding(nn.Module):
    """Adds prompt / target segment embeddings and the quantizer-index embedding (reference :12-26)."""

    def __init__(self, hidden_dim, n_quantizer):
        super().__init__()
        self.prompt_emb = nn.Parameter(torch.rand(1, 1, hidden_dim))
        self.target_emb = nn.Parameter(torch.rand(1, 1, hidden_dim))
        self.quantizer_emb = nn.Embedding(n_quantizer, hidden_dim)

    def forward(self, x, prompt_len, q_idx):
        b, l, _ = x.shape
        seg = torch.cat([self.prompt_emb.expand(b, prompt_len, -1), self.target_emb.expand(b, l - prompt_len, -1)], 1)
        q = self.quantizer_emb(torch.tensor([q_idx], device=x.device))
        return (x + seg.to(x.device)) + q.unsqueeze(0).expand(b, l, -1)


class PriorGenerator(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        tc = config["transformer"]
        vocab = config["codec"]["vocab_size"]
        nq = config["codec"]["n_quantizers"]
        self.encoder = Encoder(config)
        self.pva = PVA(config["variance_adaptor"])
        self.bridge = nn.Linear(tc["encoder_hidden"], tc["decoder_hidden"])
        self.code_embedding = nn.Embedding(vocab + 1, tc["decoder_hidden"], padding_idx=vocab)
        self.shared_decoder = Decoder(config, tc["decoder_shared_layers"])
        self.pre_encode = PreEncoding(tc["decoder_hidden"], nq)
        self.prior_decoder = nn.ModuleList([Decoder(config, tc["decoder_layers"][i]) for i in range(nq)])
        self.head = nn.Linear(tc["decoder_hidden"], vocab + 1)
        self.hip_graph = True
        # decoder-side GEMM operands on the HIP path: "bf16" (fp32 accumulation; the encoder, which feeds the
        # rounded durations, always stays fp32) or "f32" (exact, the reference's arithmetic)
        self.hip_dec_dtype = "bf16"
        self._hip = None

    # -- HIP dispatch (inference on ROCm tensors)
    def _use_hip(self, x: torch.Tensor) -> bool:
        if not x.is_cuda:
            return False
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return False  # autograd training: the HIP path is inference-only
        return self.hip_dims_ok()

    def hip_dims_ok(self) -> bool:
        """flamed_prior_create specialises these dims (head widths 32 / 48, ...); else torch ops."""
        d = PriorHIP.dims_of(self)
        return nat.supported("prior", tuple(d), len(d))

    def hip(self) -> "PriorHIP":
        if self._hip is None:
            self._hip = PriorHIP(self)
        return self._hip

    def hip_invalidate(self):
        if self._hip is not None:
            self._hip._sig = None

    def _load_from_state_dict(self, *args, **kwargs):
        self.hip_invalidate()
        super()._load_from_state_dict(*args, **kwargs)

    def _decode(self, output, tgt_lens, tgt_masks, prompts, prompts_len):
        output, tgt_masks = self.shared_decoder(output, tgt_masks)
        dec_mask = get_mask_from_lengths(prompts_len + tgt_lens, prompts_len + output.size(1))
        prompt_embs = self.code_embedding(prompts)
        hiddens = []
        for i, layer in enumerate(self.prior_decoder):
            q = self.pre_encode(torch.cat([prompt_embs[:, i], output], dim=1), prompts_len, i)
            output, dec_mask = layer(q, dec_mask)
            output = output[:, prompts_len:, :]
            hiddens.append(output.unsqueeze(1))
        output = torch.cat(hiddens, dim=1)
        logits = self.head(output)
        logits = logits * ~tgt_masks.unsqueeze(1).expand(-1, logits.size(1), -1).unsqueeze(3)
        return output, logits.permute(0, 3, 1, 2).contiguous(), tgt_masks

    def compute_loss(self, texts, src_lens, max_src_len, codes, tgt_lens, max_tgt_len, phone_durations,
                     sil_durations, prompts, prompts_len):
        """reference :64-139 (training objective)."""
        src_masks = get_mask_from_lengths(src_lens, max_src_len)
        tgt_masks = get_mask_from_lengths(tgt_lens, max_tgt_len) if tgt_lens is not None else None
        output = self.encoder(texts, src_masks)
        output, pva_losses = self.pva.compute_loss(output, src_lens, src_masks, max_tgt_len, phone_durations,
                                                   sil_durations)
        output, logits, tgt_masks = self._decode(self.bridge(output), tgt_lens, tgt_masks, prompts, prompts_len)
        loss = sum(F.cross_entropy(logits[:, :, i, :], codes[:, i, :]) for i in range(codes.size(1))) / codes.size(1)
        return output, tgt_masks, pva_losses | {"prior_loss": loss}

    def sample(self, texts, src_lens, max_src_len, prompts, prompts_len, nfe=4, temperature=1.0):
        """reference :141-196 -> (prior embeddings (B,Q,T,D), logits (B,V+1,Q,T), tgt mask (B,T))."""
        src_masks = get_mask_from_lengths(src_lens, max_src_len)
        hip = self._use_hip(texts)
        output = ops.prior_encode(self.hip().oid, texts, src_masks) if hip else self.encoder(texts, src_masks)
        output, tgt_lens = self.pva.sample(output, src_lens, src_masks, nfe=nfe, temperature=temperature)
        tgt_masks = get_mask_from_lengths(tgt_lens, output.size(1))
        if hip:
            embs, logits = ops.prior_decode(self.hip().oid, output, tgt_masks, prompts, int(prompts_len))
            return embs, logits, tgt_masks
        return self._decode(self.bridge(output), tgt_lens, tgt_masks, prompts, prompts_len)


def _fft_layer_weights(layer) -> List[torch.Tensor]:
    """One FFTBlock in the flamed_prior_load order (include/flamed_hip.h)."""
    a, f = layer.slf_attn, layer.pos_ffn
    return [a.w_qs.weight, a.w_qs.bias, a.w_ks.weight, a.w_ks.bias, a.w_vs.weight, a.w_vs.bias, a.fc.weight, a.fc.bias,
            a.layer_norm.weight, a.layer_norm.bias, f.w_1.weight, f.w_1.bias, f.w_2.weight, f.w_2.bias,
            f.layer_norm.weight, f.layer_norm.bias]


def prior_weight_list(pg: PriorGenerator) -> List[torch.Tensor]:
    w = [pg.encoder.src_word_emb.weight, pg.encoder.position_enc]
    for ly in pg.encoder.layer_stack:
        w += _fft_layer_weights(ly)
    w += [pg.bridge.weight, pg.bridge.bias, pg.code_embedding.weight, pg.shared_decoder.position_enc]
    for ly in pg.shared_decoder.layer_stack:
        w += _fft_layer_weights(ly)
    w += [pg.pre_encode.prompt_emb, pg.pre_encode.target_emb, pg.pre_encode.quantizer_emb.weight]
    for dec in pg.prior_decoder:
        w.append(dec.position_enc)
        for ly in dec.layer_stack:
            w += _fft_layer_weights(ly)
    return w + [pg.head.weight, pg.head.bias]


class PriorHIP:
    """Owns one flamed_prior_t handle (the prior transformer stack of a PriorGenerator on one device)."""

    def __init__(self, pg: PriorGenerator):
        self.pg = pg
        self.handle = None
        self._sig = None
        self._keep = []
        self.ws = nat.Workspace()
        self._bufs = {}
        self.oid = ops.register(self)  # torch.ops.flamed_hip.prior_encode / prior_decode

    def __del__(self):
        try:
            if self.handle is not None:
                nat.destroy(self.handle, "flamed_prior_destroy")
        except Exception:
            pass

    def dims(self) -> List[int]:
        return PriorHIP.dims_of(self.pg)

    @staticmethod
    def dims_of(pg: PriorGenerator) -> List[int]:
        tc = pg.config["transformer"]
        e, s = pg.encoder, pg.shared_decoder
        n_sym = e.src_word_emb.weight.shape[0] - 1
        return [n_sym, tc["encoder_hidden"], tc["encoder_head"], tc["encoder_conv_filter_size"],
                *tc["encoder_conv_kernel_size"], len(e.layer_stack), e.max_seq_len,
                tc["decoder_hidden"], tc["decoder_head"], tc["decoder_conv_filter_size"],
                *tc["decoder_conv_kernel_size"], len(s.layer_stack), s.max_seq_len,
                pg.head.weight.shape[0] - 1, len(pg.prior_decoder), *[len(d.layer_stack) for d in pg.prior_decoder]]

    def _ensure(self, dev):
        params = prior_weight_list(self.pg)
        sig = tuple((p.data_ptr(), nat.tensor_version(p)) for p in params) + (str(dev),)
        if sig == self._sig and self.handle is not None:
            return
        L = nat.lib()
        if self.handle is None:
            h = ctypes.c_void_p()
            d = self.dims()
            nat.check(L.flamed_prior_create((ctypes.c_int * len(d))(*d), len(d), ctypes.byref(h)), "flamed_prior_create")
            self.handle = h
            nat.track(h, "flamed_prior_destroy")
        keep = [p.detach().to(device=dev, dtype=torch.float32).contiguous() for p in params]
        arr = (ctypes.c_void_p * len(keep))(*[t.data_ptr() for t in keep])
        nat.check(L.flamed_prior_load(self.handle, arr, len(keep), nat.stream_ptr(dev)), "flamed_prior_load")
        torch.cuda.current_stream(dev).synchronize()  # the arena copies read `keep`
        self._sig = sig
        self._bufs = {}

    def _buf(self, key, make):
        """Persistent I/O buffers of the latest shape per call kind (their pointers key the captured
        graph); a new shape replaces the previous buffers instead of accumulating one set per length."""
        b = self._bufs.get(key)
        if b is None:
            b = make()
            self._bufs = {k: v for k, v in self._bufs.items() if k[0] != key[0]}
            self._bufs[key] = b
        return b

    def encode(self, texts: torch.Tensor, src_mask: torch.Tensor) -> torch.Tensor:
        """texts (B, L) int, src_mask (B, L) bool (True = padding) -> encoder output (B, L, hidden)."""
        dev = texts.device
        self._ensure(dev)
        B, n = texts.shape
        D = self.pg.encoder.d_model
        bufs = self._buf(("enc", B, n), lambda: {
            "ids": torch.empty((B, n), dtype=torch.int64, device=dev),
            "mask": torch.empty((B, n), dtype=torch.uint8, device=dev),
            "out": torch.empty((B, n, D), dtype=torch.float32, device=dev),
            "pos": (get_sinusoid_encoding_table(n, D).to(dev) if n > self.pg.encoder.max_seq_len else None)})
        bufs["ids"].copy_(texts)
        bufs["mask"].copy_(src_mask[:, :n])
        L = nat.lib()
        ws = self.ws.get(L.flamed_prior_workspace_size(self.handle, B, n, 0, 0), dev)
        nat.check(L.flamed_prior_encode(self.handle, nat.ptr(bufs["ids"]), nat.ptr(bufs["mask"]), B, n,
                                        nat.ptr(bufs["pos"]), nat.ptr(bufs["out"]), nat.ptr(ws), ws.numel(),
                                        int(bool(self.pg.hip_graph)), nat.stream_ptr(dev)), "flamed_prior_encode")
        return bufs["out"].clone()

    def decode(self, x: torch.Tensor, tgt_mask: torch.Tensor, prompts: torch.Tensor, P: int):
        """x (B, T, enc hidden) regulated encoder output, tgt_mask (B, T) bool, prompts (B, n_q, P) codes ->
        (prior embeddings (B, n_q, T, hidden), logits (B, vocab+1, n_q, T))."""
        dev = x.device
        self._ensure(dev)
        B, T, De = x.shape
        pg = self.pg
        D, nq, V1 = pg.shared_decoder.d_model, len(pg.prior_decoder), pg.head.weight.shape[0]
        n = P + T
        bufs = self._buf(("dec", B, T, P), lambda: {
            "x": torch.empty((B, T, De), dtype=torch.float32, device=dev),
            "mask": torch.empty((B, T), dtype=torch.uint8, device=dev),
            "prompts": torch.zeros((B, nq, max(P, 1)), dtype=torch.int64, device=dev),
            "embs": torch.empty((B, nq, T, D), dtype=torch.float32, device=dev),
            "logits": torch.empty((B, V1, nq, T), dtype=torch.float32, device=dev),
            "pos": (get_sinusoid_encoding_table(n, D).to(dev) if n > pg.shared_decoder.max_seq_len else None)})
        bufs["x"].copy_(x)
        bufs["mask"].copy_(tgt_mask)
        if P:
            bufs["prompts"].copy_(prompts)
        L = nat.lib()
        if pg.hip_dec_dtype not in ("bf16", "f32"):
            raise ValueError(f"PriorGenerator.hip_dec_dtype must be 'bf16' or 'f32' (got {pg.hip_dec_dtype!r})")
        nat.check(L.flamed_prior_set_dtype(self.handle, nat.FLAMED_BF16 if pg.hip_dec_dtype == "bf16" else nat.FLAMED_F32),
                  "flamed_prior_set_dtype")
        ws = self.ws.get(L.flamed_prior_workspace_size(self.handle, B, 0, T, P), dev)
        nat.check(L.flamed_prior_decode(self.handle, nat.ptr(bufs["x"]), nat.ptr(bufs["mask"]), nat.ptr(bufs["prompts"]),
                                        B, T, P, nat.ptr(bufs["pos"]), nat.ptr(bufs["embs"]), nat.ptr(bufs["logits"]),
                                        nat.ptr(ws), ws.numel(), int(bool(pg.hip_graph)), nat.stream_ptr(dev)),
                  "flamed_prior_decode")
        return bufs["embs"].clone(), bufs["logits"].clone()
