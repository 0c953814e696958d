"""PriorGenerator — text encoder, PVA (HIP duration flow + length regulator on GPU), shared and six
per-quantizer prompt-prefixed decoders, code head (drop-in for reference
flamed/models/synthesizer/prior_generator.py; same state-dict keys).  The transformer parts run on
PyTorch ops; the PVA part is the HIP path of flamed/models/synthesizer/pva.py."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from flamed.models.module import Encoder, Decoder
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
        output = self.encoder(texts, src_masks)
        output, tgt_lens = self.pva.sample(output, src_lens, src_masks, nfe=nfe, temperature=temperature)
        output = self.bridge(output)
        tgt_masks = get_mask_from_lengths(tgt_lens, output.size(1))
        return self._decode(output, tgt_lens, tgt_masks, prompts, prompts_len)
