"""Per-stage wall time of the end-to-end synthesis path on the GPU (seeded random weights):
frontend, prompt encode, text encoder, PVA, prior decoders, denoiser (cond fold + solve), decode.
Usage: python tools/e2e_profile.py [--batch B] [--phonemes L] [--prompt-sec S] [--nfe N] [--iters K]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from flamed.utils.seeded_init import fill_state_dict  # noqa: E402


def build(dev, dtype):
    import yaml
    from flamed import Flamed
    from flamed.utils.random_ckpt import codec_models, load_yaml
    cfg = {"prior_generator": load_yaml("prior.yaml"), "prob_generator": load_yaml("prob.yaml")}
    m = Flamed(cfg).eval()
    m.load_state_dict(fill_state_dict(m.state_dict(), 20251205))
    enc, dec = codec_models(load_yaml("codec.yaml"))
    enc.load_state_dict(fill_state_dict(enc.state_dict(), 20251205))
    dec.load_state_dict(fill_state_dict(dec.state_dict(), 20251205))
    m.prob_generator.denoiser.hip_dtype = dtype
    dec.hip_dtype = dtype
    return m.to(dev), enc.eval().to(dev), dec.eval().to(dev)


class Clock:
    def __init__(self, dev):
        self.dev, self.t, self.rows = dev, None, {}

    def __enter__(self):
        torch.cuda.synchronize(self.dev)
        self.t = time.perf_counter()
        return self

    def lap(self, name):
        torch.cuda.synchronize(self.dev)
        now = time.perf_counter()
        self.rows.setdefault(name, []).append((now - self.t) * 1e3)
        self.t = now

    def __exit__(self, *a):
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--phonemes", type=int, default=60)
    ap.add_argument("--prompt-sec", type=float, default=3.0)
    ap.add_argument("--nfe", type=int, default=128)
    ap.add_argument("--nfe-durgen", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--fixed-seed", action="store_true", help="same PVA noise every iteration (same T)")
    ap.add_argument("--torch-prof", action="store_true", help="print a torch.profiler table of the last iteration")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m, enc, dec = build(dev, a.dtype)
    pg, prob = m.prior_generator, m.prob_generator
    from flamed.utils.tools import get_mask_from_lengths
    B, L = a.batch, a.phonemes
    g = torch.Generator().manual_seed(0)
    phon = torch.randint(1, 300, (B, L), generator=g).to(dev)
    src_lens = torch.full((B,), L, dtype=torch.long, device=dev)
    n = int(a.prompt_sec * 16000)
    wav = (0.1 * torch.randn(1, 1, n, generator=g)).to(dev)
    timbres = torch.randn(B, 256, generator=g).to(dev)
    ck = Clock(dev)
    text = "the quick brown fox jumps over the lazy dog, and then it runs far away into the forest."
    prof = None
    for it in range(a.iters + 1):
        if a.torch_prof and it == a.iters:
            prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                      torch.profiler.ProfilerActivity.CUDA])
            prof.__enter__()
        with torch.inference_mode(), ck:
            m._preprocess_english(text)
            ck.lap("frontend (text->phonemes, CPU)")
            z = enc(wav)
            ck.lap("prompt encoder (FACodecEncoder)")
            _, codes, _, _, spk = dec(z, eval_vq=False, vq=True)
            ck.lap("prompt RVQ + timbre transformer")
            prompts = codes.permute(1, 0, 2).expand(B, -1, -1).contiguous()
            P = prompts.size(-1)
            src_masks = get_mask_from_lengths(src_lens, L)
            out = pg.encoder(phon, src_masks)
            ck.lap("text encoder (transformer)")
            torch.manual_seed(0 if a.fixed_seed else it)
            out, tgt_lens = pg.pva.sample(out, src_lens, src_masks, nfe=a.nfe_durgen, temperature=0.3)
            ck.lap("PVA flow + length regulator (HIP)")
            out = pg.bridge(out)
            tgt_masks = get_mask_from_lengths(tgt_lens, out.size(1))
            pe, pl, tm = pg._decode(out, tgt_lens, tgt_masks, prompts, P)
            ck.lap("prior decoders + head (transformer)")
            lat = prob.sample(cond=pe, spk=timbres, nfe=a.nfe, temperature=0.3, mask=~tm.unsqueeze(-1))
            ck.lap("cond fold + denoiser solve (HIP)")
            w = dec.inference(lat, timbres)
            ck.lap("FaCodec decode (HIP)")
            w.cpu()
            ck.lap("D2H")
        if it == 0:
            ck.rows = {}
    if prof is not None:
        prof.__exit__(None, None, None)
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
        print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=25))
    T = int(tgt_lens.max())
    rows = {k: float(np.median(v)) for k, v in ck.rows.items()}
    total = sum(rows.values())
    audio = B * T * 200 / 16000.0
    print(f"B={B} L={L} P={P} T={T} nfe={a.nfe} dtype={a.dtype}  audio={audio:.2f}s")
    for k, v in rows.items():
        print(f"  {k:40s} {v:9.2f} ms  {100 * v / total:5.1f}%")
    print(f"  {'total':40s} {total:9.2f} ms   RTF(prompt-mode-like)={total / 1e3 / audio:.4f}")
    print(json.dumps({"B": B, "T": T, "P": P, "rows_ms": rows, "total_ms": total, "audio_s": audio}))


if __name__ == "__main__":
    main()
