#!/usr/bin/env python3
"""Unified Flamed-TTS synthesis CLI (drop-in for the reference synthesize.py).

Same flags, modes, validation errors and RTF bookkeeping as the reference (synthesize.py:1-386):
  * prompt-list mode (`--text --prompt-list`): RTF = mean over prompts of `Flamed.sample()` wall time
    (frontend + prompt encode + prior/PVA + denoiser + decode + D2H) / (len(wav)/16000)
    (reference :165-217);
  * metadata mode (`--metadata-file`, lines `target|prompt|text`): batches of `--batch-size`, per-sample
    time = `sample_batch()['time'] / len(batch)` (decode excluded, reference :220-303).
On a ROCm device the denoiser solve, PVA flow + length regulator and FaCodec decoder run in the gfx950
HIP library (flamed/_native); `--device cpu` runs the torch path.

Multi-GPU: launched under torchrun (one process per GPU, `--master-addr 127.0.0.1`), each rank takes a
shard of the prompts (round-robin) / metadata entries (length buckets balanced by total length,
flamed.utils.dist.bucket_shard) on cuda:LOCAL_RANK, seeded seed + rank with --seed; there is no data-path
collective, only the timing records are gathered for the RTF printed by rank 0.

Additions (all optional; the reference's invocations behave the same):
  * `--codec-ckpt-dir DIR` — where ns3_facodec_{encoder,decoder}.bin live (reference: fixed path under
    flamed/models/facodec/checkpoints, :72-73);
  * a second summary line with latent frames/s over the measured sample time.
Config files are read with yaml.safe_load (omegaconf is not installed); checkpoints with
torch.load(weights_only=True) only.  `python -m flamed.utils.random_ckpt --out-dir D` writes a seeded
random-init checkpoint + config + codec weights (BASELINE config 0).
"""
import argparse
import math
import os
import sys
from typing import Dict, List, Optional, Tuple

import torch
import yaml
from torch.nn.utils.rnn import pad_sequence

CURDIR = os.path.dirname(os.path.abspath(__file__))
if CURDIR not in sys.path:
    sys.path.insert(0, CURDIR)

from flamed import Flamed  # noqa: E402
from flamed.models.facodec import FACodecEncoder, FACodecDecoder  # noqa: E402
from flamed.utils import dist as fdist  # noqa: E402
from flamed.utils.audio import load_wav, write_wav  # noqa: E402

SR = 16000
HOP = 200  # FaCodec samples per latent frame


def _progress(it, total=None, desc=""):
    try:
        from tqdm import tqdm
        return tqdm(it, total=total, desc=desc)
    except ImportError:  # pragma: no cover
        return it


def str2bool(value):
    if isinstance(value, bool):
        return value
    value = str(value).strip().lower()
    if value in {"true", "1", "yes", "y"}:
        return True
    if value in {"false", "0", "no", "n"}:
        return False
    raise argparse.ArgumentTypeError(f"Cannot interpret '{value}' as boolean.")


def resolve_device(device_str: str) -> torch.device:
    device = torch.device(device_str)
    if device.type.startswith("cuda") and not torch.cuda.is_available():
        print("CUDA not available. Falling back to CPU.")
        return torch.device("cpu")
    _, world, local = fdist.dist_env()
    if device.type == "cuda" and world > 1:  # one GPU per rank
        device = torch.device("cuda", local)
    return device


def load_audio(wav_path: str) -> torch.Tensor:
    return torch.from_numpy(load_wav(wav_path, sr=SR)).float().unsqueeze(0).unsqueeze(0)


def get_codec(device: torch.device, ckpt_dir: Optional[str] = None):
    """FaCodec encoder/decoder with the reference's fixed hyper-parameters (synthesize.py:46-79)."""
    fa_encoder = FACodecEncoder(ngf=32, up_ratios=[2, 4, 5, 5], out_channels=256)
    fa_decoder = FACodecDecoder(in_channels=256, upsample_initial_channel=1024, ngf=32, up_ratios=[5, 5, 4, 2],
                                vq_num_q_c=2, vq_num_q_p=1, vq_num_q_r=3, vq_dim=256, codebook_dim=8,
                                codebook_size_prosody=10, codebook_size_content=10, codebook_size_residual=10,
                                use_gr_x_timbre=True, use_gr_residual_f0=True, use_gr_residual_phone=True)
    ckpt_dir = ckpt_dir or os.path.join(CURDIR, "flamed", "models", "facodec", "checkpoints")
    enc_path = os.path.join(ckpt_dir, "ns3_facodec_encoder.bin")
    dec_path = os.path.join(ckpt_dir, "ns3_facodec_decoder.bin")
    for p in (enc_path, dec_path):
        if not os.path.isfile(p):
            raise FileNotFoundError(f"FaCodec checkpoint not found: {p} (pass --codec-ckpt-dir)")
    fa_encoder.load_state_dict(torch.load(enc_path, map_location=device, weights_only=True))
    fa_decoder.load_state_dict(torch.load(dec_path, map_location=device, weights_only=True))
    fa_encoder.to(device).eval()
    fa_decoder.to(device).eval()
    return fa_encoder, fa_decoder


def prepare_model(cfg_path: str, ckpt_path: str, device: torch.device, weights_only: bool):
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    cfg["prob_generator"]["device"] = str(device)
    cfg["prior_generator"]["device"] = str(device)
    model = Flamed.from_pretrained(cfg=cfg, ckpt_path=ckpt_path, device=device, weights_only=weights_only,
                                   training_mode=False)
    model.to(device)
    return model


def _resolve_prompt_path(prompt_dir: str, prompt_name: str) -> str:
    return prompt_name if os.path.isabs(prompt_name) else os.path.join(prompt_dir, prompt_name)


def chunked(seq, size):
    for idx in range(0, len(seq), size):
        yield seq[idx: idx + size]


def encode_prompt_features(model: Flamed, codec_encoder, codec_decoder, prompt_path: str,
                           cache: Dict[str, Tuple[torch.Tensor, torch.Tensor]]):
    """Prompt wav -> (codes (6, P), timbre (256,)), cached per path (reference :124-141)."""
    if prompt_path in cache:
        return cache[prompt_path]
    with torch.inference_mode():
        acoustic_prompt = model._preprocess_acoustic_prompt(prompt_path, sr=SR)
        enc_out = codec_encoder(acoustic_prompt)
        _, prompts, _, _, timbre = codec_decoder(enc_out, eval_vq=False, vq=True)
    prompts = prompts.permute(1, 0, 2).contiguous().squeeze(0).detach().cpu()
    cache[prompt_path] = (prompts, timbre.squeeze(0).detach().cpu())
    return cache[prompt_path]


def pad_prompts(prompt_tensors: List[torch.Tensor], pad_value: int, device: torch.device):
    if not prompt_tensors:
        raise ValueError("pad_prompts received an empty list.")
    n_q = prompt_tensors[0].size(0)
    max_len = max(t.size(-1) for t in prompt_tensors)
    padded = torch.full((len(prompt_tensors), n_q, max_len), fill_value=pad_value,
                        dtype=prompt_tensors[0].dtype, device=device)
    for i, t in enumerate(prompt_tensors):
        padded[i, :, : t.size(-1)] = t.to(device)
    return padded, max_len


def build_metadata_batch(model: Flamed, codec_encoder, codec_decoder, batch_items: List[Dict[str, str]],
                         prompt_cache: Dict[str, Tuple[torch.Tensor, torch.Tensor]]):
    """(phonemes (B, L) zero-padded, src_lens, prompts (B, 6, P) padded with the codec vocab size,
    timbres (B, 256)) (reference :162-191)."""
    phonemes, src_lens, prompts, timbres = [], [], [], []
    for item in batch_items:
        seq = model._preprocess_english(item["text"])[0].squeeze(0)
        phonemes.append(seq)
        src_lens.append(seq.size(0))
        codes, timbre = encode_prompt_features(model, codec_encoder, codec_decoder, item["prompt_path"], prompt_cache)
        prompts.append(codes)
        timbres.append(timbre)
    pad_value = model.prior_generator.config["codec"]["vocab_size"]
    prompts_t, _ = pad_prompts(prompts, pad_value=pad_value, device=torch.device("cpu"))
    return (pad_sequence(phonemes, batch_first=True, padding_value=0), torch.tensor(src_lens, dtype=torch.long),
            prompts_t, torch.stack(timbres, dim=0))


class RtfMeter:
    """RTF = mean_i(time_i / duration_i) (reference :214-217, :300-303) plus latent frames/s."""

    def __init__(self):
        self.times, self.durations = [], []

    def add(self, seconds: float, n_samples: int):
        self.times.append(seconds)
        self.durations.append(n_samples / SR)

    def gathered(self) -> "RtfMeter":
        """A meter holding every rank's records (this one when not distributed)."""
        g = RtfMeter()
        for t, d in fdist.gather_records(list(zip(self.times, self.durations))):
            g.times.append(t)
            g.durations.append(d)
        return g

    def rtf(self):
        if not self.times:
            return None
        return sum(t / d for t, d in zip(self.times, self.durations)) / len(self.times)

    def frames_per_second(self):
        total = sum(self.times)
        return sum(d * SR / HOP for d in self.durations) / total if total > 0 else float("nan")


def synthesize_with_prompts(model: Flamed, codec_encoder, codec_decoder, text: str, prompt_dir: str,
                            prompt_list: List[str], output_dir: str, nsteps_durgen: int, nsteps_denoiser: int,
                            temp_durgen: float, temp_denoiser: float, meter: Optional[RtfMeter] = None):
    """One `Flamed.sample` per prompt (reference :194-217)."""
    os.makedirs(output_dir, exist_ok=True)
    meter = meter if meter is not None else RtfMeter()
    rank, world, _ = fdist.dist_env()
    for prompt_name in _progress(fdist.shard(prompt_list, rank, world), desc="Synthesizing prompts"):
        audio_prompt = load_audio(_resolve_prompt_path(prompt_dir, prompt_name))
        res = model.sample(text=text, prompt_raw=audio_prompt, sr=SR, codec_encoder=codec_encoder,
                           codec_decoder=codec_decoder, nsteps_durgen=nsteps_durgen, nsteps_denoiser=nsteps_denoiser,
                           temp_durgen=temp_durgen, temp_denoiser=temp_denoiser)
        meter.add(res["time"], len(res["wav"]))
        stem = os.path.splitext(os.path.basename(prompt_name))[0]
        out_name = f"{stem}-{nsteps_durgen}-{nsteps_denoiser}-{temp_durgen}-{temp_denoiser}.wav"
        write_wav(os.path.join(output_dir, out_name), res["wav"], SR)
    return meter.rtf()


def synthesize_with_metadata(model: Flamed, codec_encoder, codec_decoder, metadata_file: str, prompt_dir: str,
                             output_dir: str, nsteps_durgen: int, nsteps_denoiser: int, temp_durgen: float,
                             temp_denoiser: float, skip_existing: bool, batch_size: int,
                             meter: Optional[RtfMeter] = None):
    """Batched `Flamed.sample_batch` over a `target|prompt|text` file (reference :220-303)."""
    with open(metadata_file, "r", encoding="utf-8") as fin:
        entries = [line.strip() for line in fin if line.strip()]
    target_dir = os.path.join(output_dir, f"nfe{nsteps_denoiser}-temp{temp_denoiser}")
    os.makedirs(target_dir, exist_ok=True)
    meter = meter if meter is not None else RtfMeter()
    cache: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
    pending: List[Dict[str, str]] = []
    for entry in entries:
        try:
            filename, prompt_filename, transcript = entry.split("|", 2)
        except ValueError:
            print(f"[WARN] Malformed line skipped: {entry}")
            continue
        out_path = os.path.join(target_dir, filename)
        if skip_existing and os.path.exists(out_path):
            continue
        pending.append({"filename": filename, "prompt_path": _resolve_prompt_path(prompt_dir, prompt_filename),
                        "text": transcript, "out_path": out_path})
    rank, world, _ = fdist.dist_env()
    if world > 1:  # length buckets: phoneme count is the utterance-length (T x nfe work) proxy
        costs = [int(model._preprocess_english(it["text"])[0].size(-1)) for it in pending]
        pending = fdist.bucket_shard(pending, costs, rank, world)
    if not pending:
        return None
    for batch in _progress(chunked(pending, batch_size), total=math.ceil(len(pending) / batch_size),
                           desc="Synthesizing metadata entries"):
        phonemes, src_lens, prompts, timbres = build_metadata_batch(model, codec_encoder, codec_decoder, batch, cache)
        out = model.sample_batch(phonemes=phonemes, src_lens=src_lens, prompts=prompts, timbres=timbres,
                                 codec_decoder=codec_decoder, temp_durgen=temp_durgen, temp_denoiser=temp_denoiser,
                                 nsteps_durgen=nsteps_durgen, nsteps_denoiser=nsteps_denoiser)
        per_sample = out["time"] / len(batch)
        for item, wav_t in zip(batch, out["wav"]):
            wav = wav_t[0].detach().cpu().numpy()
            write_wav(item["out_path"], wav, SR)
            meter.add(per_sample, len(wav))
    return meter.rtf()


def _normalize_args(args: argparse.Namespace) -> argparse.Namespace:
    if getattr(args, "prompt_dir", None) is None and hasattr(args, "input_dir"):
        args.prompt_dir = args.input_dir
    return args


def _validate_args(args: argparse.Namespace):
    """Reference :312-325 (same messages)."""
    metadata_mode = args.metadata_file is not None
    prompt_mode = args.prompt_list is not None
    if metadata_mode == prompt_mode:
        raise ValueError("Specify either --prompt-list (direct mode) or --metadata-file (batch mode), but not both.")
    if args.prompt_dir is None:
        raise ValueError("--prompt-dir/--input-dir is required.")
    if prompt_mode and not args.text:
        raise ValueError("--text is required when using --prompt-list.")
    if metadata_mode:
        if not os.path.isfile(args.metadata_file):
            raise ValueError(f"Metadata file not found: {args.metadata_file}")
        if args.batch_size < 1:
            raise ValueError("--batch-size must be >= 1.")


def build_arg_parser():
    """Reference flags (:328-345) plus --codec-ckpt-dir."""
    p = argparse.ArgumentParser(description="Unified Flamed-TTS synthesis script.")
    p.add_argument("--ckpt-path", type=str, required=True, help="Path to Flamed checkpoint.")
    p.add_argument("--cfg-path", type=str, required=True, help="Path to model config yaml.")
    p.add_argument("--text", type=str, default=None, help="Text content (prompt-list mode).")
    p.add_argument("--prompt-list", nargs="+", default=None, help="Prompt filenames for direct synthesis.")
    p.add_argument("--prompt-dir", "--input-dir", dest="prompt_dir", type=str, default=None,
                   help="Directory containing prompt WAV files.")
    p.add_argument("--metadata-file", "--text-file", dest="metadata_file", type=str, default=None,
                   help="Metadata file with lines formatted as target|prompt|text.")
    p.add_argument("--output-dir", type=str, default=".", help="Directory to store outputs.")
    p.add_argument("--weights-only", type=str2bool, default=True, help="Load checkpoint weights_only flag (default: True).")
    p.add_argument("--nsteps-durgen", type=int, default=64, help="Duration generator sampling steps.")
    p.add_argument("--nsteps-denoiser", type=int, default=64, help="Denoiser sampling steps.")
    p.add_argument("--temp-durgen", type=float, default=0.3, help="Duration generator temperature.")
    p.add_argument("--temp-denoiser", type=float, default=0.3, help="Denoiser temperature.")
    p.add_argument("--device", type=str, default="cuda:0", help="Device to run inference on.")
    p.add_argument("--skip-existing", type=str2bool, default=True,
                   help="Skip samples whose output files already exist (metadata mode).")
    p.add_argument("--batch-size", type=int, default=4, help="Number of metadata samples to synthesize per batch.")
    p.add_argument("--codec-ckpt-dir", type=str, default=None,
                   help="Directory with ns3_facodec_{encoder,decoder}.bin (default: flamed/models/facodec/checkpoints).")
    p.add_argument("--seed", type=int, default=None,
                   help="Seed the global RNGs (rank r of a torchrun job uses seed + r); default: unseeded, as the reference.")
    return p


def main(args: Optional[argparse.Namespace] = None):
    parser = build_arg_parser()
    cli_invocation = args is None
    if cli_invocation:
        args = parser.parse_args()
    args = _normalize_args(args)
    try:
        _validate_args(args)
    except ValueError as exc:
        if cli_invocation:
            parser.error(str(exc))
        raise
    device = resolve_device(args.device)
    distributed = fdist.init(device.type)
    if getattr(args, "seed", None) is not None:
        torch.manual_seed(fdist.rank_seed(args.seed))
    codec_encoder, codec_decoder = get_codec(device, getattr(args, "codec_ckpt_dir", None))
    model = prepare_model(args.cfg_path, args.ckpt_path, device, args.weights_only)
    meter = RtfMeter()
    common = dict(model=model, codec_encoder=codec_encoder, codec_decoder=codec_decoder, prompt_dir=args.prompt_dir,
                  output_dir=args.output_dir, nsteps_durgen=args.nsteps_durgen, nsteps_denoiser=args.nsteps_denoiser,
                  temp_durgen=args.temp_durgen, temp_denoiser=args.temp_denoiser, meter=meter)
    if args.metadata_file:
        rtf = synthesize_with_metadata(metadata_file=args.metadata_file, skip_existing=args.skip_existing,
                                       batch_size=args.batch_size, **common)
    else:
        rtf = synthesize_with_prompts(text=args.text, prompt_list=args.prompt_list, **common)
    if distributed:  # every rank's records; each rank's frames/s summed over the ranks' wall time
        local_fps = meter.frames_per_second() if meter.times else 0.0
        meter = meter.gathered()
        rtf = meter.rtf()
        total_fps = sum(fdist.gather_records([local_fps]))
    else:
        total_fps = meter.frames_per_second() if meter.times else 0.0
    if fdist.dist_env()[0] == 0:
        if rtf is not None:
            print("=" * 20, "Avg RTF", "=" * 20)
            print(">" * 5, "RTF:", round(rtf, 3))
            print(">" * 5, "latent frames/s:", round(total_fps, 1))
        else:
            print("No samples were generated.")
    return rtf


if __name__ == "__main__":
    main()
