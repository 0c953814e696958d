"""synthesize.py: flags and validation errors, both modes end to end on CPU,
and the two RTF definitions (reference synthesize.py:209-217 prompt mode, :293-303 metadata mode)."""
import argparse
import os
import sys

import numpy as np
import pytest
import torch

from _common import PKG
from _flamed_common import build_flamed, build_codec_encoder

sys.path.insert(0, PKG)
import synthesize as syn  # noqa: E402
from flamed.utils.audio import load_wav, write_wav  # noqa: E402


def _ns(**kw):
    base = dict(ckpt_path="x", cfg_path="y", text=None, prompt_list=None, prompt_dir=None, metadata_file=None,
                output_dir=".", weights_only=True, nsteps_durgen=4, nsteps_denoiser=4, temp_durgen=0.3,
                temp_denoiser=0.3, device="cpu", skip_existing=True, batch_size=4, codec_ckpt_dir=None)
    base.update(kw)
    return argparse.Namespace(**base)


def test_flags_and_validation(tmp_path):
    p = syn.build_arg_parser()
    a = p.parse_args(["--ckpt-path", "c", "--cfg-path", "g", "--input-dir", "d", "--text-file", "m",
                      "--weights-only", "no", "--skip-existing", "0"])
    assert a.prompt_dir == "d" and a.metadata_file == "m" and a.weights_only is False and a.skip_existing is False
    assert (a.nsteps_durgen, a.nsteps_denoiser, a.temp_durgen, a.temp_denoiser, a.batch_size, a.device) == \
        (64, 64, 0.3, 0.3, 4, "cuda:0")
    with pytest.raises(ValueError, match="not both"):
        syn.main(_ns(prompt_dir="d"))
    with pytest.raises(ValueError, match="prompt-dir"):
        syn.main(_ns(prompt_list=["a.wav"], text="hi"))
    with pytest.raises(ValueError, match="--text is required"):
        syn.main(_ns(prompt_list=["a.wav"], prompt_dir="d"))
    with pytest.raises(ValueError, match="Metadata file not found"):
        syn.main(_ns(metadata_file=str(tmp_path / "none.txt"), prompt_dir="d"))
    meta = tmp_path / "m.txt"
    meta.write_text("a|b|c\n")
    with pytest.raises(ValueError, match="batch-size"):
        syn.main(_ns(metadata_file=str(meta), prompt_dir="d", batch_size=0))
    with pytest.raises(argparse.ArgumentTypeError):
        syn.str2bool("maybe")


def test_wav_io_roundtrip(tmp_path):
    x = (0.5 * np.sin(np.arange(800) / 7.0)).astype(np.float32)
    write_wav(str(tmp_path / "a.wav"), x, 16000)
    y = load_wav(str(tmp_path / "a.wav"), 16000)
    assert np.max(np.abs(y - x)) < 1e-4
    z = load_wav(str(tmp_path / "a.wav"), 8000)
    assert abs(len(z) - 400) <= 1


@pytest.fixture(scope="module")
def stack():
    torch.set_num_threads(8)
    m, dec = build_flamed("cpu")
    return m, build_codec_encoder("cpu"), dec


def _prompts(d, n=2):
    rng = np.random.default_rng(0)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        write_wav(os.path.join(d, f"p{i}.wav"), rng.normal(0, 0.1, 4000 + 2000 * i).astype(np.float32))


def test_prompt_mode_rtf(stack, tmp_path):
    m, enc, dec = stack
    _prompts(tmp_path / "pr")
    meter = syn.RtfMeter()
    rtf = syn.synthesize_with_prompts(m, enc, dec, "hello world.", str(tmp_path / "pr"), ["p0.wav", "p1.wav"],
                                      str(tmp_path / "out"), 4, 4, 0.3, 0.3, meter=meter)
    files = sorted(os.listdir(tmp_path / "out"))
    assert files == ["p0-4-4-0.3-0.3.wav", "p1-4-4-0.3-0.3.wav"]
    assert len(meter.times) == 2
    expect = np.mean([t / d for t, d in zip(meter.times, meter.durations)])
    assert rtf == pytest.approx(expect)
    assert all(d * 16000 % 200 == 0 for d in meter.durations)  # whole latent frames


def test_metadata_mode_batches(stack, tmp_path):
    m, enc, dec = stack
    _prompts(tmp_path / "pr")
    meta = tmp_path / "meta.txt"
    meta.write_text("u0.wav|p0.wav|hello world.\nbad line\nu1.wav|p1.wav|good morning to you.\n"
                    "u2.wav|p0.wav|a third one.\n")
    calls = []
    orig = m.sample_batch

    def spy(**kw):
        out = orig(**kw)
        calls.append((kw["phonemes"].shape[0], out["time"]))
        return out

    m.sample_batch = spy
    try:
        meter = syn.RtfMeter()
        rtf = syn.synthesize_with_metadata(m, enc, dec, str(meta), str(tmp_path / "pr"), str(tmp_path / "out"),
                                           4, 4, 0.3, 0.3, skip_existing=True, batch_size=2, meter=meter)
    finally:
        del m.sample_batch
    tgt = tmp_path / "out" / "nfe4-temp0.3"
    assert sorted(os.listdir(tgt)) == ["u0.wav", "u1.wav", "u2.wav"]
    assert [c[0] for c in calls] == [2, 1]
    per = [calls[0][1] / 2] * 2 + [calls[1][1]]
    assert meter.times == pytest.approx(per)             # batch time / len(batch), decode excluded
    assert rtf == pytest.approx(np.mean([t / d for t, d in zip(per, meter.durations)]))
    # skip_existing: a second run has nothing to do
    assert syn.synthesize_with_metadata(m, enc, dec, str(meta), str(tmp_path / "pr"), str(tmp_path / "out"),
                                        4, 4, 0.3, 0.3, skip_existing=True, batch_size=2) is None


def test_cli_config0_random_ckpt(tmp_path):
    """BASELINE config 0: the CLI on CPU with a random-init checkpoint; exits 0, writes a wav, prints RTF."""
    from flamed.utils.random_ckpt import write
    paths = write(str(tmp_path / "ck"))
    _prompts(tmp_path / "pr", 1)
    args = syn.build_arg_parser().parse_args([
        "--ckpt-path", paths["ckpt"], "--cfg-path", paths["cfg"], "--codec-ckpt-dir", str(tmp_path / "ck"),
        "--text", "hello world.", "--prompt-list", "p0.wav", "--prompt-dir", str(tmp_path / "pr"),
        "--output-dir", str(tmp_path / "out"), "--device", "cpu", "--nsteps-durgen", "4", "--nsteps-denoiser", "4"])
    rtf = syn.main(args)
    assert rtf is not None and rtf > 0
    assert os.listdir(tmp_path / "out") == ["p0-4-4-0.3-0.3.wav"]
