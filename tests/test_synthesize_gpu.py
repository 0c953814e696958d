"""synthesize.py CLI on the GPU: BASELINE config 0's command line with
`--device cuda:0` in both modes — prompt mode (raw prompt wav -> FaCodec encode -> prior/PVA ->
denoiser -> decode, RTF by synthesize.py:209-217) and metadata mode (batched, per-sample time =
batch time / len(batch), decode excluded, :293-303) — through the HIP library.  Random-init weights,
so the check is the contract: exit, files, lengths in whole latent frames, finite audio, RTF > 0."""
import os
import sys

import numpy as np
import pytest
import torch

from _common import PKG

sys.path.insert(0, PKG)
import synthesize as syn  # noqa: E402
from flamed.utils.audio import load_wav, write_wav  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from flamed.utils.random_ckpt import write
    d = tmp_path_factory.mktemp("ck")
    paths = write(str(d))
    pr = d / "pr"
    os.makedirs(pr)
    rng = np.random.default_rng(0)
    for i in range(2):
        write_wav(str(pr / f"p{i}.wav"), rng.normal(0, 0.1, 16000 + 4000 * i).astype(np.float32), 16000)
    return paths, d, pr


def _check_wavs(d, names):
    assert sorted(os.listdir(d)) == sorted(names)
    for n in names:
        w = load_wav(os.path.join(d, n), 16000)
        assert len(w) > 0 and len(w) % 200 == 0 and np.all(np.isfinite(w))


def test_cli_prompt_mode_gpu(ckpt, tmp_path, capsys):
    paths, d, pr = ckpt
    args = syn.build_arg_parser().parse_args([
        "--ckpt-path", paths["ckpt"], "--cfg-path", paths["cfg"], "--codec-ckpt-dir", str(d),
        "--text", "hello world, this is a test.", "--prompt-list", "p0.wav", "p1.wav", "--prompt-dir", str(pr),
        "--output-dir", str(tmp_path / "out"), "--device", "cuda:0", "--nsteps-durgen", "16",
        "--nsteps-denoiser", "32"])
    rtf = syn.main(args)
    assert rtf is not None and 0 < rtf < 1.0
    _check_wavs(tmp_path / "out", ["p0-16-32-0.3-0.3.wav", "p1-16-32-0.3-0.3.wav"])
    assert "RTF" in capsys.readouterr().out


def test_cli_metadata_mode_gpu(ckpt, tmp_path):
    paths, d, pr = ckpt
    meta = tmp_path / "meta.txt"
    meta.write_text("u0.wav|p0.wav|hello world.\nu1.wav|p1.wav|good morning to you all.\nu2.wav|p0.wav|a third one.\n")
    args = syn.build_arg_parser().parse_args([
        "--ckpt-path", paths["ckpt"], "--cfg-path", paths["cfg"], "--codec-ckpt-dir", str(d),
        "--text-file", str(meta), "--input-dir", str(pr), "--output-dir", str(tmp_path / "out"),
        "--device", "cuda:0", "--nsteps-durgen", "16", "--nsteps-denoiser", "32", "--batch-size", "2"])
    rtf = syn.main(args)
    assert rtf is not None and 0 < rtf < 1.0
    _check_wavs(tmp_path / "out" / "nfe32-temp0.3", ["u0.wav", "u1.wav", "u2.wav"])
    from flamed import _native as nat
    assert nat._lib is not None  # the HIP library served the run
