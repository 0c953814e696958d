#!/bin/bash
# GPU run of the synthesize.py CLI (BASELINE metric: RTF + latent frames/s at nsteps-denoiser=128),
# both modes, random-init checkpoint.  Usage: tools/gpu_cli.sh TAG
set -euo pipefail
TAG=${1:-cli}
OUT=gpurun_out/$TAG
mkdir -p $OUT/prompts
cd flamed-tts_amd
timeout -k 10 300 python -m flamed.utils.random_ckpt --out-dir /tmp/frand > ../$OUT/ckpt.log 2>&1
cd ..
python - "$TAG" <<'PY'
import numpy as np, sys
sys.path.insert(0, "flamed-tts_amd")
from flamed.utils.audio import write_wav
rng = np.random.default_rng(0)
t = np.arange(48000) / 16000.0
for i in range(4):
    x = 0.3 * np.sin(2 * np.pi * (180 + 40 * i) * t) + 0.05 * rng.standard_normal(t.size)
    write_wav(f"gpurun_out/{sys.argv[1] if len(sys.argv) > 1 else 'cli'}/prompts/p{i}.wav", x.astype(np.float32))
PY
TEXT="the quick brown fox jumps over the lazy dog, and then it runs far away into the forest."
{
  for i in 0 1 2 3; do echo "u$i.wav|p$i.wav|$TEXT"; done
} > $OUT/meta.txt
COMMON="--ckpt-path /tmp/frand/flamed.pt --cfg-path /tmp/frand/config.yaml --codec-ckpt-dir /tmp/frand --prompt-dir $OUT/prompts --nsteps-denoiser 128 --nsteps-durgen 64 --device cuda:0"
timeout -k 10 300 python flamed-tts_amd/synthesize.py $COMMON --text "$TEXT" --prompt-list p0.wav p1.wav p0.wav p1.wav --output-dir $OUT/wav_prompt > $OUT/prompt_mode.log 2>&1
timeout -k 10 300 python flamed-tts_amd/synthesize.py $COMMON --metadata-file $OUT/meta.txt --batch-size 4 --output-dir $OUT/wav_meta > $OUT/meta_mode.log 2>&1
rm -rf $OUT/wav_prompt $OUT/wav_meta $OUT/prompts
grep -h "RTF\|frames" $OUT/prompt_mode.log $OUT/meta_mode.log
