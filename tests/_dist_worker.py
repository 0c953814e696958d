"""torchrun worker for tests/test_dist_cpu.py: one rank of a sharded synthesize run on CPU (gloo).
argv: WORKDIR MODE(metadata|prompts)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "flamed-tts_amd"))

import torch  # noqa: E402

from _flamed_common import build_flamed, build_codec_encoder  # noqa: E402
import synthesize as syn  # noqa: E402
from flamed.utils import dist as fdist  # noqa: E402


def main():
    work, mode = sys.argv[1], sys.argv[2]
    torch.set_num_threads(2)
    assert fdist.init("cpu")
    rank, world, _ = fdist.dist_env()
    m, dec = build_flamed("cpu")
    enc = build_codec_encoder("cpu")
    meter = syn.RtfMeter()
    if mode == "metadata":
        syn.synthesize_with_metadata(m, enc, dec, os.path.join(work, "meta.txt"), os.path.join(work, "pr"),
                                     os.path.join(work, "out"), 2, 2, 0.3, 0.3, skip_existing=False, batch_size=2,
                                     meter=meter)
    else:
        syn.synthesize_with_prompts(m, enc, dec, "hello there.", os.path.join(work, "pr"),
                                    ["p0.wav", "p1.wav", "p2.wav"], os.path.join(work, "out"), 2, 2, 0.3, 0.3,
                                    meter=meter)
    local = len(meter.times)
    g = meter.gathered()
    if rank == 0:
        with open(os.path.join(work, f"result_{mode}.json"), "w") as f:
            json.dump({"world": world, "n_total": len(g.times), "rtf": g.rtf()}, f)
    with open(os.path.join(work, f"rank{rank}_{mode}.json"), "w") as f:
        json.dump({"local": local}, f)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
