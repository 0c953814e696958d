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
    extra = {}
    if mode == "metadata":
        # the bucket this rank was given (same rule synthesize_with_metadata applied) and a per-shard
        # parity check: this rank's ProbGenerator.sample on a batch shaped by its shard, seeded
        # seed + rank, against the oracle with the same seed
        entries = [ln.strip().split("|", 2) for ln in open(os.path.join(work, "meta.txt")) if ln.strip()]
        costs = [int(m._preprocess_english(t)[0].size(-1)) for _, _, t in entries]
        mine = fdist.bucket_shard(list(range(len(entries))), costs, rank, world)
        from oracle import flamed_oracle as orc
        B, T = len(mine), 3 * max(costs[i] for i in mine)
        g = torch.Generator().manual_seed(fdist.rank_seed(100))
        cond = torch.randn(B, 6, T, 384, generator=g)
        spk = torch.randn(B, 256, generator=g)
        mask = torch.ones(B, T, 1, dtype=torch.bool)
        pg = m.prob_generator
        sd = {"prob_generator." + k: v.detach() for k, v in pg.state_dict().items()}
        with torch.inference_mode():
            torch.manual_seed(fdist.rank_seed(7))
            lat = pg.sample(cond, spk, mask, nfe=3, temperature=0.3)
            torch.manual_seed(fdist.rank_seed(7))
            ref = orc.prob_sample(sd, cond, spk, mask, nfe=3, temperature=0.3)
        err = float((lat - ref).norm() / ref.norm())
        extra = {"shard": mine, "cost": sum(costs[i] for i in mine), "costs": costs, "shard_rel_l2": err}
    g = meter.gathered()
    if rank == 0:
        with open(os.path.join(work, f"result_{mode}.json"), "w") as f:
            json.dump({"world": world, "n_total": len(g.times), "rtf": g.rtf()}, f)
    with open(os.path.join(work, f"rank{rank}_{mode}.json"), "w") as f:
        json.dump({"local": local, **extra}, f)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
