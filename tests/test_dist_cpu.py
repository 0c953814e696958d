"""Multi-GPU path rehearsed on CPU: utterances round-robin sharded over ranks, no
data-path collective, timing records gathered once; world_size 2 over gloo via torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from _common import PKG

sys.path.insert(0, PKG)
from flamed.utils.audio import write_wav  # noqa: E402
from flamed.utils.dist import shard  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_partition():
    items = list(range(11))
    parts = [shard(items, r, 4) for r in range(4)]
    assert sorted(x for p in parts for x in p) == items
    assert max(map(len, parts)) - min(map(len, parts)) <= 1
    assert shard(items, 0, 1) == items
    with pytest.raises(ValueError):
        shard(items, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["metadata", "prompts"])
def test_two_rank_sharded_synthesis(tmp_path, mode):
    rng = np.random.default_rng(0)
    os.makedirs(tmp_path / "pr")
    for i in range(3):
        write_wav(str(tmp_path / "pr" / f"p{i}.wav"), rng.normal(0, 0.1, 4000).astype(np.float32))
    lines = [f"u{i}.wav|p{i % 3}.wav|utterance number {i}." for i in range(5)]
    (tmp_path / "meta.txt").write_text("\n".join(lines) + "\n")
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "_dist_worker.py"),
           str(tmp_path), mode]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads((tmp_path / f"result_{mode}.json").read_text())
    locs = [json.loads((tmp_path / f"rank{k}_{mode}.json").read_text())["local"] for k in range(2)]
    n = 5 if mode == "metadata" else 3
    assert res["world"] == 2 and res["n_total"] == n and sum(locs) == n and min(locs) >= 1
    out = tmp_path / "out" / ("nfe2-temp0.3" if mode == "metadata" else "")
    files = sorted(os.listdir(out))
    if mode == "metadata":
        assert files == [f"u{i}.wav" for i in range(5)]
    else:
        assert files == [f"p{i}-2-2-0.3-0.3.wav" for i in range(3)]
    assert res["rtf"] > 0
