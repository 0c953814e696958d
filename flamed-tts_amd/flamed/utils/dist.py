"""One process per GPU, utterances sharded across ranks.

Synthesis has no cross-utterance dependency, so the data path needs no collective: each rank takes a
round-robin shard of the work items, runs it on its own device, and only the per-utterance timing
records (for the RTF summary) are gathered once at the end.  Launch with torchrun
(`--master-addr 127.0.0.1`); RANK / WORLD_SIZE / LOCAL_RANK come from the environment.  The process
group uses RCCL ("nccl") on ROCm devices and gloo on CPU.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple, TypeVar

import torch

T = TypeVar("T")


def dist_env() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard(items: Sequence[T], rank: int, world: int) -> List[T]:
    """Round-robin shard: item i goes to rank i % world (balanced to within one item)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world: {rank}/{world}")
    return list(items[rank::world])


def init(device_type: str) -> bool:
    """Initialise the default process group when WORLD_SIZE > 1; returns True if distributed."""
    import torch.distributed as td
    _, world, local = dist_env()
    if world <= 1:
        return False
    if not td.is_initialized():
        backend = "nccl" if device_type == "cuda" else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        td.init_process_group(backend)
    return True


def gather_records(records: list) -> list:
    """All ranks' (time, n_samples) records, concatenated in rank order (identity when not distributed)."""
    import torch.distributed as td
    if not (td.is_available() and td.is_initialized()) or td.get_world_size() == 1:
        return list(records)
    out = [None] * td.get_world_size()
    td.all_gather_object(out, list(records))
    return [r for part in out for r in part]
