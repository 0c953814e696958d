"""One process per GPU, utterances sharded across ranks.

Synthesis has no cross-utterance dependency, so the data path needs no collective: each rank takes a
shard of the work items, runs it on its own device, and only the per-utterance timing records (for the
RTF summary) are gathered once at the end.  Metadata (batch) mode shards by length (bucket_shard):
utterances sorted by their expected length and cut into contiguous buckets of near-equal total work
(Euler cost is T x nfe per utterance), so every rank finishes at about the same time and batches
inside a rank pad little.  Launch with torchrun
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


def bucket_bounds(costs: Sequence[float], world: int) -> List[Tuple[int, int]]:
    """Cut a cost sequence (already sorted) into `world` contiguous [start, end) buckets whose sums are
    as close as possible to total / world: cut k sits at the prefix closest to k * total / world
    (leaving at least one item for every later bucket while items remain)."""
    n = len(costs)
    if world < 1:
        raise ValueError(f"bad world: {world}")
    prefix = [0.0]
    for c in costs:
        prefix.append(prefix[-1] + float(c))
    total = prefix[-1]
    cuts = [0]
    for k in range(1, world):
        lo = cuts[-1] + (1 if cuts[-1] < n else 0)
        hi = max(lo, n - (world - k)) if n >= world else n
        lo = min(lo, hi)
        target = total * k / world
        best = min(range(lo, hi + 1), key=lambda j: (abs(prefix[j] - target), j))
        cuts.append(best)
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def bucket_shard(items: Sequence[T], costs: Sequence[float], rank: int, world: int) -> List[T]:
    """Length-bucketed shard: sort by cost (stable, so ties keep input order), cut into
    `world` contiguous buckets balanced by total cost (bucket_bounds); rank r takes bucket r."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world: {rank}/{world}")
    if len(items) != len(costs):
        raise ValueError("bucket_shard: items and costs differ in length")
    order = sorted(range(len(items)), key=lambda i: costs[i])
    a, b = bucket_bounds([costs[i] for i in order], world)[rank]
    return [items[i] for i in order[a:b]]


def rank_seed(seed: int) -> int:
    """Per-rank RNG seed (seed + rank): ranks draw independent noise, and a shard's outputs are
    reproducible from (seed, rank) alone."""
    return int(seed) + dist_env()[0]


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
