"""Static sharding of a signature batch across GPUs + RCCL all-gather of verdict bitmaps
(north_star: "Batches shard statically across the 8xMI355X node, and the only cross-GPU traffic
is an RCCL all-gather of per-signature verdict bitmaps over xGMI").

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Rank r verifies the
contiguous range [lo_r, hi_r) whose start is a multiple of 64, so every rank's 64-bit ballot
words drop into the global bitmap without re-packing; the all-gather moves ceil(shard/64) words
per rank (16 KiB per GPU for a 1M batch on 8 GPUs): latency-bound, one collective per batch.
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_size(n: int, world: int) -> int:
    """Per-rank shard length: ceil(n / world) rounded up to a multiple of 64."""
    per = -(-n // world)
    return -(-per // 64) * 64


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    s = shard_size(n, world)
    lo = min(n, rank * s)
    return lo, min(n, lo + s)


def gather_verdicts(local_words, n: int, world: int, dist):
    """All-gather each rank's verdict words (int64 tensor of shard_size/64 words, zero-padded)
    and return the global ceil(n/64)-word bitmap on every rank."""
    import torch

    words = shard_size(n, world) // 64
    assert local_words.numel() == words, (local_words.numel(), words)
    out = torch.empty(world * words, dtype=local_words.dtype, device=local_words.device)
    dist.all_gather_into_tensor(out, local_words)
    return out[: (n + 63) // 64]


def verify_sharded(n: int, world: int, rank: int, verify_range: Callable, dist, device):
    """verify_range(lo, hi, out_words) fills out_words (int64 tensor) with the ballot words of
    signatures [lo, hi); returns the global bitmap words on every rank."""
    import torch

    lo, hi = shard_bounds(n, world, rank)
    words = torch.zeros(shard_size(n, world) // 64, dtype=torch.int64, device=device)
    if hi > lo:
        verify_range(lo, hi, words)
    return gather_verdicts(words, n, world, dist)
