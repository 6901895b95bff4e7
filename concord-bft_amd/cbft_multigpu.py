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


# ---------------------------------------------------------------------------------------------
# BLS BN-P254 across GPUs.  `backend` is a cbft_hipcrypto.Context on
# the rank's GPU (or, in the CPU tests, a stand-in with the same methods); partial points are
# opaque fixed-size byte strings (CBFT_BLS_G1/G2_PARTIAL_BYTES) exchanged with one all-gather.
# ---------------------------------------------------------------------------------------------
def share_slice(k: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank's contiguous share range; a multiple of 8 shares so the validity bitmaps' bytes
    concatenate without re-packing."""
    per = -(-k // world)
    per = -(-per // 8) * 8
    lo = min(k, rank * per)
    return lo, min(k, lo + per)


def id_slice(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank's signer-id range [lo_id, hi_id) of ids 1..n for a sharded multisig key sum."""
    per = -(-n // world)
    lo = min(n + 1, 1 + rank * per)
    return lo, min(n + 1, lo + per)


def _gather_bytes(blob: bytes, world: int, dist, device) -> list:
    import numpy as np
    import torch

    t = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).to(device)
    out = torch.empty(world * len(blob), dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, t)
    raw = out.cpu().numpy().tobytes()
    return [raw[r * len(blob):(r + 1) * len(blob)] for r in range(world)]


def bls_verify_shares_sharded(backend, kid: int, msg: bytes, shares, world: int, rank: int, dist, device):
    """Every rank verifies its slice of the shares (pairing checks are independent); one
    all-gather of the k-bit validity bitmap.  Returns the k validity flags on every rank."""
    import numpy as np

    k = len(shares)
    lo, hi = share_slice(k, world, rank)
    per = share_slice(k, world, 0)[1]
    bits = np.zeros(per, dtype=bool)
    if hi > lo:
        bits[: hi - lo] = backend.bls_verify_shares(kid, msg, shares[lo:hi])
    blob = np.packbits(bits, bitorder="little").tobytes()
    parts = _gather_bytes(blob, world, dist, device)
    allbits = np.unpackbits(np.frombuffer(b"".join(parts), dtype=np.uint8), bitorder="little").astype(bool)
    return allbits[:k]


def bls_combine_sharded(backend, shares, world: int, rank: int, dist, device, multisig: bool = False) -> bytes:
    """Lagrange-weighted MSM split by share slice: each rank sums lambda_j sigma_j over its slice
    (lambda over the full signer set), one all-gather of the partial points, then the sum and
    compression.  Every rank returns the same 33-byte combined signature."""
    lo, hi = share_slice(len(shares), world, rank)
    part = backend.bls_combine_partial(shares, lo, hi, multisig)
    return backend.bls_combine_finish(_gather_bytes(part, world, dist, device))


def bls_verify_multisig_sharded(backend, kid: int, n: int, msg: bytes, sig33: bytes, signers256: bytes,
                                world: int, rank: int, dist, device) -> bool:
    """Multisig public key sum_{id in bitmap} vk_id split by id range, one all-gather of the G2
    partial sums, then the pairing check on every rank."""
    lo_id, hi_id = id_slice(n, world, rank)
    part = backend.bls_sum_keys_partial(kid, signers256, lo_id, hi_id)
    return backend.bls_verify_multisig_partials(msg, sig33, _gather_bytes(part, world, dist, device))
