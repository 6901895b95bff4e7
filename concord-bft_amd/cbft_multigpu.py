"""Static sharding of a signature batch across GPUs + RCCL all-gather of verdict bitmaps
(north_star: "Batches shard statically across the 8xMI355X node, and the only cross-GPU traffic
is an RCCL all-gather of per-signature verdict bitmaps over xGMI").

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Rank r verifies the
contiguous range [lo_r, hi_r) whose start is a multiple of 64, so every rank's 64-bit ballot
words drop into the global bitmap without re-packing; the all-gather moves ceil(shard/64) words
per rank (16 KiB per GPU for a 1M batch on 8 GPUs): latency-bound, one collective per batch.
"""
from __future__ import annotations

import time
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def shard_size(n: int, world: int) -> int:
    """Per-rank shard length: ceil(n / world) rounded up to a multiple of 64."""
    per = -(-n // world)
    return -(-per // 64) * 64


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    s = shard_size(n, world)
    lo = min(n, rank * s)
    return lo, min(n, lo + s)


def _host_staged(dist, t) -> bool:
    """gloo has no all-gather of device tensors: a rehearsal of the rank path on a gloo process
    group (bench.py with CBFT_BENCH_SHARED_GPU=1: several ranks sharing one GPU) stages device
    tensors through the host.  RCCL runs take the device path untouched."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _all_gather_into(out, t, dist):
    if _host_staged(dist, t):
        o = out.cpu()
        dist.all_gather_into_tensor(o, t.cpu())
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, t)


def _all_reduce(t, op, dist):
    if _host_staged(dist, t):
        c = t.cpu()
        dist.all_reduce(c, op=op)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=op)


def gather_verdicts(local_words, n: int, world: int, dist):
    """All-gather each rank's verdict words (int64 tensor of shard_size/64 words, zero-padded)
    and return the global ceil(n/64)-word bitmap on every rank."""
    import torch

    words = shard_size(n, world) // 64
    assert local_words.numel() == words, (local_words.numel(), words)
    out = torch.empty(world * words, dtype=local_words.dtype, device=local_words.device)
    _all_gather_into(out, local_words, dist)
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
# The rank path of bench.py (one process per GPU): the contract's timed region, each step's
# verdict words and their all-gather, the post-region check of every step against the OpenSSL
# verdicts of the batch that step verified, and the config #5 flood plan.  bench.py calls these
# and nothing else on its N > 1 branch; tests/test_multigpu_cpu.py drives the same functions with
# gloo on CPU tensors (stream = None), so the code the 8-GPU run executes is the code CI runs.
# ---------------------------------------------------------------------------------------------
def bools_to_words(v: np.ndarray) -> np.ndarray:
    """Verdict bools -> little-endian 64-bit ballot words (bit i of word i // 64 = signature i),
    the layout cbft_ed25519_verify_*_device writes; padding bits are 0."""
    nw = (len(v) + 63) // 64
    b = np.zeros(nw * 64, dtype=np.uint8)
    b[: len(v)] = np.asarray(v, dtype=bool)
    return np.packbits(b, bitorder="little").view(np.int64)


def max_over_ranks(x: float, dist, device) -> float:
    import torch

    t = torch.tensor([x], dtype=torch.float64, device=device)
    _all_reduce(t, dist.ReduceOp.MAX, dist)
    return float(t.item())


def sum_over_ranks(x: int, dist, device) -> int:
    import torch

    t = torch.tensor([x], dtype=torch.int64, device=device)
    _all_reduce(t, dist.ReduceOp.SUM, dist)
    return int(t.item())


def timed_region(fn: Callable[[int], None], steps: int, dist=None, sync: Optional[Callable] = None,
                 device=None) -> float:
    """The bench contract's timing: barrier + device synchronize on both sides of `steps` steps,
    then the MAX of the wall time over ranks (every rank returns it)."""
    if dist is not None:
        dist.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    fn(steps)
    if sync:
        sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    return max_over_ranks(el, dist, device) if dist is not None else el


def all_gather_rows(t, world: int, dist):
    """All-gather a tensor of any shape from every rank: returns (world, *t.shape)."""
    import torch

    out = torch.empty((world * t.numel(),), dtype=t.dtype, device=t.device)
    _all_gather_into(out, t.contiguous().view(-1), dist)
    return out.view(world, *t.shape)


class StepVerdicts:
    """One rank's verdict words for `steps` steps (row j = step j, its own buffer, so every step's
    verdicts survive the timed region and are checked after it) and, when world > 1, their
    all-gathers: after step j's launch on `launch_stream`, the gather stream waits for it and
    all-gathers row j into gathered[j] (world x nwords words, rank r's at [r]).  `stream`: the
    torch.cuda.Stream the all-gathers run on (None: the current stream / a CPU process group)."""

    def __init__(self, nwords: int, steps: int, world: int, rank: int, dist, device, stream=None):
        import torch

        self.nwords, self.steps, self.world, self.rank = nwords, steps, world, rank
        self.dist, self.device, self.stream = dist, device, stream
        self.local = torch.zeros((steps, nwords), dtype=torch.int64, device=device)
        self.gathered = torch.zeros((steps, world, nwords), dtype=torch.int64, device=device) \
            if world > 1 else None

    def words_ptr(self, j: int) -> int:
        return self.local[j].data_ptr()

    def _gather(self, j: int):
        _all_gather_into(self.gathered[j].view(-1), self.local[j], self.dist)

    def after_step(self, j: int, launch_stream=None):
        """Row j was written by work queued on launch_stream: all-gather it (N > 1)."""
        if self.world == 1:
            return
        if self.stream is None:
            self._gather(j)
            return
        import torch

        if launch_stream is not None:
            self.stream.wait_stream(launch_stream)
        with torch.cuda.stream(self.stream):
            self._gather(j)

    def after_host_step(self, j: int, bitmap: np.ndarray):
        """The host-buffer path: step j's bitmap is on the host (cbft_wait returned); move it into
        row j (on the gather stream) and all-gather it (N > 1), or just keep it (N = 1)."""
        import torch

        words = torch.from_numpy(np.ascontiguousarray(bitmap[: self.nwords * 8]).view(np.int64))
        if self.stream is None:
            self.local[j].copy_(words)
        else:
            with torch.cuda.stream(self.stream):
                self.local[j].copy_(words, non_blocking=False)
        if self.world > 1:
            self.after_step(j)

    def mismatches(self, expected_rows, batch_of_step: Callable[[int], int], steps: Optional[int] = None,
                   all_expected=None) -> int:
        """Words that differ from the expectation, over steps 0..steps-1: row j against
        expected_rows[batch_of_step(j)] (this rank's OpenSSL verdict words, (nb, nwords) int64 on
        this device) and, N > 1, every rank's section of gathered[j] against all_expected
        ([world, nb, nwords], all_gather_rows of every rank's expected_rows).  Call after the
        device work is synchronised."""
        import torch

        steps = self.steps if steps is None else steps
        idx = torch.tensor([batch_of_step(j) for j in range(steps)], dtype=torch.int64, device=self.device)
        bad = int((self.local[:steps] != expected_rows.index_select(0, idx)).sum().item())
        if self.world > 1:
            if all_expected is None:
                all_expected = all_gather_rows(expected_rows, self.world, self.dist)
            want = all_expected.index_select(1, idx).transpose(0, 1)  # (steps, world, nwords)
            bad += int((self.gathered[:steps] != want).sum().item())
        return bad


def flood_plan(total: int, world: int, rank: int, batch: int) -> List[Tuple[int, int]]:
    """`total` signatures (1,048,576) statically sharded over the
    ranks (shard_bounds: 131,072 per GPU at 8), each rank's shard verified as whole calls of at
    most `batch` signatures.  Returns the rank's (offset in its shard, count) chunks; offsets are
    multiples of 64, so chunk c's verdict words start at word offset / 64 of the shard's words."""
    lo, hi = shard_bounds(total, world, rank)
    out, o = [], 0
    while lo + o < hi:
        m = min(batch, hi - lo - o)
        out.append((o, m))
        o += m
    return out


def flood_expected(plan: Sequence[Tuple[int, int]], expected: Sequence[np.ndarray], shard_words: int,
                   batch_of_chunk: Callable[[int], int]) -> np.ndarray:
    """The shard's expected words when chunk c verifies the first `count` signatures of batch
    batch_of_chunk(c) (expected[b]: that batch's OpenSSL verdict bools)."""
    v = np.zeros(shard_words * 64, dtype=bool)
    for c, (o, m) in enumerate(plan):
        v[o:o + m] = expected[batch_of_chunk(c)][:m]
    return bools_to_words(v)


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
    _all_gather_into(out, t, dist)
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
