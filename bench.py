#!/usr/bin/env python3
"""Headline benchmark: Ed25519 batch verification on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

`python bench.py --gpus N` with N > 1 and no launcher starts the N ranks itself (a child
torch.distributed.run, before anything touches the GPU) and exits with its code; a rank whose
WORLD_SIZE differs from --gpus exits non-zero.

A step = one batch of `--batch` (default 65,536) synthetic signed 256-byte messages per GPU,
4,096 keys, BASELINE config #2: the key tables resident on the GPU and, as the bench contract
defines `value`, the batch (signatures, key indices, messages) already resident in HBM when the
timed region starts.  Each GPU holds `--distinct` (default 8) different signed batches with 1 %
planted invalid signatures and the steps cycle through them over three streams
(cbft_ed25519_verify_fixed_device); each step writes its own verdict words, and after the region
every step's words are compared with the OpenSSL verdicts of the batch it verified.  When N > 1
each rank verifies its own static shard (weak scaling) and each step's verdict words are
all-gathered over RCCL (the only cross-GPU traffic north_star prescribes); the rank path is
concord-bft_amd/cbft_multigpu.py, which the gloo CPU tests drive.  value = signatures verified by
all ranks / max-over-ranks wall time.  Config #5 (1,048,576 signatures sharded over the ranks, one
all-gather) is timed beside it as `flood_config5`.

SURVEY.md §8(d) also quotes config #2 with the host -> device copy inside the step: that rate
(`pcie_inclusive_value`: pinned host batches -> cbft_ed25519_verify_fixed_async, batch i+1's copy
under batch i's kernels, bitmap back on the host) is timed the same way over the same distinct
batches, every step's bitmap checked, and reported beside it with its PCIe bound.

Verdicts are checked bit-exact against the host OpenSSL before any number is printed.  Also
reported: the roofline of the dominant kernel (INT32 VALU, SURVEY.md §8(d) algorithmic ops) with
the PCIe host->device bound of the PCIe-inclusive rate beside it,
the host-CPU OpenSSL baseline on every core this process may use (rank 0, every N), p50 latency at
batch 1K, and the config #3 / #4 / RSA side measurements.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "concord-bft_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import cbft_hipcrypto as cb  # noqa: E402  (ctypes binding; the library loads at the first Context)
import cbft_multigpu as mg  # noqa: E402  (the rank path: timing, per-step verdicts + all-gathers, flood plan)
import gpu_clocks  # noqa: E402  (sclk / mclk through amdsmi, best effort)
import parity_gate  # noqa: E402  (golden-data verdict gate, run before anything is timed)
import tree_hash  # noqa: E402  (csrc stamp: PMC records are attached only to the tree they describe)
import workload  # noqa: E402

METRIC = "Ed25519 verifies/sec at batch 64K on 1–8 MI355X; p50 latency @ batch 1K"
# INT32 VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (CDNA4 SIMDs are 32-wide;
# MI355X_MICROARCH.md; v_add_u32 measured at 0.88 of it, tools/microbench/intrate.hip)
INT32_PEAK = 256 * 4 * 32 * 2.4e9
MAD64_PEAK = INT32_PEAK / 2  # v_mad_u64_u32 issues at half the INT32 rate
# Algorithmic INT32 ops per verify, SURVEY.md §8(d) model (8x32-bit limbs: M = 72, S = 44):
OPS_DSM = 1020 * 44 + 1460 * 72            # double-scalar multiplication [S]B - [h]A = 150,000
OPS_DECODE = 256 * 44 + 20 * 72            # A decode
OPS_ENCODE = 254 * 44 + 13 * 72            # R' inversion + encode
SHA_OPS_PER_BLOCK = 5000
# PCIe Gen5 x16 host -> device: 32 GT/s x 16 lanes x 128/130 = 63.0 GB/s per direction
PCIE_PEAK = 32e9 * 16 * 128 / 130 / 8


def ops_per_verify(m: int) -> int:
    return OPS_DSM + OPS_DECODE + OPS_ENCODE + SHA_OPS_PER_BLOCK * ((64 + m + 17 + 127) // 128)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--msg-len", type=int, default=256)
    ap.add_argument("--distinct", type=int, default=8,
                    help="distinct signed batches per GPU cycled through the timed loops (8 x 21 MB of inputs)")
    ap.add_argument("--invalid-frac", type=float, default=0.01,
                    help="planted invalid signatures per batch (R / S / message bit flips, S + L, wrong key)")
    ap.add_argument("--flood", type=int, default=1 << 20,
                    help="config #5: total signatures sharded over the ranks (0 = skip)")
    ap.add_argument("--flood-reps", type=int, default=5)
    ap.add_argument("--nkeys", type=int, default=4096)
    ap.add_argument("--comb-radix", type=int, default=13,
                    help="radix 2^r of the per-key comb tables (8..15; 13 = 10.5 MB per key, 43 GB at 4,096 keys; "
                         "15 = 35.7 MB per key, 146 GB)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = every core we may use)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--latency-runs", type=int, default=200)
    ap.add_argument("--inflight", type=int, default=4, help="host-path batches in flight")
    ap.add_argument("--mixed-streams", type=int, default=4, help="config #3 device-resident streams")
    ap.add_argument("--streams", type=int, default=3, help="headline (config #2) device-resident streams")
    ap.add_argument("--single-process-devices", default="",
                    help="also time one process over these devices (comma list, repeats allowed: cbft_open_devices); "
                         "with --gpus N > 1 rank 0 does this over all N GPUs (cbft_open_mask) by default")
    ap.add_argument("--no-extras", dest="extras", action="store_false",
                    help="skip the config #3 (mixed), config #4 (BLS) and RSA-2048 side measurements")
    return ap.parse_args()


def _spawn_ranks(n: int) -> int:
    """Start n ranks (one per GPU) through torch.distributed.run as a child process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={29500 + os.getpid() % 1000}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.call(cmd)


def _cpu_cores() -> tuple[int, str]:
    """CPUs this process may use: sched_getaffinity, capped by the cgroup CPU quota (cpu.max) when
    one is set — more threads than the quota only get throttled (measured: 256 threads on a
    16-CPU quota verify 4x slower than 16)."""
    affinity = len(os.sched_getaffinity(0))
    cores, note = affinity, f"sched_getaffinity = {affinity}"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
            cores = max(1, min(affinity, int(quota + 0.5)))
            note += f", cgroup cpu.max quota = {quota:.1f} CPUs"
    except Exception:  # noqa: BLE001
        pass
    return cores, note


def _bind_near_gpu(torch, index: int):
    """Multi-GPU: run this rank on the CPUs of its GPU's NUMA node (sysfs local_cpulist of the PCIe
    device), so that its pinned staging buffers -- allocated by this process, first-touch -- sit in
    the memory next to its PCIe link and 8 ranks do not pull 8 x 54 GB/s across the socket link.
    Best effort: returns the node, or None when the topology is not readable."""
    try:
        pr = torch.cuda.get_device_properties(index)
        bdf = f"{getattr(pr, 'pci_domain_id', 0):04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        base = f"/sys/bus/pci/devices/{bdf}"
        node = int(open(f"{base}/numa_node").read())
        cpus = set()
        for part in open(f"{base}/local_cpulist").read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        mine = cpus & os.sched_getaffinity(0)
        if node < 0 or not mine:
            return None
        os.sched_setaffinity(0, mine)
        return node
    except Exception:  # noqa: BLE001
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args.gpus))  # before anything initialises the GPU
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CBFT_BENCH_SHARED_GPU=1: a rehearsal of the N > 1 rank path on a one-GPU box -- every rank on
    # device 0, a gloo process group (cbft_multigpu stages the collectives through the host).  It
    # runs the same code as an N-GPU run except RCCL; its rates are not a scaling measurement.
    shared_gpu = world > 1 and os.environ.get("CBFT_BENCH_SHARED_GPU") == "1"
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(0 if shared_gpu else local)
        dist.init_process_group("gloo" if shared_gpu else "nccl")  # RCCL on ROCm
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    numa = _bind_near_gpu(torch, dev.index) if world > 1 else None
    cores, quota = _cpu_cores()
    cpu_threads = args.cpu_threads or cores
    clocks = gpu_clocks.Clocks(torch, dev.index)
    clk_before = clocks.read()  # here, not between the warm-up and the timed region (no idle gap there)

    # ---- workload: this rank's static shard (weak scaling).  --distinct batches (default 8), each its
    # own set of n OpenSSL-signed L-byte messages over the same 4,096 keys with --invalid-frac
    # (default 1 %) planted bad signatures (a flipped bit of R, S or M, S + L, the wrong key: every one
    # runs the whole hash -> ladder -> finish pipeline).  The timed loops cycle through the batches,
    # each step writes its own verdict words, and after each timed region every step's words are
    # compared with the OpenSSL verdicts of the batch it verified (a stale or skipped launch leaves
    # zero words, which 99 % valid batches cannot match).
    n, L = args.batch, args.msg_len
    nb = max(1, args.distinct)
    nwords = (n + 63) // 64
    gen_t0 = time.perf_counter()
    sets = [workload.make_sigset(n, nkeys=args.nkeys, msg_len=L, seed=0xC0FFEE + rank + 7919 * b,
                                 invalid_frac=args.invalid_frac, threads=min(cpu_threads, 64)) for b in range(nb)]
    gen_s = time.perf_counter() - gen_t0
    ss = sets[0]
    invalid = [int((~s.expected).sum()) for s in sets]
    ctx = cb.Context(device=dev.index, max_batch=n)
    # parity first: every golden verdict class (Ed25519 edge cases through both key modes, the
    # RELIC key fixture, RSA accepts and rejects); any mismatch exits non-zero before timing
    parity = parity_gate.run(ctx, rsa=args.extras, relic=args.extras)
    # the OpenSSL verdict words of every batch on this device (and, N > 1, every rank's)
    exp_rows = torch.from_numpy(np.stack([mg.bools_to_words(s.expected) for s in sets])).to(dev)
    all_exp = mg.all_gather_rows(exp_rows, world, dist) if world > 1 else None
    gstream = torch.cuda.Stream(device=dev) if world > 1 else None

    def verdicts(steps):  # per-step verdict words (+ their all-gathers when N > 1)
        return mg.StepVerdicts(nwords, steps, world, rank, dist, dev, gstream)

    def require_exact(ver, what, steps=None):
        bad = ver.mismatches(exp_rows, lambda j: j % nb, steps, all_exp)
        if world > 1:
            bad = mg.sum_over_ranks(bad, dist, dev)
        if bad:
            raise SystemExit(f"rank {rank}: {what}: {bad} verdict words differ from OpenSSL's")

    def sync_all():
        torch.cuda.synchronize()
        if gstream is not None:
            gstream.synchronize()

    def timed(fn, steps):
        """Contract timing: barrier + synchronize on both sides, max over ranks."""
        return mg.timed_region(fn, steps, dist if world > 1 else None, sync_all, dev)

    # the batches as a caller builds them: each in one pinned host block (cbft_host_alloc) laid out as
    # cbft_ed25519_batch_layout says, so each step's host -> device transfer is one DMA
    blocks = []
    for s in sets:
        blk, h_kidx, h_sig, b_raw = ctx.batch_views(n, L)
        h_kidx[:] = s.key_idx
        h_sig[:] = s.sig
        b_raw[:] = s.blob[: n * L]
        blocks.append((blk, h_kidx, h_sig, b_raw))
    depth = max(1, args.inflight)

    def run(steps, bitmaps, ver=None):
        """Host-buffer pipeline: step st verifies batch st % nb into bitmaps[st % len(bitmaps)],
        `depth` batches in flight; ver (N > 1: the gather, and the post-region check) takes each
        step's bitmap once cbft_wait has delivered it."""
        tickets = []

        def done(st):
            ctx.wait(tickets[st])
            if ver is not None:
                ver.after_host_step(st, bitmaps[st % len(bitmaps)])

        for st in range(steps):
            _, h_kidx, h_sig, b_raw = blocks[st % nb]
            tickets.append(ctx.verify_async(tid, h_kidx, h_sig, b_raw, bitmaps[st % len(bitmaps)], msg_len=L, n=n))
            if st >= depth - 1:
                done(st - depth + 1)
        for st in range(max(0, steps - depth + 1), steps):
            done(st)

    def host_mismatch(bitmaps, steps):
        bad = 0
        for st in range(steps):
            got = cb.bitmap_to_bools(bitmaps[st][: (n + 7) // 8].tobytes(), n)
            bad += int((got != sets[st % nb].expected).sum())
        return bad

    # ---- the headline: inputs resident in HBM, cbft_ed25519_verify_fixed_device (the device form
    # of the fixed-length call; config #2's messages are all L bytes) rotating over --streams streams
    # (default 3: each stream's hash -> ladder -> finish chain then covers three batches) and over
    # the nb distinct batches; verdict words left in HBM (a buffer per step); with N > 1 each step's
    # words are all-gathered over RCCL on the gather stream.
    def to_dev(a: np.ndarray, dtype):
        return torch.from_numpy(np.ascontiguousarray(a).view(dtype)).to(dev)

    for s in sets:
        assert np.array_equal(s.off, np.arange(n, dtype=s.off.dtype) * L), "config #2 blob is n x L bytes"
    dsets = [(to_dev(s.sig.reshape(-1), np.uint8), to_dev(s.blob, np.uint8), to_dev(s.key_idx.view(np.int32), np.int32))
             for s in sets]
    nst = max(1, args.streams)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nst)]

    def dstep(j, ver, table=None):
        s = streams[j % nst]
        d_sig, d_blob, d_kidx = dsets[j % nb]
        ctx.verify_fixed_device(tid if table is None else table, 0, d_kidx.data_ptr(), d_sig.data_ptr(),
                                d_blob.data_ptr(), L, n, ver.words_ptr(j), s.cuda_stream)
        ver.after_step(j, s)

    def drun_with(ver, table=None):
        def go(steps):
            for j in range(steps):
                dstep(j, ver, table)
        return go

    def headline():
        """warm-up + the contract's timed region; every step's words checked after it."""
        drun_with(verdicts(max(args.warmup, 2)))(max(args.warmup, 2))
        ver = verdicts(args.steps)
        el = timed(drun_with(ver), args.steps)
        clk = clocks.read()
        require_exact(ver, "headline (device-resident)")
        return el, clk

    t_keys = time.perf_counter()
    tid = ctx.load_keys(ss.pk, radix=args.comb_radix)  # key tables resident, like SigManager's verifiers
    key_load_ms = (time.perf_counter() - t_keys) * 1e3
    # ---- the host pipeline's first check: one pass over every batch, before anything else is timed
    first = [np.zeros(nwords * 8, dtype=np.uint8) for _ in range(nb)]
    run(nb, first)
    if host_mismatch(first, nb):
        raise SystemExit(f"rank {rank}: host pipeline: GPU verdicts differ from OpenSSL on "
                         f"{host_mismatch(first, nb)} signatures")
    # ---- PCIe-inclusive rate (SURVEY.md §8(d) config #2 as written: sig + msg copied from pinned
    # host memory each step, bitmap back to the host).  Reported beside `value`, never as it: the
    # contract's value has its inputs resident in HBM when the timed region starts.
    run(args.warmup, [np.zeros(nwords * 8, dtype=np.uint8) for _ in range(depth)])
    bitmaps = [np.zeros(nwords * 8, dtype=np.uint8) for _ in range(max(1, args.steps))]
    hver = verdicts(args.steps) if world > 1 else None
    pcie_elapsed = timed(lambda k: run(k, bitmaps, hver), args.steps)
    pcie_value = world * n * args.steps / pcie_elapsed
    if host_mismatch(bitmaps, args.steps):  # every step's bitmap, against its own batch
        raise SystemExit(f"rank {rank}: PCIe-inclusive leg: GPU verdicts differ from OpenSSL")
    if hver is not None:
        require_exact(hver, "PCIe-inclusive leg (all-gathered bitmaps)")
    # the same K steps right after the PCIe leg, whose PCIe-bound batches leave the GPU mostly idle:
    # the first ~200 device-resident batches after idle run 10-20 % slower (the memory-side clocks
    # ramp), so this is the cold-start figure, reported beside `value`
    cold_elapsed, _ = headline()
    parity["config2_headline"] = {"batches": nb, "n": n * nb, "invalid": int(sum(invalid)), "mismatch": 0,
                                  "steps_checked": args.steps,
                                  "reference": "host OpenSSL EVP_DigestVerify(ED25519), each step's verdict words "
                                               "against the batch it verified (device and PCIe legs)"}

    # ---- 1,048,576 signatures (--flood) statically sharded over the ranks
    # (131,072 per GPU at N = 8), each rank's shard as calls of `n` over the distinct batches on the
    # headline's streams, then ONE all-gather of the shard's verdict words (16 KiB per GPU at 8);
    # a fixed total, so this is the strong-scaling figure beside the weak-scaling `value`
    flood = None
    if args.flood:
        total = args.flood
        plan = mg.flood_plan(total, world, rank, n)
        sw = mg.shard_size(total, world) // 64
        fwords = torch.zeros(sw, dtype=torch.int64, device=dev)
        fexp = torch.from_numpy(mg.flood_expected(plan, [s.expected for s in sets], sw, lambda c: c % nb)).to(dev)
        cur = torch.cuda.current_stream(dev)
        fout = {}

        def flood_run(reps):
            for _ in range(reps):
                for c, (o, m) in enumerate(plan):
                    s = streams[c % nst]
                    s.wait_stream(cur)  # the previous flood's gather has read the words
                    d_sig, d_blob, d_kidx = dsets[c % nb]
                    ctx.verify_fixed_device(tid, 0, d_kidx.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), L, m,
                                            fwords.data_ptr() + (o // 64) * 8, s.cuda_stream)
                for s in streams:
                    cur.wait_stream(s)
                fout["g"] = mg.gather_verdicts(fwords, total, world, dist) if world > 1 else fwords

        flood_run(1)
        reps = max(1, args.flood_reps)
        fel = timed(flood_run, reps)
        bad = int((fwords != fexp).sum().item())
        if world > 1:
            want = mg.all_gather_rows(fexp, world, dist).view(-1)[: (total + 63) // 64]
            bad = mg.sum_over_ranks(bad + int((fout["g"] != want).sum().item()), dist, dev)
        if bad:
            raise SystemExit(f"rank {rank}: config #5 flood: {bad} verdict words differ from OpenSSL's")
        flood = {"total_signatures": total, "per_rank": mg.shard_size(total, world), "calls_per_rank": len(plan),
                 "reps": reps, "ms_per_flood": fel / reps * 1e3, "value": total * reps / fel, "mismatch": 0,
                 "gather_bytes_per_rank": sw * 8 if world > 1 else 0,
                 "scaling": "strong (fixed total over the ranks)"}
        parity["config5_flood"] = {"n": total, "mismatch": 0}


    # ---- the spread of the step: the same pipeline again, untimed by the
    # contract, with an event after each batch on its stream: intervals between consecutive batch
    # completions (median / min / max), and the GFX clock sampled by amdsmi while it runs
    def drun_events(steps, ver):
        evs = []
        for j in range(steps):
            dstep(j, ver)
            e = torch.cuda.Event(enable_timing=True)
            e.record(streams[j % nst])
            evs.append(e)
        torch.cuda.synchronize()
        return evs

    spread_steps = max(args.steps, 200)
    sver = verdicts(spread_steps)
    evs, clk_load = clocks.sample_during(lambda: drun_events(spread_steps, sver))
    require_exact(sver, "step-spread run")
    del sver
    done = sorted(evs[0].elapsed_time(e) for e in evs)
    gaps = [b - a for a, b in zip(done, done[1:])]
    step_spread = {"steps": spread_steps, "median_ms": statistics.median(gaps), "min_ms": min(gaps),
                   "max_ms": max(gaps), "steady_ms_per_step": (done[-1] - done[0]) / (len(done) - 1),
                   "first_steps_ms": [round(g, 4) for g in gaps[:5]]}

    # ---- the contract's timed region: W warm-up steps + K timed steps, every step's verdict words
    # checked after it, on the GPU that has just run the flood and the 200-batch spread run above
    # (sustained operation, as a replica's verifier runs)
    elapsed, clk_after = headline()
    value = world * n * args.steps / elapsed
    step_spread["timed_region_ms_per_step"] = elapsed / args.steps * 1e3
    gpu_clk = {"at_start": clk_before, "after_timed": clk_after, "under_load": clk_load,
               "note": clocks.why}

    # ---- the client-count cliff: the key table's comb radix falls from 13 to
    # 11 past ~5.9K keys and to 8 past ~21K keys per device ($CBFT_COMB_BUDGET_GB = 64, whole
    # 256-key chunks; include/cbft_hipcrypto.h); the same headline loop at each radix
    cliff = []
    if args.extras:
        budget = float(os.environ.get("CBFT_COMB_BUDGET_GB", "64")) * 1e9
        for r in sorted({13, 11, 8} - {args.comb_radix} | {args.comb_radix}, reverse=True):
            per_key = _comb_npos(r) * ((1 << (r - 1)) + 1) * 128
            row = {"comb_radix": r, "additions_per_verify": _comb_npos(r) + 12,
                   "table_mb_per_key": round(per_key / 1e6, 3),
                   "table_gb_per_device_at_nkeys": round(args.nkeys * per_key / 1e9, 2),
                   "max_keys_in_budget": int(budget // (256 * per_key)) * 256}
            if r == args.comb_radix:
                row["value"] = value
            else:
                tr = ctx.load_keys(ss.pk, radix=r)
                try:
                    drun_with(verdicts(max(args.warmup, 2)), tr)(max(args.warmup, 2))
                    rver = verdicts(args.steps)
                    row["value"] = world * n * args.steps / timed(drun_with(rver, tr), args.steps)
                    require_exact(rver, f"comb radix {r}")
                finally:
                    ctx.unload_keys(tr)
            cliff.append(row)

    # ---- kernel durations inside this same pipeline (per-batch HIP events on the launch streams)
    ctx.set_profiling(True, per_batch=True)
    pver = verdicts(args.steps)
    drun_with(pver)(args.steps)
    torch.cuda.synchronize()
    pipe_stage, pipe_batches = ctx.stage_times_avg_ms()
    ctx.set_profiling(False)
    require_exact(pver, "profiled pipeline")
    ladder_ms = pipe_stage["ladder"]
    ctx.set_profiling(True)
    iso = {"hash": [], "ladder": [], "finish": []}
    iver = verdicts(5)
    for j in range(5):
        dstep(j, iver)  # one batch at a time: kernel durations without overlap
        for k, v in ctx.stage_times_ms().items():
            iso[k].append(v)
    ctx.set_profiling(False)
    torch.cuda.synchronize()
    require_exact(iver, "isolated batches")
    del dsets, pver, iver

    # ---- PCIe host -> device copy rate of this box (pinned, 256 MiB), for the PCIe bound
    src = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        dst.copy_(src, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    h2d_rate = 4 * (256 << 20) / (e0.elapsed_time(e1) * 1e-3)
    del src, dst

    # ---- roofline: the dominant kernel (INT32 VALU) + the PCIe bound of the whole step
    # the ladder layout the library picks (cbft_hipcrypto.cpp): two lanes per signature from 32K
    lanes = 2 if n >= 32768 else 4
    b_radix = 22  # CBFT_COMB_B_RADIX (ed25519_verify.h)
    kname = "ed25519_comb2_ladder_kernel" if lanes == 2 else "ed25519_comb_ladder_kernel"
    # PMC record of the headline workload (tools/ed_pmc_probe.py --mode headline under
    # tools/pmc_passes.sh): attached only while it was collected on this csrc tree
    traffic = slot_ops = None
    lrec, lstat = _pmc_record("pmc_ed25519_headline.json", kname)
    if lrec:
        traffic = lrec.get("hbm_bytes")
        slot_ops = (lrec["SQ_INSTS_VALU"] + lrec["SQ_INSTS_VALU_INT64"]) * 64 \
            if "SQ_INSTS_VALU" in lrec and "SQ_INSTS_VALU_INT64" in lrec else None
    # Algorithmic work of the comb ladder: one mixed addition per comb position (radix-2^w_A key
    # table + radix-2^w_B B table), 7 field multiplications each, 81 + 9 v_mad_u64_u32 per
    # multiplication (9 x 29-bit limbs, fe25519.h); the pair / quad combines are parallelisation
    # overhead and not counted.  Bound: the MAD64 pipe (half the INT32 issue rate).
    npos = {8: 32, 9: 29, 10: 26, 11: 23, 12: 22, 13: 20, 14: 19, 15: 17}[args.comb_radix] + \
        {16: 16, 17: 15, 18: 15, 19: 14, 20: 13, 21: 13, 22: 12, 23: 11, 24: 11, 25: 11, 26: 10}[b_radix]
    # each pair-ladder lane's first addition starts from the identity and is a point set (1 M, not
    # 7: ed25519_comb2_ladder_kernel), so a verify is (npos - 2) x 7 + 2 x 1 M
    first_sets = 2 if lanes == 2 else 0
    mads_per_unit = ((npos - first_sets) * 7 + first_sets) * 90
    achieved = mads_per_unit * n / (ladder_ms * 1e-3)
    h2d_bytes = 4 + 64 + L  # key index + R||S + message, per signature (fixed-length batch)
    roofline = {"bound": "valu_mad64", "achieved": achieved / 1e12, "peak": MAD64_PEAK / 1e12, "unit": "T MAD64/s",
                "frac": achieved / MAD64_PEAK, "traffic": traffic,
                "kernel": kname, "kernel_ms": ladder_ms, "units_per_launch": n,
                "ops_per_unit": mads_per_unit,
                "achieved_basis": f"{npos} comb positions: {npos - first_sets} additions x 7 field mults + {first_sets} first "
                                  f"point sets x 1, x 90 v_mad_u64_u32 per verify x units / "
                                  f"mean ladder launch ({pipe_batches} launches, HIP events on the launch streams, "
                                  f"inside the timed pipeline)",
                "issue_frac": (slot_ops / (ladder_ms * 1e-3) / INT32_PEAK) if slot_ops else None,
                "pmc": _pmc_brief(lrec, lstat),
                "stage_ms_pipelined": {k: round(v, 4) for k, v in pipe_stage.items()},
                "stage_ms_isolated": {k: round(statistics.median(v), 4) for k, v in iso.items()},
                # the same work over the ladder's duration when it runs alone (one batch at a time):
                # inside the pipeline the batches' kernels share the SIMDs (from three streams two
                # ladders co-run), which stretches every launch while the step gets shorter
                "frac_isolated": mads_per_unit * n / (statistics.median(iso["ladder"]) * 1e-3) / MAD64_PEAK,
                # the ladder's work per step over the whole step time (ms_per_step)
                "frac_of_step": mads_per_unit * n / (elapsed / args.steps) / MAD64_PEAK,
                "pcie": {"bound": "pcie_h2d", "of": "pcie_inclusive_value",
                         "achieved": pcie_value / world * h2d_bytes / 1e9, "peak": PCIE_PEAK / 1e9,
                         "measured_copy_rate": h2d_rate / 1e9, "unit": "GB/s",
                         "frac": pcie_value / world * h2d_bytes / PCIE_PEAK,
                         "frac_of_measured": pcie_value / world * h2d_bytes / h2d_rate,
                         "bytes_per_unit": h2d_bytes}}

    # ---- the replica's own multi-GPU form: ONE process over all N devices (cbft_open_mask), the
    # same per-device batch as a shard of one N x batch call, verdicts gated as above
    single = None
    sp_devices = [int(x) for x in args.single_process_devices.split(",") if x] or \
        (([0] * world if shared_gpu else list(range(world))) if world > 1 else [])
    if world > 1:
        dist.barrier()
    if rank == 0 and sp_devices:
        single = bench_single_process(args, ss, sp_devices, mask=(world > 1 and not args.single_process_devices and not shared_gpu))
    if world > 1:
        dist.barrier()
    # config #4 sharded over the ranks (the BLS multi-GPU rows); the single-GPU legs below run at N = 1
    bls_sharded = bench_bls_sharded(ctx, args, cpu_threads, world, rank, dist, dev) if (world > 1 and args.extras) else None

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu:  # every N (north_star: "in the same run"), after every timed region
            kc = workload.cpu_lib().cbft_cpu_keys_new(workload._p(ss.pk), ss.pk.shape[0])
            try:
                workload.cpu_verify(ss, threads=cpu_threads, keycache=kc)  # warm-up batch
                ts = []
                for _ in range(5):
                    c0 = time.perf_counter()
                    v = workload.cpu_verify(ss, threads=cpu_threads, keycache=kc)
                    ts.append(time.perf_counter() - c0)
                assert np.array_equal(v.astype(bool), ss.expected)
            finally:
                workload.cpu_lib().cbft_cpu_keys_free(kc, ss.pk.shape[0])
            cpu = {"value": n / statistics.median(ts), "unit": "verifies/s", "cores": cpu_threads,
                   "kind": "reference",
                   "sample": f"OpenSSL {_openssl_version()} EVP_DigestVerify(ED25519), EVP_PKEY cached per key, "
                             f"{cpu_threads} pthreads = every CPU this process may use ({quota}"
                             + (f"; rank 0 bound to NUMA node {numa}" if numa is not None else "") +
                             f"), static ranges; median of 5 passes over batch 0 ({n} x {L} B, "
                             f"{invalid[0]} invalid) after 1 warm-up pass"}
        # p50 end-to-end latency at batch 1K: the caller's (pageable) host arrays -> one blocking
        # cbft_ed25519_verify_batch -> bitmap on host (what a C++ SigManager::verifySigBatch call
        # costs); the Python-list form (messages packed by the binding each call) beside it
        lat = lat_py = None
        if args.latency_runs > 0:
            k = min(1024, n)
            msgs = ss.msgs()[:k]
            kidx, sig = np.ascontiguousarray(ss.key_idx[:k]), np.ascontiguousarray(ss.sig[:k])
            blob_k, off_k, len_k = cb.pack_messages(msgs)

            def p50(fn):
                for _ in range(5):
                    fn()
                lt = []
                for _ in range(args.latency_runs):
                    c0 = time.perf_counter()
                    bm = fn()
                    lt.append((time.perf_counter() - c0) * 1e3)
                assert np.array_equal(cb.bitmap_to_bools(bm, k), ss.expected[:k])
                return statistics.median(lt)

            lat = p50(lambda: ctx.verify_packed(tid, kidx, sig, blob_k, off_k, len_k))
            lat_py = p50(lambda: ctx.verify(tid, kidx, sig, msgs))
        # pageable caller buffers, blocking calls (the library packs them into pinned staging)
        ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len)
        ht = []
        for _ in range(5):
            c0 = time.perf_counter()
            bm = ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len)
            ht.append(time.perf_counter() - c0)
        assert np.array_equal(cb.bitmap_to_bools(bm, n), ss.expected)
        pageable = n / statistics.median(ht)
        mixed = bench_mixed(ctx, args, cpu_threads) if (args.extras and world == 1) else None
        bls = bench_bls(ctx, args, cpu_threads) if (args.extras and world == 1) else None
        rsa = bench_rsa(ctx, args, cpu_threads) if (args.extras and world == 1) else None
        per_request = bench_per_request(cpu_threads) if (args.extras and world == 1) else None
        if mixed:
            parity["config3_mixed"] = {"n": mixed["n"], "invalid": mixed["invalid"],
                                       "mismatch": mixed["n"] - mixed["exact_match"],
                                       "pipelined_exact": mixed["pipelined_verdicts_exact"]}
        if bls:
            parity["config4_bls"] = bls.pop("parity")
        if rsa:
            parity["rsa_2048_bench_sets"] = {"n": 2 * args.batch, "mismatch": 0}
        detail = _write_detail({"workload_gen_s": gen_s, "flood_config5": flood, "step_spread": step_spread, "gpu_clocks": gpu_clk, "comb_radix_cliff": cliff,
                                "comb_radix_cliff_fields": "comb radix, M verifies/s, MB per key, max keys in budget",
                                "parity": parity, "roofline": roofline, "mixed_config3": mixed, "bls_config4": bls,
                                "rsa_2048": rsa, "per_request_path": per_request, "single_process_multi_gpu": single,
                                "bls_config4_sharded": bls_sharded})
        small_name = "ed25519_small3_kernel"  # the fused small-batch kernel
        small_k, small_stat = _pmc_record("pmc_ed25519_small.json", small_name)
        # The line: the contract's keys first, then side measurements, and LAST what the driver's
        # stdout tail must keep: the second half of the metric (p50 @ 1K), the
        # device-resident ceiling, the per-request path, the key-table load and the BLS timings.
        out = {
            "metric": METRIC, "value": value, "unit": "verifies/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "ed25519_verify_64k_256B_4096keys (BASELINE config #2, inputs resident in HBM: "
                                   "sig + key index + msg, key tables resident; PCIe-inclusive rate in "
                                   "pcie_inclusive_value)",
                       "batch_per_gpu": n, "msg_len": L, "nkeys": args.nkeys, "comb_radix": args.comb_radix,
                       "b_comb_radix": b_radix, "ladder_lanes_per_signature": lanes,
                       "inputs": f"HBM (cbft_ed25519_verify_fixed_device, {nst} streams); verdict words stay in HBM",
                       "timed_after": "the PCIe leg, the config #5 flood and a 200-batch untimed run of the same "
                                      "pipeline (warm GPU); the same K steps right after the PCIe leg: "
                                      "cold_start_value",
                       "batches": f"{nb} distinct signed batches per GPU cycled through every timed loop, "
                                  f"{args.invalid_frac:.0%} planted invalid ({invalid}); every step's verdicts "
                                  f"checked against OpenSSL after the region",
                       "config5": "flood_config5: --flood total (1,048,576) sharded over the ranks, 131,072 per "
                                  "GPU at N = 8 (= --batch 131072 per rank), one RCCL all-gather of verdict words",
                       "pcie_inclusive_inputs": "pinned host memory (cbft_host_alloc) -> GPU each step; bitmap -> host",
                       "inflight_batches": depth,
                       "parallelism": f"static shard x{world}" + (
                           ", REHEARSAL: every rank on GPU 0, gloo process group (CBFT_BENCH_SHARED_GPU=1), "
                           "not a scaling measurement" if shared_gpu else
                           ", RCCL all-gather of verdict bitmaps" if world > 1 else ""),
                       "rank0_numa_node": numa},
            "roofline": roofline, "cpu_baseline": cpu,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu else None,
            "verdicts": "bit-exact vs host OpenSSL (checked before and after timing)",
            "parity": {"all_exact": True, "blocks": _parity_counts(parity), "detail": detail},
            "flood_config5": _brief(flood, ("value", "ms_per_flood", "per_rank", "calls_per_rank", "mismatch")),
            "cold_start_value": world * n * args.steps / cold_elapsed,
            "cold_start_ms_per_step": cold_elapsed / args.steps * 1e3,
            "pageable_host_value": pageable,
            "single_process_multi_gpu": _brief(single, ("value", "devices", "open", "ms_per_step")),
            "bls_config4_sharded": bls_sharded,
            "step_spread_ms": [round(step_spread[k], 4) for k in ("median_ms", "min_ms", "max_ms",
                                                                   "steady_ms_per_step")],
            "sclk_mhz": _clk_brief(gpu_clk),
            "comb_radix_cliff": [[r["comb_radix"], round(r["value"] / 1e6, 1), r["table_mb_per_key"],
                                  r["max_keys_in_budget"]] for r in cliff],
            "rsa_2048": _rsa_brief(rsa),
            "mixed_config3": _brief(mixed, ("value", "pipelined_pinned_value", "device_resident_value", "device_resident_batches",
                                            "hash_kernel_ms", "hash_pmc", "exact_match", "n")),
            "bls_config4": _bls_brief(bls),
            "per_request_path": _per_request_brief(per_request),
            "key_table_load_ms": key_load_ms,
            "pcie_inclusive_value": pcie_value,
            "pcie_inclusive_ms_per_step": pcie_elapsed / args.steps * 1e3,
            "p50_small_kernel_pmc": _pmc_tail(small_k, small_stat),
            "p50_latency_ms_batch1k_python_lists": lat_py,
            "p50_latency_ms_batch1k": lat,
        }
        print(json.dumps(out), flush=True)
    for blk in blocks:
        ctx.host_free(blk[0])
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def _clk_brief(clk: dict):
    """[sclk at the start of the run, after the timed region, median / min under load] (MHz) and mclk,
    or why not."""
    b, a, ld = clk.get("at_start"), clk.get("after_timed"), clk.get("under_load")
    if not (b or a or ld):
        return clk.get("note")
    return [b and b["sclk_mhz"], a and a["sclk_mhz"], ld and ld["sclk_mhz_median"], ld and ld["sclk_mhz_min"],
            (a or b or {}).get("mclk_mhz")]


def _comb_npos(radix: int) -> int:
    """Positions of a radix-2^radix comb over 253-bit scalars (ed25519_verify.h CombGeom)."""
    return {8: 32, 9: 29, 10: 26, 11: 23, 12: 22, 13: 20, 14: 19, 15: 17}[radix]


def _pmc_record(fname: str, kernel: str):
    """(counters of `kernel`, status) from profiles/<fname> (tools/pmc_record.py), or (None, why):
    a record collected on another csrc tree (tools/tree_hash.py) is stale and dropped."""
    path = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(path):
        return None, f"profiles/{fname} absent"
    try:
        rec = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, f"profiles/{fname} unreadable: {e}"
    if rec.get("csrc_tree") != tree_hash.csrc_tree_hash():
        return None, f"profiles/{fname} stale (csrc tree {rec.get('csrc_tree')} != {tree_hash.csrc_tree_hash()}): dropped"
    k = rec.get("kernels", {}).get(kernel)
    if k is None:
        return None, f"profiles/{fname} has no {kernel}"
    return k, f"profiles/{fname} (csrc tree {rec['csrc_tree']})"


def _pmc_brief(k, status):
    """The per-kernel PMC fields the bench line carries."""
    out = {"source": status}
    if k:
        for key in ("duration_ms", "waves_per_simd", "valu_insts_per_wave", "valu_active_frac", "issue_stall_frac",
                    "waitcnt_frac", "wave_cycles_per_valu", "mad_frac_of_peak", "hbm_bytes"):
            if k.get(key) is not None:
                out[key] = round(k[key], 4) if isinstance(k[key], float) else k[key]
    return out


def _pmc_tail(k, status):
    """A short form for the end of the line (the driver keeps ~2 KB of stdout): the full fields
    are in the record under profiles/."""
    if not k:
        return {"source": status}
    return {"us": round(k["duration_ms"] * 1e3, 1) if k.get("duration_ms") else None,
            "valu_active": round(k.get("valu_active_frac") or 0, 3), "waitcnt": round(k.get("waitcnt_frac") or 0, 3),
            "waves_per_simd": k.get("waves_per_simd"), "stamp": status.split("csrc tree ")[-1].rstrip(")")}


def _write_detail(rec: dict) -> str:
    """The full per-class parity record and every side measurement, as a file beside the run
    (gpurun_out/ when it exists, which gpurun brings back; the builder copies it under profiles/)."""
    d = os.path.join(ROOT, "gpurun_out")
    path = os.path.join(d if os.path.isdir(d) else os.path.join(ROOT, "profiles"), "bench_detail_last.json")
    try:
        with open(path, "w") as f:
            json.dump(rec, f, indent=1, default=str)
    except OSError:
        return "unwritten"
    return os.path.relpath(path, ROOT)


def _brief(rec, keys):
    if not rec:
        return None
    return {k: (round(rec[k], 5) if isinstance(rec[k], float) else rec[k]) for k in keys if k in rec}


def _per_request_brief(pr):
    if not pr:
        return None
    v, o, one = pr["verify_mt"], pr["openssl_mt"], pr["single"]
    return {"verify_mt_per_s": v["verifies_per_s"], "verify_mt_p50_us": v["p50_us"], "verify_mt_p99_us": v["p99_us"],
            "threads": v["threads"], "calls_per_batch": v["calls_per_batch"], "single_call_p50_us": one["p50_us"],
            "verifysig_mt_per_s": pr["verifysig_mt"]["verifies_per_s"], "openssl_mt_per_s": o["verifies_per_s"],
            "openssl_threads": o["threads"], "gpu_vs_openssl_mt": pr["gpu_vs_openssl_mt"]}


def _rsa_brief(rsa):
    if not rsa:
        return None
    out = {}
    for label in ("client_e65537", "replica_e17"):
        r = rsa.get(label)
        if r:
            out[label] = {"value": r["value"], "kernel_ms": round(r["kernel_ms"], 4),
                          "frac": round(r["roofline"]["frac"], 4), "cpu_value": r["cpu_baseline"]["value"]}
    return out


def _bls_brief(bls):
    if not bls:
        return None
    out = {k: (round(bls[k], 4) if isinstance(bls[k], float) else bls[k])
           for k in ("certificate_ms", "certificate_fused_ms", "certificate_policy_ms", "share_verify_ms",
                     "combine_ms", "verify_ms", "optimistic_ms", "multisig_ms", "sign_ms", "public_key_ms",
                     "keyset_load_ms") if k in bls}
    rf = bls.get("roofline") or {}
    # compact for the driver's ~2 KB stdout tail: the kernels on the certificate / sign / key paths
    # as [mean us, VALU-active fraction, MAD64 fraction of peak]; every kernel's record is in the
    # detail file (bench_detail_last.json) and profiles/pmc_bls.json
    ks = rf.get("kernels") or {}
    keep = ("bls_share_verify_kernel", "bls_verify_kernel", "bls_verify_multisig_kernel", "bls_msm_row_kernel",
            "bls_sign_row_kernel", "bls_pubkey_row_kernel", "bls_keys_row_kernel")
    brief = {}
    for name, k in ks.items():
        base = name.split("(")[0].split("<")[0].replace("void ", "")
        if base in keep and k.get("duration_ms") is not None:
            brief[name.replace("void ", "").split("(")[0]] = [round(k["duration_ms"] * 1e3, 1),
                                                                round(k.get("valu_active_frac") or 0, 3),
                                                                round(k.get("mad_frac_of_peak") or 0, 4)]
    out["kernels_pmc"] = brief or None
    out["kernels_pmc_fields"] = "mean us, valu_active, mad_frac_of_peak"
    out["pmc_source"] = rf.get("source")
    if bls.get("cpu_baseline"):
        out["cpu_baseline_shares_per_s"] = bls["cpu_baseline"]["value"]
    return out


def _parity_counts(parity: dict) -> dict:
    """Counts per gate block for the bench line (the per-class detail goes to a file)."""
    out = {}
    for name, blk in parity.items():
        if not isinstance(blk, dict):
            continue
        if "vectors" in blk:
            out[name] = {"n": blk["vectors"], "mismatch": blk.get("mismatch", 0)}
        elif "n" in blk or "shares" in blk:
            out[name] = {"n": blk.get("n", blk.get("shares")),
                         "mismatch": blk.get("mismatch", blk.get("share_verdict_mismatch", 0))}
        else:
            out[name] = {"checks": sum(v for v in blk.values() if isinstance(v, int)), "mismatch": 0}
    return out


def bench_single_process(args, ss, devices, mask):
    """One process over several GPUs (cbft_open_mask / cbft_open_devices): each step is ONE
    len(devices) x batch signature call, cut by the library into per-device shards of whole
    64-signature words that run concurrently, verdicts landing in one bitmap (the
    in-process form a replica would use).  Key table replicated per device; same pinned-host
    pipeline as the headline; every slot's verdicts checked against OpenSSL's."""
    G, n, L = len(devices), args.batch, args.msg_len
    N = G * n
    g = cb.Context(device_mask=sum(1 << d for d in devices), max_batch=N) if mask else \
        cb.Context(devices=devices, max_batch=N)
    try:
        tid = g.load_keys(ss.pk, radix=args.comb_radix)
        blk, h_kidx, h_sig, b_raw = g.batch_views(N, L)
        h_kidx[:] = np.tile(ss.key_idx, G)
        h_sig[:] = np.tile(ss.sig, (G, 1))
        b_raw[:] = np.tile(ss.blob[: n * L], G)
        expected = np.tile(ss.expected, G)
        depth = max(1, args.inflight)
        outs = [np.zeros(N // 8 + 1, dtype=np.uint8) for _ in range(depth)]

        def run(steps):
            tk = []
            for st in range(steps):
                tk.append(g.verify_async(tid, h_kidx, h_sig, b_raw, outs[st % depth], msg_len=L, n=N))
                if st >= depth - 1:
                    g.wait(tk[st - depth + 1])
            for st in range(max(0, steps - depth), steps):
                g.wait(tk[st])

        run(1)
        if not np.array_equal(cb.bitmap_to_bools(outs[0][: (N + 7) // 8].tobytes(), N), expected):
            raise SystemExit("single-process multi-GPU: verdicts differ from OpenSSL")
        run(args.warmup)
        t0 = time.perf_counter()
        run(args.steps)
        dt = time.perf_counter() - t0
        for j in range(min(depth, args.steps)):
            if not np.array_equal(cb.bitmap_to_bools(outs[j][: (N + 7) // 8].tobytes(), N), expected):
                raise SystemExit("single-process multi-GPU: pipelined verdicts differ from OpenSSL")
        g.host_free(blk)
        return {"value": N * args.steps / dt, "unit": "verifies/s", "devices": devices,
                "open": "cbft_open_mask" if mask else "cbft_open_devices", "batch_per_call": N,
                "ms_per_step": dt / args.steps * 1e3, "verdicts_exact": True,
                "basis": f"{args.steps} steps of one {N}-signature call (per-device shards of {n}), "
                         f"{depth} in flight, pinned host inputs, H2D included"}
    finally:
        g.close()


def bench_per_request(cpu_threads):
    """The per-request path: 64 threads each calling HipEdDSAVerifier::verify /
    HipSigManager::verifySig one signature at a time, as the reference's pool threads call
    IVerifier::verify (ClientRequestMsg.cpp:197-213, ReplicaConfig.hpp:202-212); the engine
    coalesces concurrent calls into GPU batches.  tools/host_bench (C++, the unsanitized host
    library) checks every verdict and exits non-zero on a mismatch."""
    exe = os.path.join(ROOT, "tools", "host_bench")
    if not os.path.exists(exe):
        raise SystemExit("tools/host_bench missing: make host")
    r = subprocess.run([exe, "64", "2000", "1024", str(cpu_threads)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"host_bench failed (verdict mismatch or error): {r.stdout[-2000:]} {r.stderr[-2000:]}")
    out = json.loads(r.stdout)
    out["basis"] = ("64 threads x 2000 single calls over 1024 client keys, 256-B messages, every 10th signature "
                    "corrupted; openssl_mt = OpenSSL 3 EVP_DigestVerify on the same signatures, EVP_PKEY cached "
                    f"per key, {cpu_threads} threads")
    return out


def _median_ms(fn, runs: int) -> float:
    ts = []
    for _ in range(runs):
        c0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - c0) * 1e3)
    return statistics.median(ts)


def bench_mixed(ctx, args, cpu_threads):
    """BASELINE config #3 (SigManager mixed): 4,096 keys, lengths log-uniform in [64, 4096] B,
    10 % invalid (R/S bit flips, S + L, message byte, wrong key).  Host buffers in, bitmap out
    (what SigManager::verifySigBatch does); exact-match count against OpenSSL."""
    n = args.batch
    ss = workload.make_sigset(n, nkeys=args.nkeys, msg_len=(64, 4096), seed=0xBADC0DE, invalid_frac=0.10,
                              threads=min(cpu_threads, 64))
    tid = ctx.load_keys(ss.pk)
    try:
        bm = ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len)
        got = cb.bitmap_to_bools(bm, n)
        match = int((got == ss.expected).sum())
        if match != n:
            raise SystemExit(f"config #3: GPU verdicts differ from OpenSSL on {n - match} signatures")
        ms = _median_ms(lambda: ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), 5)
        # the same batches handed over the way the headline does: arrays in pinned host memory
        # (cbft_host_alloc), cbft_ed25519_verify_batch_async with 4 batches in flight
        views = []

        def pinned(a: np.ndarray) -> np.ndarray:
            raw = ctx.host_alloc(max(1, a.nbytes))
            views.append(raw)
            v = raw[:a.nbytes].view(a.dtype).reshape(a.shape)
            v[...] = a
            return v
        try:
            pk_idx, p_sig, p_blob = pinned(ss.key_idx), pinned(ss.sig), pinned(ss.blob)
            p_off, p_len = pinned(ss.off), pinned(ss.len)
            depth, steps = 4, 20
            outs = [np.zeros(n // 8 + 1, dtype=np.uint8) for _ in range(depth)]

            def run(k):
                tk = []
                for st in range(k):
                    if st >= depth:
                        ctx.wait(tk[st - depth])
                    tk.append(ctx.verify_async(tid, pk_idx, p_sig, p_blob, outs[st % depth], offs=p_off,
                                               lens=p_len, n=n))
                for t in tk[max(0, k - depth):]:
                    ctx.wait(t)
            run(depth)
            c0 = time.perf_counter()
            run(steps)
            pipe = n * steps / (time.perf_counter() - c0)
            pipe_match = all(np.array_equal(cb.bitmap_to_bools(o[: (n + 7) // 8].tobytes(), n), ss.expected)
                             for o in outs)
            if not pipe_match:
                raise SystemExit("config #3: pipelined verdicts differ from OpenSSL")
        finally:
            for v in views:
                ctx.host_free(v)
        dres, hash_ms, dsteps = _mixed_device_resident(ctx, tid, ss, args)
    finally:
        ctx.unload_keys(tid)
    hk, hstat = _pmc_record("pmc_ed25519_mixed.json", "ed25519_hash_kernel<0>")
    return {"config": f"config #3: {n} sigs, 4096 keys, msg 64-4096 B log-uniform, 10% invalid",
            "device_resident_value": dres, "device_resident_batches": dsteps, "hash_kernel_ms": hash_ms, "hash_pmc": _pmc_brief(hk, hstat),
            "value": n / (ms * 1e-3), "unit": "verifies/s (pageable host buffers, blocking call, PCIe included)",
            "pipelined_pinned_value": pipe,
            "pipelined_pinned_basis": "pinned host arrays (cbft_host_alloc), cbft_ed25519_verify_batch_async, "
                                      "4 batches in flight, 20 batches timed, PCIe included",
            "pipelined_verdicts_exact": bool(pipe_match),
            "exact_match": match, "n": n, "invalid": int((~ss.expected).sum()),
            "msg_bytes_total": int(ss.len.sum())}


def _mixed_device_resident(ctx, tid, ss, args):
    """Config #3 with its inputs already in HBM (cbft_ed25519_verify_batch_device, --mixed-streams):
    the GPU's own rate on the variable-length batch, and the hash kernel's isolated duration."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device())
    n = ss.n

    def to_dev(a, dtype):
        return torch.from_numpy(np.ascontiguousarray(a).view(dtype).copy()).to(dev)

    d_sig, d_blob = to_dev(ss.sig.reshape(-1), np.uint8), to_dev(ss.blob, np.uint8)
    d_off, d_len, d_k = to_dev(ss.off, np.int64), to_dev(ss.len, np.int32), to_dev(ss.key_idx, np.int32)
    # more streams than the fixed-length headline's two: a batch's long-message tail (up to 33
    # SHA-512 blocks on one lane) then runs under the next batches' short hashes and ladders
    # (the library rotates over as many work slots, CBFT_OPT_WORK_SLOTS, default 4)
    ns = max(1, getattr(args, "mixed_streams", 4))
    streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    outs = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(ns)]

    def dstep(j):
        ctx.verify_device(tid, 0, d_k.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), d_off.data_ptr(),
                          d_len.data_ptr(), n, outs[j % ns].data_ptr(), streams[j % ns].cuda_stream)

    for j in range(8):
        dstep(j)
    torch.cuda.synchronize()
    # a sustained sample (>= 100 batches, ~30 ms): with four streams in flight a short run is mostly
    # pipeline fill and drain, and the first ~200 batches after an idle gap run 10-20 % slow on
    # every kernel; config #3 is a side figure, not bound to the headline's K
    steps = max(100, args.steps)
    c0 = time.perf_counter()
    for j in range(steps):
        dstep(j)
    torch.cuda.synchronize()
    value = n * steps / (time.perf_counter() - c0)
    for o in outs:
        if not np.array_equal(cb.bitmap_to_bools(o.cpu().numpy().view(np.uint8).tobytes(), n), ss.expected):
            raise SystemExit("config #3: device-path verdicts differ from OpenSSL")
    ctx.set_profiling(True)
    hs = []
    for _ in range(3):
        dstep(0)
        hs.append(ctx.stage_times_ms()["hash"])
    ctx.set_profiling(False)
    return value, statistics.median(hs), steps


# MAD64_PEAK (top): v_mad_u64_u32 issues at half the INT32 rate (MI355X_MICROARCH.md): 256 CU x 4
# SIMD x 16 lanes x 2.4 GHz = 3.93e13 MAC/s; measured 3.28e13 on the microbench
# (tools/microbench/intrate.hip, profiles/r01_intrate_microbench.txt), reported beside it
MAD64_MEASURED = 3.277e13


def bench_rsa(ctx, args, cpu_threads):
    """RSA-2048 PKCS#1 v1.5 / SHA-256 batch verify (the verifier SigManager
    instantiates today).  64K signatures over 256-byte messages, inputs resident in HBM, client
    keys (e = 65537) and replica keys (e = 17); verdicts checked against the host OpenSSL and the
    host-buffer path before timing.  CPU baseline: OpenSSL RSA verify on 16 threads, same set."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rsagen

    n = args.batch
    keys = rsagen.load_keys()
    out = {"config": f"{n} x 256 B messages, RSA-2048, 256 distinct signed messages tiled", "unit": "verifies/s"}
    dev = torch.device("cuda", torch.cuda.current_device())
    mods = np.frombuffer(b"".join(k["n"].to_bytes(256, "big") for k in keys), dtype=np.uint8)
    exps = np.array([k["e"] for k in keys], dtype=np.uint32)
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    kc = workload.cpu_lib().cbft_cpu_rsa_keys_new(workload._p(mods), workload._p(exps), len(keys))
    try:
        for label, e in (("client_e65537", 65537), ("replica_e17", 17)):
            ids = [i for i, k in enumerate(keys) if k["e"] == e]
            _, kidx, sigs, msgs, _ = rsagen.signed_batch(n, nuniq=256, msg_len=args.msg_len, invalid_frac=0.0,
                                                        seed=e, key_ids=ids)
            blob, offs, lens = cb.pack_messages(msgs)
            kidx_a = np.asarray(kidx, dtype=np.uint32)
            sig_a = np.frombuffer(b"".join(sigs), dtype=np.uint8)
            d_k = torch.from_numpy(kidx_a.view(np.int32).copy()).to(dev)
            d_s = torch.from_numpy(sig_a.copy()).to(dev)
            d_m = torch.from_numpy(blob.copy()).to(dev)
            d_o = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
            d_l = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
            d_v = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            a = (tid, d_k.data_ptr(), d_s.data_ptr(), d_m.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), n,
                 d_v.data_ptr())
            ctx.rsa_verify_device(*a)
            ctx.sync()
            words = d_v.cpu().numpy().view(np.uint64)
            got = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)
            host = cb.bitmap_to_bools(ctx.rsa_verify(tid, kidx_a, sig_a, msgs), n)
            cpu_v = np.zeros(n, dtype=np.uint8)
            workload.cpu_lib().cbft_cpu_rsa_verify(kc, workload._p(kidx_a), workload._p(sig_a), workload._p(blob),
                                                   workload._p(offs), workload._p(lens), n, workload._p(cpu_v),
                                                   cpu_threads)
            if not (got.all() and np.array_equal(got, host) and np.array_equal(got, cpu_v.astype(bool))):
                raise SystemExit(f"RSA verdicts differ ({label})")
            steps = max(5, args.steps // 2)
            for _ in range(2):
                ctx.rsa_verify_device(*a)
            ctx.sync()
            c0 = time.perf_counter()
            for _ in range(steps):
                ctx.rsa_verify_device(*a)
            ctx.sync()
            wall = (time.perf_counter() - c0) / steps
            ctx.set_profiling(True)
            kms = []
            for _ in range(5):
                ctx.rsa_verify_device(*a)
                kms.append(ctx.rsa_kernel_ms())
            ctx.set_profiling(False)
            kms = statistics.median(kms)
            nbits = e.bit_length()
            products = 1 + (nbits - 1) + bin(e).count("1") + 1  # CONV + squarings + multiplies + REDC
            # v_mad_u64_u32 per verify of the lane-pair radix-2^28 schedule (74 rows x 2 x 74 columns)
            macs = products * 74 * 148
            ts = []
            workload.cpu_lib().cbft_cpu_rsa_verify(kc, workload._p(kidx_a), workload._p(sig_a), workload._p(blob),
                                                   workload._p(offs), workload._p(lens), n, workload._p(cpu_v),
                                                   cpu_threads)
            for _ in range(3):
                c0 = time.perf_counter()
                workload.cpu_lib().cbft_cpu_rsa_verify(kc, workload._p(kidx_a), workload._p(sig_a),
                                                       workload._p(blob), workload._p(offs), workload._p(lens), n,
                                                       workload._p(cpu_v), cpu_threads)
                ts.append(time.perf_counter() - c0)
            cpu_value = n / statistics.median(ts)
            out[label] = {
                "value": n / wall, "kernel_ms": kms, "kernel_value": n / (kms * 1e-3),
                "roofline": {"bound": "valu_mad_u64_u32", "achieved": macs * n / (kms * 1e-3) / 1e12,
                             "peak": MAD64_PEAK / 1e12, "unit": "T MAC/s",
                             "frac": macs * n / (kms * 1e-3) / MAD64_PEAK, "macs_per_verify": macs,
                             "frac_of_measured_mad_rate": macs * n / (kms * 1e-3) / MAD64_MEASURED,
                             "kernel": "rsa_verify_pair_kernel"},
                "cpu_baseline": {"value": cpu_value, "unit": "verifies/s", "cores": cpu_threads,
                                 "kind": "reference",
                                 "sample": f"OpenSSL {_openssl_version()} EVP_DigestVerify(RSA PKCS#1 v1.5, "
                                           f"SHA-256), EVP_PKEY per key, {cpu_threads} pthreads; median of "
                                           f"3 passes over the same {n} signatures"},
                "gpu_vs_cpu": (n / wall) / cpu_value,
            }
            del d_k, d_s, d_m, d_o, d_l, d_v
    finally:
        workload.cpu_lib().cbft_cpu_keys_free(kc, len(keys))
        ctx.rsa_unload_keys(tid)
    out["verdicts"] = "device path == host path == host OpenSSL, all accept"
    return out


def bench_bls(ctx, args, cpu_threads):
    """BASELINE config #4: threshold BLS on BN-P254, n = 1,024 replicas, k = 2f+1 = 683, 32-byte
    digest.  Unit = one commit certificate: verify 760 shares (10 % of them doubled, i.e. bad),
    Lagrange-combine 683 valid ones, verify the combined signature.  Also the multisig variant
    (sum of shares, signer bitmap, 1 verify) and the 0 %-bad optimistic path (combine + verify)."""
    n, k = 1024, 683
    cert = workload.make_bls_cert(n, k, extra=77, bad_frac=0.10, seed=2024, threads=cpu_threads)
    kid = ctx.bls_load_keys(cert.pk, cert.vks)
    try:
        if not all(ctx.bls_key_status(kid, n)):
            raise SystemExit("BLS keyset: a verification key failed to decode on the GPU")
        h33 = ctx.bls_hash_to_g1(cert.msg)
        valid = ctx.bls_verify_shares(kid, cert.msg, cert.shares)
        exp = np.array([j not in cert.bad for j in range(len(cert.shares))])
        if not np.array_equal(np.asarray(valid, dtype=bool), exp):
            raise SystemExit("BLS share verdicts differ from the expected bad set")
        use = [s for j, s in enumerate(cert.shares) if valid[j]][:k]
        comb = ctx.bls_combine(use)
        if comb != cert.expected_sig or not ctx.bls_verify(kid, cert.msg, comb):
            raise SystemExit("BLS combined signature differs from sk * H(m)")
        ids = [int.from_bytes(s[:4], "big") for s in use]
        bitmap = bytearray(256)
        for i in ids:
            bitmap[(i - 1) // 8] |= 1 << ((i - 1) % 8)
        msig = ctx.bls_combine(use, multisig=True)
        if not ctx.bls_verify_multisig(kid, cert.msg, msig, bytes(bitmap)):
            raise SystemExit("BLS multisig does not verify")
        planted = ~exp
        bad_bitmaps = {}
        for label, opt in (("fallback", False), ("policy", True)):
            sig, ok, badv = ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=opt)
            if not ok or sig != cert.expected_sig or not np.array_equal(np.asarray(badv, dtype=bool), planted):
                raise SystemExit(f"BLS combine_threshold ({label}): ok={ok}, signature or bad-share bitmap differs "
                                 f"({int((np.asarray(badv, dtype=bool) != planted).sum())} bits)")
            bad_bitmaps[label] = int(np.asarray(badv, dtype=bool).sum())
        parity = {"shares": len(cert.shares), "planted_bad": len(cert.bad), "share_verdict_mismatch": 0,
                  "combine_threshold_bad_bitmap": bad_bitmaps, "combined_sig": "== sk*H(m) byte-exact",
                  "multisig": "verifies under the signer bitmap",
                  "note": "expected shares / signature from the host build of the same BN-P254 source; the "
                          "independent oracle bytes are gated by relic_bls_fixture"}
        runs = 5
        t_share = _median_ms(lambda: ctx.bls_verify_shares(kid, cert.msg, cert.shares), runs)
        t_comb = _median_ms(lambda: ctx.bls_combine(use), runs)
        t_ver = _median_ms(lambda: ctx.bls_verify(kid, cert.msg, comb), runs)

        def certificate():
            v = ctx.bls_verify_shares(kid, cert.msg, cert.shares)
            u = [s for j, s in enumerate(cert.shares) if v[j]][:k]
            c = ctx.bls_combine(u)
            assert ctx.bls_verify(kid, cert.msg, c)

        def optimistic():
            c = ctx.bls_combine(use)
            assert ctx.bls_verify(kid, cert.msg, c)

        def multisig():
            c = ctx.bls_combine(use, multisig=True)
            assert ctx.bls_verify_multisig(kid, cert.msg, c, bytes(bitmap))

        def fused():  # cbft_bls_combine_threshold, fallback form: verify shares, combine valid, verify
            sig, ok, badv = ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=False)
            assert ok and sig == cert.expected_sig and np.array_equal(np.asarray(badv, dtype=bool), planted)

        def policy():  # reference policy: optimistic combine of all 760 (fails: 10 % bad) -> fallback
            sig, ok, badv = ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=True)
            assert ok and sig == cert.expected_sig and np.array_equal(np.asarray(badv, dtype=bool), planted)

        # a threshold keyset (re)load, as on a per-window key rotation (CryptoManager.hpp:116-141):
        # 1,024 vks + the group key decoded, subgroup-checked and their Miller-loop lines built
        t_load = _median_ms(lambda: ctx.bls_unload_keys(ctx.bls_load_keys(cert.pk, cert.vks)), 3)
        t_cert = _median_ms(certificate, runs)
        t_fused = _median_ms(fused, runs)
        t_policy = _median_ms(policy, runs)
        t_opt = _median_ms(optimistic, runs)
        t_ms = _median_ms(multisig, runs)
        # replica-side signing (IThresholdSigner::signData, BlsThresholdSigner.cpp:32-47) and the
        # signer's verification key (sk * g2), checked against the host build's bytes
        sid, sk, share = cert.sign_probe
        if ctx.bls_sign(sk, sid, cert.msg) != share:
            raise SystemExit("BLS signData: GPU share differs from the expected bytes")
        if ctx.bls_public_key(sk) != cert.vks[sid - 1]:
            raise SystemExit("BLS public key: GPU sk*g2 differs from the key set's vk")
        t_sign = _median_ms(lambda: ctx.bls_sign(sk, sid, cert.msg), runs)
        t_pub = _median_ms(lambda: ctx.bls_public_key(sk), 3)
    finally:
        ctx.bls_unload_keys(kid)
    nsh = len(cert.shares)
    out = {"config": f"config #4: n={n}, k={k}, {nsh} shares ({len(cert.bad)} bad, doubled), 32-B digest",
           "certificate_ms": t_cert, "certificates_per_s": 1e3 / t_cert,
           "share_verify_ms": t_share, "shares_per_s": nsh / (t_share * 1e-3),
           "pairings_per_s": 2 * nsh / (t_share * 1e-3),
           "certificate_fused_ms": t_fused,
           "certificate_fused_basis": "one cbft_bls_combine_threshold(optimistic=0) call: 760 share verifies, "
                                      "Lagrange + MSM over the valid ones, final verify, all on the device",
           "certificate_policy_ms": t_policy,
           "certificate_policy_basis": "cbft_bls_combine_threshold(optimistic=1): the reference's "
                                       "SignaturesProcessingJob order -- optimistic combine of all shares + verify "
                                       "(fails with 10 % bad), then the fallback",
           "combine_ms": t_comb, "verify_ms": t_ver, "optimistic_ms": t_opt, "multisig_ms": t_ms,
           "keyset_load_ms": t_load, "sign_ms": t_sign, "public_key_ms": t_pub,
           "keyset_load_basis": f"cbft_bls_load_keys + unload of {n} vks + the group key (decode, subgroup check, "
                                f"70 normalised Miller-loop lines per key)",
           "verdicts": "share verdicts == planted bad set; combined sig == sk*H(m) byte-exact",
           "parity": parity}
    out["roofline"] = _bls_roofline()
    if not args.no_cpu:
        workload.cpu_bls_verify_shares(cert, h33, threads=cpu_threads)  # warm-up
        c0 = time.perf_counter()
        v = workload.cpu_bls_verify_shares(cert, h33, threads=cpu_threads)
        dt = time.perf_counter() - c0
        assert np.array_equal(v.astype(bool), exp)
        out["cpu_baseline"] = {"value": nsh / dt, "unit": "shares/s", "cores": cpu_threads, "kind": "port",
                               "sample": f"{nsh} share verifies (2 pairings + G2 lines each) with this library's "
                                         f"own BN-P254 code compiled for the host: an UNOPTIMISED port, not RELIC "
                                         f"(absent) and not an optimized CPU pairing; no speed-up is claimed "
                                         f"against it"}
    return out


def bench_bls_sharded(ctx, args, cpu_threads, world, rank, dist, dev):
    """Config #4 across the ranks (N > 1), through cbft_multigpu: each
    rank verifies its slice of the 760 shares (one all-gather of the validity bitmap), each rank
    Lagrange-sums its slice of the 683 valid shares (one all-gather of the G1 partials, then the
    sum), and the multisig public key is summed by id range (one all-gather of G2 partials) before
    the pairing check.  Every rank builds the same certificate; every result is checked on every
    rank; times are the contract's (barrier + synchronize, max over ranks), median of 5."""
    n, k = 1024, 683
    cert = workload.make_bls_cert(n, k, extra=77, bad_frac=0.10, seed=2024, threads=cpu_threads)
    kid = ctx.bls_load_keys(cert.pk, cert.vks)
    exp = np.array([j not in cert.bad for j in range(len(cert.shares))])
    use = [s for j, s in enumerate(cert.shares) if exp[j]][:k]
    bitmap = bytearray(256)
    for i in (int.from_bytes(s[:4], "big") for s in use):
        bitmap[(i - 1) // 8] |= 1 << ((i - 1) % 8)
    bitmap = bytes(bitmap)
    bad = 0

    def shares():
        return mg.bls_verify_shares_sharded(ctx, kid, cert.msg, cert.shares, world, rank, dist, dev)

    def combine():
        return mg.bls_combine_sharded(ctx, use, world, rank, dist, dev)

    def multisig():
        msig = mg.bls_combine_sharded(ctx, use, world, rank, dist, dev, multisig=True)
        return mg.bls_verify_multisig_sharded(ctx, kid, n, cert.msg, msig, bitmap, world, rank, dist, dev)

    def certificate():
        v = shares()
        c = mg.bls_combine_sharded(ctx, [s for j, s in enumerate(cert.shares) if v[j]][:k], world, rank, dist, dev)
        return c == cert.expected_sig and ctx.bls_verify(kid, cert.msg, c)

    try:
        bad += int((np.asarray(shares(), dtype=bool) != exp).sum())
        bad += int(combine() != cert.expected_sig)
        bad += int(not multisig())
        bad += int(not certificate())
        bad = mg.sum_over_ranks(bad, dist, dev)
        if bad:
            raise SystemExit(f"rank {rank}: sharded BLS config #4: {bad} results differ from the expected ones")

        import torch

        def med(fn):
            ts = [mg.timed_region(lambda _s: fn(), 1, dist, torch.cuda.synchronize, dev) * 1e3 for _ in range(5)]
            return statistics.median(ts)

        out = {"config": f"config #4 over {world} ranks: n={n}, k={k}, {len(cert.shares)} shares "
                         f"({len(cert.bad)} bad)",
               "share_verify_ms": med(shares), "combine_ms": med(combine), "multisig_ms": med(multisig),
               "certificate_ms": med(certificate),
               "shares_per_rank": mg.share_slice(len(cert.shares), world, 0)[1],
               "verdicts": "share bitmap == planted bad set, combined sig == sk*H(m), multisig verifies, on "
                           "every rank"}
    finally:
        ctx.bls_unload_keys(kid)
    return out


def _bls_roofline():
    """BLS kernels are latency-bound, not throughput-bound: a pairing check is one dependent
    instruction stream per wave, 760 checks fill 760 of 1,024 SIMDs once, and a certificate is a
    chain of such kernels.  Their roofline is therefore the per-wave issue rate, with the MAD64
    fraction alongside to show how far from the throughput peak the latency form sits.  From
    profiles/pmc_bls.json (tools/pmc_passes.sh over tools/bls_probe.py -> tools/pmc_record.py),
    attached only while its csrc stamp matches this tree."""
    path = os.path.join(ROOT, "profiles", "pmc_bls.json")
    if not os.path.exists(path):
        return {"source": "profiles/pmc_bls.json absent"}
    rec = json.load(open(path))
    if rec.get("csrc_tree") != tree_hash.csrc_tree_hash():
        return {"source": f"profiles/pmc_bls.json stale (csrc tree {rec.get('csrc_tree')} != "
                          f"{tree_hash.csrc_tree_hash()}): dropped"}
    ks = {}
    for name, k in rec["kernels"].items():
        ks[name] = {key: (round(k[key], 4) if isinstance(k.get(key), float) else k.get(key))
                    for key in ("duration_ms", "waves_per_simd", "mad_frac_of_peak", "wave_cycles_per_valu",
                                "valu_active_frac")}
    return {"bound": "latency: one wave per pairing check / point chain (per-wave VALU issue)",
            "kernels": ks, "source": f"profiles/pmc_bls.json (csrc tree {rec['csrc_tree']})"}


def _openssl_version():
    try:
        import ctypes
        lib = ctypes.CDLL("libcrypto.so.3")
        lib.OpenSSL_version.restype = ctypes.c_char_p
        return lib.OpenSSL_version(0).decode()
    except Exception:
        return "libcrypto"


if __name__ == "__main__":
    main()
