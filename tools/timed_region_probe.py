"""Where the contract's timed region spends its time (config #2 headline loop, inputs in HBM).

bench.py times K steps between synchronizes; the same loop with an event after each batch shows a
steadier per-step rate than the timed region's K-step average.  This probe repeats the timed region
(K steps, host wall clock) and, in the same region, records a start event on the first stream and
one event after each batch, so the region splits into: host enqueue time, start gap (host t0 ->
first batch start is not observable; the start event is enqueued first), fill (start -> first
completion), steady intervals and the tail after the last completion.  One JSON line per (K, rep).

    python tools/timed_region_probe.py [--steps 20 200] [--reps 3] [--streams 2]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "concord-bft_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, nargs="+", default=[20, 200])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--events", type=int, default=1, help="record per-batch events inside the region")
ap.add_argument("--ramp", type=int, default=0, help="after 2 s idle, N steps with events: mean step per 20-step window")
ap.add_argument("--nkeys", type=int, default=4096, help="client keys (key-table footprint 10.5 MB each at radix 13)")
ap.add_argument("--distinct", type=int, default=1,
                help="distinct batches cycled over the steps (1 = the same batch every step, as bench.py)")
ap.add_argument("--radix", type=int, default=13, help="key comb radix")
ap.add_argument("--sort-keys", action="store_true", help="every batch ordered by key index (table locality probe)")
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
n, L = 65536, 256
sets = [workload.make_sigset(n, nkeys=args.nkeys, msg_len=L, seed=0xC0FFEE + 7919 * k, threads=16) for k in range(args.distinct)]
if args.sort_keys:  # fixed 256-B messages: permute key indices, signatures, message rows
    for t in sets:
        o = np.argsort(t.key_idx, kind="stable")
        t.key_idx = np.ascontiguousarray(t.key_idx[o])
        t.sig = np.ascontiguousarray(t.sig.reshape(n, 64)[o])
        t.blob = np.ascontiguousarray(t.blob[: n * L].reshape(n, L)[o]).reshape(-1)
ss = sets[0]
ctx = cb.Context(device=0, max_batch=n)
tid = ctx.load_keys(ss.pk, radix=args.radix)
for t in sets[1:]:
    assert np.array_equal(t.pk, ss.pk), "same key set"


def to_dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a).view(dtype)).to(dev)


dsets = [(to_dev(t.sig.reshape(-1), np.uint8), to_dev(t.blob, np.uint8), to_dev(t.key_idx.view(np.int32), np.int32))
         for t in sets]
streams = [torch.cuda.Stream(device=dev) for _ in range(args.streams)]
d_verd = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(args.streams)]


def dstep(j):
    s = streams[j % args.streams]
    d_sig, d_blob, d_kidx = dsets[j % len(dsets)]
    ctx.verify_fixed_device(tid, 0, d_kidx.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), L, n,
                            d_verd[j % args.streams].data_ptr(), s.cuda_stream)


for j in range(max(args.warmup, 2)):
    dstep(j)
torch.cuda.synchronize()
for k in args.steps:
    for rep in range(args.reps):
        for j in range(max(args.warmup, 2)):
            dstep(j)
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        evs = []
        t0 = time.perf_counter()
        start.record(streams[0])
        for j in range(k):
            dstep(j)
            if args.events:
                e = torch.cuda.Event(enable_timing=True)
                e.record(streams[j % args.streams])
                evs.append(e)
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rec = {"steps": k, "rep": rep, "host_ms_per_step": (t1 - t0) * 1e3 / k,
               "enqueue_ms_per_step": (t_enq - t0) * 1e3 / k}
        if evs:
            done = sorted(start.elapsed_time(e) for e in evs)
            gaps = [b - a for a, b in zip(done, done[1:])]
            rec.update({"gpu_span_ms": done[-1], "first_done_ms": done[0],
                        "steady_ms_per_step": (done[-1] - done[0]) / max(1, k - 1),
                        "median_gap_ms": statistics.median(gaps) if gaps else None,
                        "host_minus_gpu_ms": (t1 - t0) * 1e3 - done[-1]})
        print(json.dumps({key: (round(v, 4) if isinstance(v, float) else v) for key, v in rec.items()}), flush=True)
if args.ramp:
    import threading

    import amdsmi

    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    kinds = [k for k in ("SYS", "MEM", "SOC", "DF") if hasattr(amdsmi.AmdSmiClkType, k)]

    def clocks():
        out = {}
        for k in kinds:
            try:
                out[k] = amdsmi.amdsmi_get_clock_info(h, getattr(amdsmi.AmdSmiClkType, k))["clk"]
            except Exception:  # noqa: BLE001
                out[k] = None
        return out

    for idle in (1.0, 0.02):
        time.sleep(idle)
        samples, stop = [], threading.Event()

        def loop():
            t00 = time.perf_counter()
            while not stop.is_set():
                samples.append((round((time.perf_counter() - t00) * 1e3, 1), clocks()))
                time.sleep(0.002)

        th = threading.Thread(target=loop, daemon=True)
        th.start()
        start = torch.cuda.Event(enable_timing=True)
        evs = []
        start.record(streams[0])
        for j in range(args.ramp):
            dstep(j)
            e = torch.cuda.Event(enable_timing=True)
            e.record(streams[j % args.streams])
            evs.append(e)
        torch.cuda.synchronize()
        stop.set()
        th.join()
        done = sorted(start.elapsed_time(e) for e in evs)
        win = [round((done[min(len(done) - 1, k + 20)] - done[k]) / 20, 4) for k in range(0, len(done) - 20, 20)]
        print(json.dumps({"ramp_after_idle_s": idle, "streams": args.streams, "distinct": args.distinct, "nkeys": args.nkeys, "first_done_ms": round(done[0], 4),
                          "window20_ms_per_step": win, "clock_samples_ms_mhz": samples[:: max(1, len(samples) // 12)]}),
              flush=True)
torch.cuda.synchronize()
for j in range(len(dsets)):  # one more pass, each set's verdicts checked
    s0 = streams[0]
    d_sig, d_blob, d_kidx = dsets[j]
    ctx.verify_fixed_device(tid, 0, d_kidx.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), L, n, d_verd[0].data_ptr(),
                            s0.cuda_stream)
    torch.cuda.synchronize()
    got = cb.bitmap_to_bools(d_verd[0].cpu().numpy().view(np.uint8).tobytes(), n)
    assert np.array_equal(got, sets[j].expected), f"set {j}: verdicts differ from OpenSSL"
ctx.close()
