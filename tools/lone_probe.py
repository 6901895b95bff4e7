"""Latency split of the small-batch path: p50 wall time of lone (n = 1) and 1K verify_packed calls
from pageable arrays, beside the round trip of an empty torch kernel (launch + completion, the
floor any launched kernel pays).  Run it under `rocprofv3 --kernel-trace --stats` to read the
fused kernel's own duration for the same calls."""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "concord-bft_amd"), HERE]
import numpy as np  # noqa: E402
import torch  # noqa: E402  (initialised before the library touches HIP)

torch.cuda.set_device(0)
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

RUNS = int(os.environ.get("RUNS", "300"))
ss = workload.make_sigset(1024, nkeys=64, msg_len=256, seed=11)
ctx = cb.Context(device=0)
tid = ctx.load_keys(ss.pk)


def p50(fn):
    for _ in range(20):
        fn()
    t = []
    for _ in range(RUNS):
        c0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - c0) * 1e6)
    return round(statistics.median(t), 1)


out = {}
x = torch.zeros(1, device="cuda")


def empty():
    x.add_(1)
    torch.cuda.synchronize()


out["torch_empty_kernel_roundtrip_us"] = p50(empty)
for n in (1, 1024):
    kidx, sig = np.ascontiguousarray(ss.key_idx[:n]), np.ascontiguousarray(ss.sig[:n])
    blob, off, ln = np.ascontiguousarray(ss.blob[:256 * n]), np.ascontiguousarray(ss.off[:n]), np.ascontiguousarray(ss.len[:n])
    bm = ctx.verify_packed(tid, kidx, sig, blob, off, ln)
    assert np.array_equal(cb.bitmap_to_bools(bm, n), ss.expected[:n])
    out[f"verify_packed_n{n}_p50_us"] = p50(lambda: ctx.verify_packed(tid, kidx, sig, blob, off, ln))
print(json.dumps(out), flush=True)
ctx.close()
