"""Ed25519 workloads for rocprofv3 --pmc passes (tools/pmc_passes.sh), one per process so that the
kernels of one configuration are not averaged with another's:

  --mode headline  BASELINE config #2: 64K x 256 B, 4,096 keys (radix 13), 3 batches: hash,
                   pair ladder, batched finish
  --mode small     the p50 path: 20 batches of 1,024 x 256 B through the host entry point
                   (ed25519_small_kernel, one fused launch per batch)
  --mode mixed     BASELINE config #3: 64K, 4,096 keys, 64..4,096 B log-uniform, 10 % invalid,
                   3 batches (the variable-length hash kernel)
Verdicts are checked against host OpenSSL for every batch."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "concord-bft_amd"), HERE]
import numpy as np  # noqa: E402
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=("headline", "small", "mixed"), required=True)
ap.add_argument("--reps", type=int, default=0)
ap.add_argument("--nkeys", type=int, default=0, help="client keys (default: 4,096; 1,024 for small)")
a = ap.parse_args()
n = 1024 if a.mode == "small" else 65536
msg_len = (64, 4096) if a.mode == "mixed" else 256
ss = workload.make_sigset(n, nkeys=a.nkeys or (4096 if a.mode != "small" else 1024), msg_len=msg_len, seed=0xC0FFEE,
                          invalid_frac=0.10 if a.mode == "mixed" else 0.0, threads=16)
reps = a.reps or (20 if a.mode == "small" else 3)
with cb.Context(device=0, max_batch=65536) as ctx:
    tid = ctx.load_keys(ss.pk, radix=13)
    for _ in range(reps):
        got = cb.bitmap_to_bools(ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), n)
        if not np.array_equal(got, ss.expected):
            sys.exit(f"{a.mode}: verdicts differ from OpenSSL")
    ctx.unload_keys(tid)
print(f"{a.mode}: {reps} batches of {n}, verdicts exact", flush=True)
