"""Config #3 (log-uniform 64..4,096-B messages, 4,096 keys, 64K signatures) with inputs in HBM:
device-resident rate and the hash stage's isolated duration (bench._mixed_device_resident), one
JSON line.  For A/B runs of the hash sort (tools/ab_libs.sh MODE=mixed)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--mixed-streams", type=int, default=4)
args = ap.parse_args()
import torch  # noqa: E402  (initialised first, as bench.py does)

torch.cuda.set_device(0)
ss = workload.make_sigset(65536, nkeys=4096, msg_len=(64, 4096), seed=0xBADC0DE, invalid_frac=0.10, threads=16)
with cb.Context(device=0) as ctx:
    tid = ctx.load_keys(ss.pk)
    value, hash_ms, _steps = bench._mixed_device_resident(ctx, tid, ss, args)
print(json.dumps({"device_resident_value": value, "hash_ms": hash_ms, "streams": args.mixed_streams,
                  "lib": os.environ.get("CBFT_LIB", "default")}))
