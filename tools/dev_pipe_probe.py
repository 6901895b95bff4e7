"""Device-resident Ed25519 pipeline for a rocprofv3 kernel trace: 64K x 256 B batches over 4,096
keys (radix 13), alternating over two streams as bench.py's headline value does, 30 steps
after 5 warm-up steps; prints the wall-clock rate.  The trace shows how hash, ladder and finish of
consecutive batches overlap (tools/trace_timeline.py)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "concord-bft_amd"), HERE]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

n = 65536
ss = workload.make_sigset(n, nkeys=4096, msg_len=256, seed=0xC0FFEE, threads=16)
dev = torch.device("cuda", 0)
ctx = cb.Context(device=0, max_batch=n)
tid = ctx.load_keys(ss.pk, radix=13)


def to_dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)


d_sig, d_blob = to_dev(ss.sig.reshape(-1), np.uint8), to_dev(ss.blob, np.uint8)
d_off, d_len, d_k = to_dev(ss.off, np.int64), to_dev(ss.len, np.int32), to_dev(ss.key_idx, np.int32)
NS = int(os.environ.get("NSTREAMS", "2"))  # streams the batches alternate over
streams = [torch.cuda.Stream(device=dev) for _ in range(NS)]
outs = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(NS)]


def step(j):  # fixed-length device call, as bench.py's device-resident figure (config #2)
    ctx.verify_fixed_device(tid, 0, d_k.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), 256, n,
                            outs[j % NS].data_ptr(), streams[j % NS].cuda_stream)


for j in range(5):
    step(j)
torch.cuda.synchronize()
t0 = time.perf_counter()
for j in range(30):
    step(j)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
for o in outs:
    assert np.array_equal(cb.bitmap_to_bools(o.cpu().numpy().view(np.uint8).tobytes(), n), ss.expected)
print(f"streams {NS} device-resident {n * 30 / dt / 1e6:.1f} M/s, {dt / 30 * 1e6:.1f} us/step", flush=True)
ctx.close()
