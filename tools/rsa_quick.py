"""Quick RSA-2048 timing on cuda:0: 64K signatures (256 unique, tiled), device-resident inputs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("concord-bft_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch

import cbft_hipcrypto as cb
import rsagen

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
e_sel = sys.argv[2] if len(sys.argv) > 2 else "mixed"
keys = rsagen.load_keys()
ids = None if e_sel == "mixed" else [i for i, k in enumerate(keys) if k["e"] == int(e_sel)]
keys, kidx, sigs, msgs, _ = rsagen.signed_batch(n, nuniq=256, msg_len=256, invalid_frac=0.0, seed=1, key_ids=ids)
torch.zeros(1, device="cuda:0")  # torch initialises HIP first (its runtime, then ours)
with cb.Context(0) as ctx:
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    dev = torch.device("cuda:0")
    blob, offs, lens = cb.pack_messages(msgs)
    d_k = torch.from_numpy(np.asarray(kidx, dtype=np.int32)).to(dev)
    d_s = torch.from_numpy(np.frombuffer(b"".join(sigs), dtype=np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(blob.copy()).to(dev)
    d_o = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    d_l = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
    d_v = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    ctx.set_profiling(True)
    args = (tid, d_k.data_ptr(), d_s.data_ptr(), d_m.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), n, d_v.data_ptr())
    ctx.rsa_verify_device(*args)
    ctx.sync()
    ks = []
    t0 = time.perf_counter()
    for _ in range(5):
        ctx.rsa_verify_device(*args)
        ks.append(ctx.rsa_kernel_ms())
    ctx.sync()
    dt = (time.perf_counter() - t0) / 5
    words = d_v.cpu().numpy().view(np.uint64)
    acc = int(np.unpackbits(words.view(np.uint8), bitorder="little")[:n].sum())
    print(f"rsa n={n} e={e_sel} accept={acc} wall={dt*1e3:.3f} ms kernel={np.median(ks):.3f} ms "
          f"-> {n/dt/1e6:.2f} M verifies/s (kernel {n/np.median(ks)*1e3/1e6:.2f} M/s)")
