"""Ladder timing probe (device-resident path, one batch at a time, HIP-event stage times).

python tools/ladder_probe.py [--nkeys 1 4096] [--nocheck]
Runs on whatever libcbft_hipcrypto $CBFT_LIB names (an A/B build, tools/build_variant.sh).  With
--nocheck the verdicts are not compared (probe builds that skip the table loads)."""
import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "concord-bft_amd"), os.path.join(ROOT, "tools")]
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nkeys", type=int, nargs="+", default=[4096])
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--radix", type=int, default=13)
    ap.add_argument("--b-radix", type=int, default=0, help="B's comb radix (cbft_set_option; 0 = default 22)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--nocheck", action="store_true")
    ap.add_argument("--sort-keys", action="store_true", help="order the batch by key index (table locality probe)")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    for nk in a.nkeys:
        ss = workload.make_sigset(a.batch, nkeys=nk, msg_len=256, seed=0xC0FFEE, threads=16)
        if a.sort_keys:  # fixed 256-B messages: permute key indices, signatures, message rows, verdicts
            o = np.argsort(ss.key_idx, kind="stable")
            ss.key_idx = np.ascontiguousarray(ss.key_idx[o])
            ss.sig = np.ascontiguousarray(ss.sig.reshape(a.batch, 64)[o]).reshape(ss.sig.shape)
            ss.blob = np.ascontiguousarray(ss.blob[: a.batch * 256].reshape(a.batch, 256)[o]).reshape(-1)
            ss.expected = ss.expected[o]
        ctx = cb.Context(device=0, max_batch=a.batch)
        if a.b_radix:
            ctx.set_option(cb.OPT_B_RADIX, a.b_radix)
        tid = ctx.load_keys(ss.pk, radix=a.radix)

        def to_dev(x, dt):
            return torch.from_numpy(np.ascontiguousarray(x).view(dt)).to(dev)
        d_sig, d_blob = to_dev(ss.sig.reshape(-1), np.uint8), to_dev(ss.blob, np.uint8)
        d_off, d_len = to_dev(ss.off.view(np.int64), np.int64), to_dev(ss.len.view(np.int32), np.int32)
        d_kidx = to_dev(ss.key_idx.view(np.int32), np.int32)
        d_verd = torch.zeros((a.batch + 63) // 64, dtype=torch.int64, device=dev)
        s = torch.cuda.Stream(device=dev)

        def step():  # fixed-length device call, as bench.py's device-resident figure (config #2)
            ctx.verify_fixed_device(tid, 0, d_kidx.data_ptr(), d_sig.data_ptr(), d_blob.data_ptr(), 256, a.batch,
                                    d_verd.data_ptr(), s.cuda_stream)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        ok = None
        if not a.nocheck:
            got = cb.bitmap_to_bools(d_verd.cpu().numpy().view(np.uint8).tobytes(), a.batch)
            ok = bool(np.array_equal(got, ss.expected))
        ctx.set_profiling(True)
        st = {"hash": [], "ladder": [], "finish": []}
        for _ in range(a.reps):
            step()
            for k, v in ctx.stage_times_ms().items():
                st[k].append(v)
        ctx.set_profiling(False)
        print(json.dumps({"lib": os.environ.get("CBFT_LIB", "default"), "nkeys": nk, "sorted": a.sort_keys,
                          "radix": a.radix, "verdicts_ok": ok,
                          "us": {k: round(statistics.median(v) * 1e3, 1) for k, v in st.items()}}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
