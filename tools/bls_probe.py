"""BLS config #4 probe for rocprofv3: one certificate's phases (share verify, combine, verify,
multisig), each run `--reps` times after a warm-up, printing per-phase wall times (JSON).
Run under `rocprofv3 --kernel-trace --stats` or `--pmc ...` to attribute kernel time and
counters to bls_* kernels."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "concord-bft_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--k", type=int, default=683)
a = ap.parse_args()
cert = workload.make_bls_cert(a.n, a.k, extra=77, bad_frac=0.10, seed=2024, threads=16)
ctx = cb.Context(device=0)
kid = ctx.bls_load_keys(cert.pk, cert.vks)
valid = ctx.bls_verify_shares(kid, cert.msg, cert.shares)
use = [s for j, s in enumerate(cert.shares) if valid[j]][: a.k]
comb = ctx.bls_combine(use)
assert comb == cert.expected_sig and ctx.bls_verify(kid, cert.msg, comb)
bitmap = bytearray(256)
for s in use:
    i = int.from_bytes(s[:4], "big")
    bitmap[(i - 1) // 8] |= 1 << ((i - 1) % 8)
msig = ctx.bls_combine(use, multisig=True)
assert ctx.bls_verify_multisig(kid, cert.msg, msig, bytes(bitmap))
sid, sk, share = cert.sign_probe
assert ctx.bls_sign(sk, sid, cert.msg) == share, "signData differs from the expected share"
assert ctx.bls_public_key(sk) == cert.vks[sid - 1], "sk * g2 differs from the key set's vk"
for opt in (False, True):
    sig_t, ok_t, _ = ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=opt)
    assert ok_t and sig_t == cert.expected_sig, "combine_threshold differs"
out = {}
for name, fn in (("keyset_load", lambda: ctx.bls_unload_keys(ctx.bls_load_keys(cert.pk, cert.vks))),
                 ("keyset_load_1key", lambda: ctx.bls_unload_keys(ctx.bls_load_keys(cert.pk, []))),
                 ("share_verify", lambda: ctx.bls_verify_shares(kid, cert.msg, cert.shares)),
                 ("combine", lambda: ctx.bls_combine(use)),
                 ("verify", lambda: ctx.bls_verify(kid, cert.msg, comb)),
                 ("multisig_combine", lambda: ctx.bls_combine(use, multisig=True)),
                 ("multisig_verify", lambda: ctx.bls_verify_multisig(kid, cert.msg, msig, bytes(bitmap))),
                 ("certificate_fused", lambda: ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=False)),
                 ("certificate_policy", lambda: ctx.bls_combine_threshold(kid, cert.msg, cert.shares, optimistic=True)),
                 ("sign", lambda: ctx.bls_sign(cert.sign_probe[1], cert.sign_probe[0], cert.msg)),
                 ("public_key", lambda: ctx.bls_public_key(cert.sign_probe[1]))):
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    out[name + "_ms"] = min(ts)
print(json.dumps(out))
