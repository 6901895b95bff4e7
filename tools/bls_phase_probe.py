"""Phase timing of bls_verify_kernel (needs a library built with -DCBFT_BLS_PHASES=1, selected by
$CBFT_LIB): one verify of a config #4 combined signature; the kernel's printf lines go to stdout."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "concord-bft_amd"), os.path.join(ROOT, "tools")]
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

cert = workload.make_bls_cert(1024, 683, extra=0, bad_frac=0.0, seed=2024, threads=16)
with cb.Context(device=0) as ctx:
    kid = ctx.bls_load_keys(cert.pk, cert.vks)
    comb = cert.expected_sig
    for _ in range(3):
        ok = ctx.bls_verify(kid, cert.msg, comb)
    print("verify ok", ok, flush=True)
