"""Phase timing of the BLS kernels that print them (needs a library built with
-DCBFT_BLS_PHASES=1, selected by $CBFT_LIB): bls_verify_kernel, bls_verify_multisig_kernel and
block 0 of bls_msm_row_kernel on a config #4 certificate; the kernels' printf lines go to stdout."""
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
    use = cert.shares[:683]
    for _ in range(2):
        c = ctx.bls_combine(use)
    print("combine ok", c == comb, flush=True)
    bitmap = bytearray(256)
    for s in use:
        i = int.from_bytes(s[:4], "big")
        bitmap[(i - 1) // 8] |= 1 << ((i - 1) % 8)
    msig = ctx.bls_combine(use, multisig=True)
    for _ in range(3):
        ok = ctx.bls_verify_multisig(kid, cert.msg, msig, bytes(bitmap))
    print("multisig ok", ok, flush=True)
