import sys, os
sys.path[:0] = ["concord-bft_amd", "oracle", "tests"]
import bn254_ref as B, blsgen, cbft_hipcrypto as cb
n = 20
sk, sks, pk, vks = blsgen.keyset(n, n, seed=21)
ctx = cb.Context(device=0)
kid = ctx.bls_load_keys(pk, vks)
for ids in ([4], [1], [9], [1, 2], [1, 9], [2, 5, 9], list(range(1, 9)), list(range(1, 10)), [9, 10], [9, 17], list(range(1, 21))):
    acc = None
    for i in ids:
        acc = B.ec_add(acc, B.g2_from_bytes(vks[i - 1]), None)
    got = ctx.bls_sum_keys(kid, B.signers_bitmap(ids))
    print(ids[:6], got == B.g2_to_bytes(acc), got.hex()[:20], B.g2_to_bytes(acc).hex()[:20], flush=True)
