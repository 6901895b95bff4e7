"""GPU parity of the BLS BN-P254 path with RELIC's own bytes, pinned by the reference's
RELIC-generated key files (tests/golden/relic_bls_keys.json <- tests/simpleKVBC/scripts/
set{A,B}_replica_*), through the C ABI:

* sk_i * g2 computed on the GPU (cbft_bls_public_key) == the file's vk_i, byte for byte, 40/40;
* every vk and group key decodes on the GPU (key status) and re-encodes to the same bytes
  (sum over a one-signer bitmap = decode -> encode);
* multisig cryptosystems: sum of the vks == the file's group key (BlsMultisigVerifier.cpp:33-38);
* shares signed on the GPU with each file's secret share verify under the file's vk_i; the
  threshold combination of any `threshold` of them verifies under the file's group key and
  equals group_sk * H(m) (H = g1_map, RELIC-unpinned, from the oracle); multisig aggregates
  verify under the summed key and under the bitmap path.
"""
import pytest

import bn254_ref as B
import cbft_hipcrypto as cb
import relic_keys

pytestmark = pytest.mark.gpu
SYSTEMS = relic_keys.load()


@pytest.fixture(scope="module")
def ctx():
    c = cb.Context(device=0)
    yield c
    c.close()


def _bitmap(ids):
    b = bytearray(256)
    for i in ids:
        b[(i - 1) // 8] |= 1 << ((i - 1) % 8)
    return bytes(b)


def test_public_keys_from_secret_shares(ctx):
    n = 0
    for s in SYSTEMS:
        for i, sk in s.sks.items():
            assert ctx.bls_public_key(sk) == s.vks[i - 1], f"{s.name} vk_{i}"
            n += 1
    assert n == 40


@pytest.mark.parametrize("s", SYSTEMS, ids=lambda s: s.name)
def test_decode_encode_and_key_algebra(ctx, s):
    kid = ctx.bls_load_keys(s.pk, s.vks)
    try:
        assert all(ctx.bls_key_status(kid, s.n)), "a RELIC key failed to decode on the GPU"
        for i in range(1, s.n + 1):
            assert ctx.bls_sum_keys(kid, _bitmap([i])) == s.vks[i - 1]
        if s.multisig:
            assert ctx.bls_sum_keys(kid, _bitmap(range(1, s.n + 1))) == s.pk
    finally:
        ctx.bls_unload_keys(kid)


@pytest.mark.parametrize("s", SYSTEMS, ids=lambda s: s.name)
def test_sign_verify_combine_under_relic_keys(ctx, s):
    msg = bytes((7 * len(s.name) + i) & 0xFF for i in range(32))
    shares = [ctx.bls_sign(s.sks[i], i, msg) for i in range(1, s.n + 1)]
    for i, sh in enumerate(shares, 1):
        assert sh == B.sign_share(s.sks[i], i, msg)
    bad = shares[0][:4] + B.g1_to_bytes(B.ec_mul(2, B.parse_share(shares[0])[1]))  # Double()
    kid = ctx.bls_load_keys(s.pk, s.vks)
    try:
        v = ctx.bls_verify_shares(kid, msg, shares + [bad])
        assert v.tolist() == [True] * s.n + [False]
        expected = B.g1_to_bytes(B.ec_mul(s.group_secret(), B.g1_map(msg)))
        if s.multisig:
            agg = ctx.bls_combine(shares, multisig=True)
            assert agg == expected
            assert ctx.bls_verify_multisig(kid, msg, agg, _bitmap(range(1, s.n + 1)))
            assert ctx.bls_verify(kid, msg, agg)  # the file's group key is the n-of-n key
        else:
            for lo in range(0, s.n - s.threshold + 1):
                sub = shares[lo:lo + s.threshold]
                comb = ctx.bls_combine(sub)
                assert comb == expected
                assert ctx.bls_verify(kid, msg, comb)
            assert not ctx.bls_verify(kid, msg[::-1], expected)
    finally:
        ctx.bls_unload_keys(kid)
