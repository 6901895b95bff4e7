"""BN-P254 (RELIC's "BN_P254") BLS restatement in pure Python — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

PARITY UNPINNED at the RELIC boundary: RELIC @ 0998bfcb is not available
offline, so its byte-level conventions cannot be checked.  What this file fixes, and how:

* curve constants: u = -(2^62 + 2^55 + 1), p = 36u^4+36u^3+24u^2+6u+1, r = 36u^4+36u^3+18u^2+6u+1,
  E: y^2 = x^3 + 2, G1 generator (-1, 1) (SURVEY.md §8(a) "Curve constants");
* towers: Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + i
  (the Beuchat et al. 2010 BN254 tower RELIC's BN_P254 uses);
* G2 = D-type sextic twist E': y^2 = x^3 + 2/xi = x^3 + (1 - i), generator G2_GEN below
  (checked here: on E', order r);
* g1_map(msg) (RELIC 2019-era ep_map): k = SHA-256(msg) as a big-endian integer, x = k mod p,
  try-and-increment x until x^3 + 2 is a square, y = (x^3+2)^((p+1)/4); cofactor 1;
* compressed encodings (ep_write_bin / ep2_write_bin with pack = 1):
  G1 = [0x02 | (y mod 2)] || x (32 B big-endian)  = 33 B;  infinity = 0x00 || 32 zero bytes;
  G2 = [0x02 | (y0 mod 2)] || x0 || x1 (2 x 32 B)  = 65 B;  infinity = 0x00 || zeros;
  decoding rejects x >= p, off-curve x and a G2 point outside the order-r subgroup.
* pairing: optimal ate e(P, Q) = (f_{6u+2,Q}(P) l_{T,pi(Q)}(P) l_{T+pi(Q),-pi^2(Q)}(P))^((p^12-1)/r).
  Accept/reject of every pairing check, the Lagrange coefficients and the combined signature
  sum(lambda_i sigma_i) = sk * H(m) are fixed by the mathematics (pinned by the identities in
  tests/test_bls_oracle.py); only hash-to-G1 and encodings are RELIC conventions, unpinned.

The threshold algorithms follow the reference call sites: lagrangeCoeffAccumReduced
(threshsign/src/bls/relic/LagrangeInterpolation.cpp:202-292), fastMultExp
(FastMultExp.cpp:26-59), BlsThresholdSigner::signData (BlsThresholdSigner.cpp:32-47),
BlsAccumulatorBase::verifyShare (BlsAccumulatorBase.cpp:62-84), BlsThresholdVerifier::verify
(BlsThresholdVerifier.cpp:69-96), BlsMultisigAccumulator / BlsMultisigVerifier
(BlsMultisigAccumulator.cpp:36-65, BlsMultisigVerifier.cpp:67-105), VectorOfShares::toBytes
(VectorOfShares.cpp:136-161).
"""
from __future__ import annotations

import hashlib

U = -(2**62 + 2**55 + 1)
P = 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1
R = 36 * U**4 + 36 * U**3 + 18 * U**2 + 6 * U + 1
B1 = 2
assert P == 0x2523648240000001BA344D80000000086121000000000013A700000000000013
assert R == 0x2523648240000001BA344D8000000007FF9F800000000010A10000000000000D


def inv(a: int) -> int:
    return pow(a, P - 2, P)


def fp_sqrt(a: int):
    """RELIC fp_srt for p = 3 (mod 4): y = a^((p+1)/4), None if a is not a square."""
    y = pow(a, (P + 1) // 4, P)
    return y if (y * y - a) % P == 0 else None


# ------------------------------------------------------------------------------------ Fp2
class F2:
    __slots__ = ("a", "b")  # a + b i, i^2 = -1

    def __init__(self, a, b=0):
        self.a, self.b = a % P, b % P

    def __add__(s, o):
        return F2(s.a + o.a, s.b + o.b)

    def __sub__(s, o):
        return F2(s.a - o.a, s.b - o.b)

    def __neg__(s):
        return F2(-s.a, -s.b)

    def __mul__(s, o):
        if isinstance(o, int):
            return F2(s.a * o, s.b * o)
        return F2(s.a * o.a - s.b * o.b, s.a * o.b + s.b * o.a)

    def __eq__(s, o):
        return s.a == o.a and s.b == o.b

    def iszero(s):
        return s.a == 0 and s.b == 0

    def inv(s):
        d = inv(s.a * s.a + s.b * s.b)
        return F2(s.a * d, -s.b * d)

    def __truediv__(s, o):
        return s * o.inv()

    def sq(s):
        return s * s

    def conj(s):
        return F2(s.a, -s.b)

    def pow(s, e):
        r, x = F2(1), s
        while e:
            if e & 1:
                r = r * x
            x = x * x
            e >>= 1
        return r

    def __repr__(s):
        return f"F2({hex(s.a)}, {hex(s.b)})"


XI = F2(1, 1)
B2 = F2(B1) / XI  # 2 / (1 + i) = 1 - i  (D-type twist)
assert B2 == F2(1, -1)


def f2_sqrt(a: F2):
    """Square root in Fp2 (p = 3 mod 4), None if a is not a square."""
    if a.iszero():
        return F2(0)
    a1 = a.pow((P - 3) // 4)
    alpha = a1 * a1 * a
    x0 = a1 * a
    if alpha == F2(-1):
        x = F2(0, 1) * x0
    else:
        b = (F2(1) + alpha).pow((P - 1) // 2)
        x = b * x0
    return x if x * x == a else None


# ------------------------------------------------------------------------------------ Fp12
# Fp12 = Fp[w]/(w^12 - 2 w^6 + 2): w^6 = xi = 1 + i, so i = w^6 - 1.  (Same field as the tower
# Fp2[v]/(v^3 - xi)[w]/(w^2 - v); the flat form keeps the oracle short.)
MOD12 = [2, 0, 0, 0, 0, 0, -2, 0, 0, 0, 0, 0]  # w^12 = 2 w^6 - 2


class F12:
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = [x % P for x in c]

    @staticmethod
    def one():
        return F12([1] + [0] * 11)

    @staticmethod
    def _reduce(t):
        t = list(t)
        for d in range(len(t) - 1, 11, -1):
            if t[d]:
                v = t[d]
                t[d] = 0
                # w^d = w^(d-12) * (2 w^6 - 2)
                t[d - 6] += 2 * v
                t[d - 12] -= 2 * v
        return F12(t[:12])

    def __add__(s, o):
        return F12([x + y for x, y in zip(s.c, o.c)])

    def __sub__(s, o):
        return F12([x - y for x, y in zip(s.c, o.c)])

    def __neg__(s):
        return F12([-x for x in s.c])

    def __mul__(s, o):
        if isinstance(o, int):
            return F12([x * o for x in s.c])
        t = [0] * 23
        for i, x in enumerate(s.c):
            if x:
                for j, y in enumerate(o.c):
                    t[i + j] += x * y
        return F12._reduce(t)

    def __eq__(s, o):
        return s.c == o.c

    def pow(s, e):
        r, x = F12.one(), s
        while e:
            if e & 1:
                r = r * x
            x = x * x
            e >>= 1
        return r

    def inv(s):
        """Extended Euclid on Fp[w] modulo w^12 - 2 w^6 + 2."""
        def deg(a):
            d = len(a) - 1
            while d >= 0 and a[d] % P == 0:
                d -= 1
            return d

        def trim(a):
            a = [x % P for x in a]
            while a and a[-1] == 0:
                a.pop()
            return a

        r0 = trim([2, 0, 0, 0, 0, 0, -2, 0, 0, 0, 0, 0, 1])
        r1 = trim(list(s.c))
        t0, t1 = [], [1]
        while r1:
            q = [0] * max(1, len(r0) - len(r1) + 1)
            rr = list(r0)
            il = pow(r1[-1], P - 2, P)
            while len(rr) >= len(r1) and rr:
                c = rr[-1] * il % P
                k = len(rr) - len(r1)
                q[k] = c
                for j, x in enumerate(r1):
                    rr[j + k] = (rr[j + k] - c * x) % P
                rr = trim(rr)
            # t2 = t0 - q t1
            prod = [0] * (len(q) + len(t1))
            for i, x in enumerate(q):
                for j, y in enumerate(t1):
                    prod[i + j] += x * y
            t2 = [0] * max(len(t0), len(prod))
            for i, x in enumerate(t0):
                t2[i] += x
            for i, x in enumerate(prod):
                t2[i] -= x
            r0, r1, t0, t1 = r1, rr, t1, trim(t2)
        assert len(r0) == 1, "not invertible"
        c = pow(r0[0], P - 2, P)
        out = [x * c for x in t0] + [0] * 12
        return F12._reduce(out)

    def __truediv__(s, o):
        return s * o.inv()

    def frob(s):
        return s.pow(P)

    def conj(s):  # s^(p^6): w^(p^6) = -w
        return F12([x if k % 2 == 0 else -x for k, x in enumerate(s.c)])


def f2_to_f12(x: F2) -> F12:
    c = [0] * 12
    c[0] = x.a - x.b
    c[6] = x.b
    return F12(c)


W = F12([0, 1] + [0] * 10)
W2 = W * W
W3 = W2 * W


# ------------------------------------------------------------------------------------ curves
INF = None


def ec_add(p1, p2, zero):
    """Affine addition on y^2 = x^3 + b over any of Fp(int)/F2/F12 (None = infinity)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if _eq(x1, x2):
        if _eq(y1, _neg(y2)):
            return None
        lam = _div(_mulc(_sq(x1), 3), _mulc(y1, 2))
    else:
        lam = _div(_sub(y2, y1), _sub(x2, x1))
    x3 = _sub(_sub(_sq(lam), x1), x2)
    y3 = _sub(_mul(lam, _sub(x1, x3)), y1)
    return (x3, y3)


def _isint(x):
    return isinstance(x, int)


def _eq(a, b):
    return (a - b) % P == 0 if _isint(a) else a == b


def _neg(a):
    return (-a) % P if _isint(a) else -a


def _sub(a, b):
    return (a - b) % P if _isint(a) else a - b


def _mul(a, b):
    return (a * b) % P if _isint(a) else a * b


def _mulc(a, k):
    return (a * k) % P if _isint(a) else a * k


def _sq(a):
    return _mul(a, a)


def _div(a, b):
    if _isint(a):
        return a * inv(b) % P
    return a / b


def ec_mul(k: int, pt, zero=None):
    if k < 0:
        return ec_mul(-k, ec_neg(pt))
    acc = None
    while k:
        if k & 1:
            acc = ec_add(acc, pt, zero)
        pt = ec_add(pt, pt, zero)
        k >>= 1
    return acc


def ec_neg(pt):
    if pt is None:
        return None
    return (pt[0], _neg(pt[1]))


G1_GEN = (P - 1, 1)
G2_GEN = (F2(0x061A10BB519EB62FEB8D8C7E8C61EDB6A4648BBB4898BF0D91EE4224C803FB2B,
             0x0516AAF9BA737833310AA78C5982AA5B1F4D746BAE3784B70D8C34C1E7D54CF3),
          F2(0x021897A06BAF93439A90E096698C822329BD0AE6BDBE09BD19F0E07891CD2B9A,
             0x0EBB2B0E7C8B15268F6D4456F5F38D37B09006FFD739C9578A2D1AEC6B3ACE9B))


def g1_on_curve(pt) -> bool:
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt) -> bool:
    x, y = pt
    return y * y == x * x * x + B2


# ------------------------------------------------------------------------------------ pairing
def untwist(q):
    """E'(Fp2) -> E(Fp12): (x, y) -> (x w^2, y w^3) (D-type: w^6 = xi, b' = b/xi)."""
    x, y = q
    return (f2_to_f12(x) * W2, f2_to_f12(y) * W3)


def _line(a, b, p):
    """l_{A,B}(P) for A, B in E(Fp12) (affine), P = (xp, yp) with Fp coordinates."""
    xp, yp = F12([p[0]] + [0] * 11), F12([p[1]] + [0] * 11)
    x1, y1 = a
    x2, y2 = b
    if x1 == x2 and y1 == y2:
        lam = (x1 * x1 * 3) / (y1 * 2)
    elif x1 == x2:
        return xp - x1
    else:
        lam = (y2 - y1) / (x2 - x1)
    return yp - y1 - lam * (xp - x1)


ATE = 6 * U + 2
GX1 = XI.pow((P - 1) // 3)       # Frobenius twist constants: pi(psi(x, y)) = psi(conj(x) gx, conj(y) gy)
GY1 = XI.pow((P - 1) // 2)
GX2 = XI.pow((P * P - 1) // 3)
GY2 = XI.pow((P * P - 1) // 2)


def _tline(t, q, p):
    """Line through T, Q in E'(Fp2) evaluated at P, as an element of Fp12 (D-type twist:
    the slope on E(Fp12) is lambda' w, so l(P) = yP - lambda' xP w + (lambda' x_T - y_T) w^3);
    also returns T + Q."""
    xt, yt = t
    xq, yq = q
    if xt == xq and yt == yq:
        lam = xt * xt * 3 / (yt * 2)
    elif xt == xq:
        return F12([p[0]] + [0] * 11) - f2_to_f12(xt) * W2, None
    else:
        lam = (yq - yt) / (xq - xt)
    x3 = lam * lam - xt - xq
    y3 = lam * (xt - x3) - yt
    l = F12([p[1]] + [0] * 11) + f2_to_f12(lam * (-p[0])) * W + f2_to_f12(lam * xt - yt) * W3
    return l, (x3, y3)


def miller(p, q):
    """f_{6u+2,Q}(P) * l_{T,pi(Q)}(P) * l_{T+pi(Q),-pi^2(Q)}(P) (optimal ate for BN), with T on
    the twist; equals the same loop on psi(Q) in E(Fp12)."""
    if p is None or q is None:
        return F12.one()
    m = abs(ATE)
    T = q
    f = F12.one()
    for bit in bin(m)[3:]:
        l, T = _tline(T, T, p)
        f = f * f * l
        if bit == "1":
            l, T = _tline(T, q, p)
            f = f * l
    if ATE < 0:
        f = f.conj()
        T = (T[0], -T[1])
    q1 = (q[0].conj() * GX1, q[1].conj() * GY1)
    q2 = (q[0] * GX2, q[1] * GY2)
    l, T = _tline(T, q1, p)
    f = f * l
    l, T = _tline(T, (q2[0], -q2[1]), p)
    return f * l


FINAL_EXP = (P**12 - 1) // R


def final_exp(f: F12) -> F12:
    # easy part (p^6 - 1)(p^2 + 1), then the hard part (p^4 - p^2 + 1)/r
    f = f.conj() / f
    f = f.pow(P * P) * f
    return f.pow((P**4 - P**2 + 1) // R)


def pairing(p, q) -> F12:
    return final_exp(miller(p, q))


def pairing_check(pairs) -> bool:
    """prod e(P_i, Q_i) == 1 (one shared final exponentiation)."""
    f = F12.one()
    for p, q in pairs:
        f = f * miller(p, q)
    return final_exp(f) == F12.one()


# ------------------------------------------------------------------------------------ codecs
# RELIC keeps Fp elements in Montgomery form (R = 2^256: FP_PRIME = 254 on 4 x 64-bit digits)
# and its compressed encodings take the y "parity" with fp_get_bit(y, 0) on that raw form
# (ep_write_bin / ep2_write_bin with pack = 1, called from BlsNumTypes.cpp:216-243): the prefix
# bit is lsb(y * 2^256 mod p), not lsb(y).  Pinned for G2 by the reference's own RELIC-generated
# key files (tests/simpleKVBC/scripts/set{A,B}_replica_*: sk * g2 == vk byte for byte, 40/40;
# tests/golden/relic_bls_keys.json); G1 uses the same fp_get_bit rule (ep_write_bin), inferred.
MONT_R = pow(2, 256, P)


def relic_bit(y: int) -> int:
    return ((y * MONT_R) % P) & 1


def g1_to_bytes(pt) -> bytes:
    if pt is None:
        return bytes(33)
    x, y = pt
    return bytes([2 | relic_bit(y)]) + x.to_bytes(32, "big")


def g1_from_bytes(b: bytes):
    """Returns the point, None for infinity, raises ValueError on an invalid encoding."""
    if len(b) != 33:
        raise ValueError("G1 encoding must be 33 bytes")
    if b[0] == 0:
        if any(b[1:]):
            raise ValueError("bad infinity")
        return None
    if b[0] not in (2, 3):
        raise ValueError("bad prefix")
    x = int.from_bytes(b[1:], "big")
    if x >= P:
        raise ValueError("x >= p")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise ValueError("not on curve")
    if relic_bit(y) != (b[0] & 1):
        y = P - y
    return (x, y)


def g2_to_bytes(pt) -> bytes:
    if pt is None:
        return bytes(65)
    x, y = pt
    return bytes([2 | relic_bit(y.a)]) + x.a.to_bytes(32, "big") + x.b.to_bytes(32, "big")


def g2_from_bytes(b: bytes):
    if len(b) != 65:
        raise ValueError("G2 encoding must be 65 bytes")
    if b[0] == 0:
        if any(b[1:]):
            raise ValueError("bad infinity")
        return None
    if b[0] not in (2, 3):
        raise ValueError("bad prefix")
    x0, x1 = int.from_bytes(b[1:33], "big"), int.from_bytes(b[33:], "big")
    if x0 >= P or x1 >= P:
        raise ValueError("x >= p")
    x = F2(x0, x1)
    y = f2_sqrt(x * x * x + B2)
    if y is None:
        raise ValueError("not on curve")
    if relic_bit(y.a) != (b[0] & 1):
        y = -y
    pt = (x, y)
    if ec_mul(R, pt) is not None:
        raise ValueError("not in G2")
    return pt


# ------------------------------------------------------------------------------------ BLS
def g1_map(msg: bytes):
    """RELIC 2019-era ep_map: SHA-256, x = digest mod p, try-and-increment, y = t^((p+1)/4)."""
    x = int.from_bytes(hashlib.sha256(msg).digest(), "big") % P
    while True:
        t = (x * x * x + B1) % P
        y = fp_sqrt(t)
        if y is not None:
            return (x, y)
        x = (x + 1) % P


def sign_share(sk: int, share_id: int, digest: bytes) -> bytes:
    """BlsThresholdSigner::signData: 4-byte big-endian id || G1 compressed (37 B)."""
    return share_id.to_bytes(4, "big") + g1_to_bytes(ec_mul(sk, g1_map(digest)))


def parse_share(b: bytes):
    """BlsSigshareParser (BlsAccumulatorBase.cpp:33-43)."""
    return int.from_bytes(b[:4], "big"), g1_from_bytes(b[4:])


def verify_share(H, sigma, vk) -> bool:
    """e(H, vk) == e(sigma, g2)  <=>  e(H, vk) * e(-sigma, g2) == 1."""
    return pairing_check([(H, vk), (ec_neg(sigma), G2_GEN)])


def verify(msg: bytes, sig33: bytes, pk) -> bool:
    """BlsThresholdVerifier::verify(msg, sig)."""
    try:
        s = g1_from_bytes(sig33)
    except ValueError:
        return False
    return verify_share(g1_map(msg), s, pk)


def lagrange_coeffs(ids):
    """lambda_i = prod_{j != i} j / (j - i) mod r (unique; LagrangeInterpolation.cpp:202-292)."""
    out = {}
    for i in ids:
        num, den = 1, 1
        for j in ids:
            if j != i:
                num = num * j % R
                den = den * (j - i) % R
        out[i] = num * pow(den, R - 2, R) % R
    return out


def combine_threshold(shares: dict):
    """sum lambda_i sigma_i over the signer set (BlsThresholdAccumulator)."""
    lam = lagrange_coeffs(sorted(shares))
    acc = None
    for i, s in shares.items():
        acc = ec_add(acc, ec_mul(lam[i], s), None)
    return acc


def signers_bitmap(ids, max_shares: int = 2048) -> bytes:
    """VectorOfShares::toBytes: bit (id-1), LSB-first, 256 bytes."""
    b = bytearray(max_shares // 8)
    for i in ids:
        b[(i - 1) // 8] |= 1 << ((i - 1) % 8)
    return bytes(b)


def keygen(n: int, k: int, seed: int):
    """Shamir sharing of a random sk with a degree-(k-1) polynomial (BlsThresholdKeygen):
    sk_i = f(i), vk_i = sk_i * g2, pk = sk * g2."""
    import random

    rng = random.Random(seed)
    coeffs = [rng.randrange(1, R) for _ in range(k)]

    def f(x):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R
        return acc

    sks = {i: f(i) for i in range(1, n + 1)}
    return coeffs[0], sks
