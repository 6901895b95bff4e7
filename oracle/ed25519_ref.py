"""Ed25519 CPU restatement — TEST INFRASTRUCTURE ONLY (the oracle / checker).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is never on the product path.

What it restates
----------------
The reference snapshot (vmware/concord-bft) contains no Ed25519 code.
The verify semantics the product must reproduce are those of the third-party library the
reference's crypto idiom binds: OpenSSL 3.0.2 (15 Mar 2022) ``EVP_DigestVerify`` with
``EVP_PKEY_ED25519`` (its ``ossl_ed25519_verify`` in crypto/ec/curve25519.c), called the way
the reference calls OpenSSL verifiers (``util/src/openssl_crypto.cpp:229-253``: success only
when the return value is exactly 1).  The published algorithm (RFC 8032 §5.1.7, cofactorless
variant as OpenSSL implements it) is restated here in plain Python integers:

1. ``len(sig) == 64``  (EVP layer; IVerifier::signatureLength, crypto_utils.hpp:44)
2. ``S < L``  (strict, canonical S; S >= L rejected)
3. decode A: y = low 255 bits taken **mod p without a canonicity check** (y >= p accepted),
   x recovered by the (p+3)/8 square root, sign bit applied by negation (so x = 0 with the
   sign bit set is accepted), off-curve y rejected
4. ``h = SHA-512(R || A_bytes || M) mod L``  (A_bytes = the 32 key bytes as given)
5. ``R' = [S]B - [h]A``  (cofactorless: no multiplication by 8)
6. accept iff ``encode(R') == R`` byte for byte (so a non-canonical R never matches)

Pinned by ``tests/golden/ed25519_vectors.bin`` (verdicts computed by the container's
OpenSSL 3.0.2 via ctypes, generator ``tests/golden/gen_ed25519_vectors.py``) and by the
RFC 8032 test vectors 1-3.

Pure-Python big-int arithmetic: small cases only (~ms per verify).
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Base point B (RFC 8032 §5.1): y = 4/5, x positive (even).
_BY = (4 * pow(5, P - 2, P)) % P


def _recover_x(y: int, sign: int):
    """x from y per RFC 8032 §5.1.3 step 2-4, OpenSSL flavour (no x==0&&sign reject)."""
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = (u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P)) % P
    vxx = (v * x * x) % P
    if vxx != u:
        if vxx != (-u) % P:
            return None
        x = (x * SQRT_M1) % P
    if (x & 1) != sign:
        x = (-x) % P  # x == 0 stays 0: accepted (OpenSSL does not reject)
    return x


_BX = _recover_x(_BY, 0)
# Extended twisted-Edwards coordinates (X, Y, Z, T) with x = X/Z, y = Y/Z, xy = T/Z.
B = (_BX, _BY, 1, (_BX * _BY) % P)
IDENTITY = (0, 1, 1, 0)


def point_add(p1, p2):
    """Unified addition on -x^2 + y^2 = 1 + d x^2 y^2 (RFC 8032 §5.1.4 formulas)."""
    x1, y1, z1, t1 = p1
    x2, y2, z2, t2 = p2
    a = ((y1 - x1) * (y2 - x2)) % P
    b = ((y1 + x1) * (y2 + x2)) % P
    c = (2 * t1 * t2 * D) % P
    d = (2 * z1 * z2) % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return ((e * f) % P, (g * h) % P, (f * g) % P, (e * h) % P)


def point_neg(pt):
    x, y, z, t = pt
    return ((-x) % P, y, z, (-t) % P)


def scalar_mult(k: int, pt):
    q = IDENTITY
    while k > 0:
        if k & 1:
            q = point_add(q, pt)
        pt = point_add(pt, pt)
        k >>= 1
    return q


def point_equal(p1, p2) -> bool:
    x1, y1, z1, _ = p1
    x2, y2, z2, _ = p2
    return (x1 * z2 - x2 * z1) % P == 0 and (y1 * z2 - y2 * z1) % P == 0


def encode_point(pt) -> bytes:
    x, y, z, _ = pt
    zi = pow(z, P - 2, P)
    x = (x * zi) % P
    y = (y * zi) % P
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


def decode_point(s: bytes):
    """OpenSSL ge_frombytes_vartime semantics: y is NOT required to be < p."""
    if len(s) != 32:
        return None
    v = int.from_bytes(s, "little")
    sign = v >> 255
    y = (v & ((1 << 255) - 1)) % P
    x = _recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, (x * y) % P)


def sha512_modl(*parts: bytes) -> int:
    h = hashlib.sha512()
    for p in parts:
        h.update(p)
    return int.from_bytes(h.digest(), "little") % L


def secret_expand(sk: bytes):
    h = hashlib.sha512(sk).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def public_key(sk: bytes) -> bytes:
    a, _ = secret_expand(sk)
    return encode_point(scalar_mult(a, B))


def sign(sk: bytes, msg: bytes) -> bytes:
    a, prefix = secret_expand(sk)
    A = encode_point(scalar_mult(a, B))
    r = sha512_modl(prefix, msg)
    Rs = encode_point(scalar_mult(r, B))
    h = sha512_modl(Rs, A, msg)
    s = (r + h * a) % L
    return Rs + int.to_bytes(s, 32, "little")


def verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    """Accept/reject exactly as OpenSSL 3.0.2 EVP_DigestVerify(ED25519) == 1."""
    if len(sig) != 64 or len(pk) != 32:
        return False
    Rs, Sb = sig[:32], sig[32:]
    s = int.from_bytes(Sb, "little")
    if s >= L:
        return False
    A = decode_point(pk)
    if A is None:
        return False
    h = sha512_modl(Rs, pk, msg)
    Rp = point_add(scalar_mult(s, B), point_neg(scalar_mult(h, A)))
    return encode_point(Rp) == Rs


# ---- helpers for constructing adversarial fixtures (generator + tests only) ----

def small_order_points():
    """The 8 torsion points E[8] as extended coordinates (identity first)."""
    pts = [IDENTITY]
    # order-2: (0, -1); order-4: (+-sqrt(-1)... ) found by decoding known y values
    cands = []
    y2 = P - 1  # (0,-1)
    cands.append(decode_point(int.to_bytes(y2, 32, "little")))
    # order-4 points: y = 0, x = +-1/sqrt(a)=... ; decode y=0 both signs
    cands.append(decode_point(bytes(32)))
    cands.append(decode_point(bytes(31) + b"\x80"))
    # order-8 points: y^2 = ... solve via known encoding c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a
    o8 = bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a")
    t = decode_point(o8)
    for k in range(1, 8):
        cands.append(scalar_mult(k, t))
    for c in cands:
        if c is None:
            continue
        if not any(point_equal(c, q) for q in pts):
            pts.append(c)
    return pts


def point_order_small(pt) -> int:
    q = pt
    for k in range(1, 9):
        if point_equal(q, IDENTITY):
            return k
        q = point_add(q, pt)
    return 0
