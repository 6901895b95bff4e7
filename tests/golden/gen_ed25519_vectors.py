#!/usr/bin/env python3
"""Generate tests/golden/ed25519_vectors.bin — golden Ed25519 verify vectors.

Ground truth: the container's OpenSSL 3.0.2 libcrypto (EVP_PKEY_new_raw_public_key(ED25519) +
EVP_DigestVerify, verdict = (rc == 1)), i.e. the library whose semantics the reference's verify
idiom binds (util/src/openssl_crypto.cpp:229-253).  Adversarial points are constructed with the
pure-Python restatement oracle/ed25519_ref.py; signing uses oracle/libcbft_oracle.so (RFC 8032
§5.1.6) and the generator asserts that OpenSSL accepts every honest signature.

Record format (little-endian), after the 16-byte header b"CBFTED25519V1\\0\\0\\0" + u32 count:
    u32 msg_len | u8 verdict | u8 class | u16 0 | pk[32] | sig[64] | msg[msg_len]
Run:  python3 tests/golden/gen_ed25519_vectors.py   (needs libcrypto.so.3 and `make oracle`)
"""
from __future__ import annotations

import ctypes
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ed25519_ref as E  # noqa: E402

CLASSES = {
    "rfc8032": 0, "valid": 1, "flip_r": 2, "flip_s": 3, "s_plus_l": 4, "s_high_bits": 5,
    "flip_msg": 6, "wrong_key": 7, "small_order_a": 8, "noncanon_a": 9, "noncanon_r": 10,
    "offcurve_a": 11, "mixed_order_a": 12, "flip_a": 13, "long_msg": 14,
}

RFC8032 = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


class OpenSSL:
    NID_ED25519 = 1087

    def __init__(self):
        self.lib = ctypes.CDLL("libcrypto.so.3")
        L = self.lib
        L.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
        L.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.EVP_MD_CTX_new.restype = ctypes.c_void_p
        L.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        L.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        L.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t]

    def verify(self, pk: bytes, msg: bytes, sig: bytes) -> int:
        L = self.lib
        key = L.EVP_PKEY_new_raw_public_key(self.NID_ED25519, None, pk, 32)
        assert key, "raw public key rejected"
        ctx = L.EVP_MD_CTX_new()
        try:
            assert L.EVP_DigestVerifyInit(ctx, None, None, None, key) == 1
            rc = L.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg))
            return 1 if rc == 1 else 0
        finally:
            L.EVP_MD_CTX_free(ctx)
            L.EVP_PKEY_free(key)


class Signer:
    def __init__(self):
        self.lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "libcbft_oracle.so"))

    def pk(self, sk: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.cbft_oracle_ed25519_pubkey(sk, out)
        return out.raw

    def sign(self, sk: bytes, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.cbft_oracle_ed25519_sign(sk, msg, ctypes.c_size_t(len(msg)), out)
        return out.raw


def flip(b: bytes, bit: int) -> bytes:
    a = bytearray(b)
    a[bit // 8] ^= 1 << (bit % 8)
    return bytes(a)


def le(x: int) -> bytes:
    return int.to_bytes(x, 32, "little")


def main():
    rng = random.Random(0xC0FFEE)
    ossl, signer = OpenSSL(), Signer()
    recs = []

    def add(cls, pk, msg, sig):
        v = ossl.verify(pk, msg, sig)
        recs.append((CLASSES[cls], v, pk, sig, msg))
        return v

    # RFC 8032 7.1 tests 1-3
    for sk, pk, msg, sig in RFC8032:
        assert signer.pk(bytes.fromhex(sk)).hex() == pk
        assert add("rfc8032", bytes.fromhex(pk), bytes.fromhex(msg), bytes.fromhex(sig)) == 1

    keys = []
    for i in range(24):
        sk = rng.randbytes(32)
        keys.append((sk, signer.pk(sk)))

    # honest signatures over SHA-512 block boundaries (64 + m + 17 vs 128 k)
    lengths = [0, 1, 2, 7, 8, 31, 32, 46, 47, 48, 49, 63, 64, 65, 111, 112, 113, 127, 128, 129, 174, 175, 176,
               177, 255, 256, 257, 302, 303, 304, 511, 512, 1000]
    for m in lengths:
        for _ in range(3):
            sk, pk = rng.choice(keys)
            msg = rng.randbytes(m)
            assert add("valid", pk, msg, signer.sign(sk, msg)) == 1
    for m in [2048, 4095, 4096]:
        sk, pk = rng.choice(keys)
        msg = rng.randbytes(m)
        assert add("long_msg", pk, msg, signer.sign(sk, msg)) == 1

    # corruptions of honest signatures
    for _ in range(60):
        sk, pk = rng.choice(keys)
        msg = rng.randbytes(rng.randint(0, 300))
        sig = signer.sign(sk, msg)
        add("flip_r", pk, msg, flip(sig, rng.randrange(256)))
        add("flip_s", pk, msg, flip(sig, 256 + rng.randrange(256)))
        s = int.from_bytes(sig[32:], "little")
        add("s_plus_l", pk, msg, sig[:32] + le(s + E.L))
        hi = bytearray(sig)
        hi[63] |= rng.choice([0x20, 0x40, 0x80, 0xe0])
        add("s_high_bits", pk, msg, bytes(hi))
        if msg:
            add("flip_msg", pk, flip(msg, rng.randrange(8 * len(msg))), sig)
        else:
            add("flip_msg", pk, b"\x00", sig)
        other = rng.choice([k for k in keys if k[1] != pk])[1]
        add("wrong_key", other, msg, sig)
        add("flip_a", flip(pk, rng.randrange(256)), msg, sig)

    # small-order A, canonical and non-canonical encodings
    so = E.small_order_points()
    enc = set()
    for p in so:
        e = E.encode_point(p)
        enc.add(e)
        enc.add(e[:31] + bytes([e[31] ^ 0x80]))  # other sign bit (x = 0 stays 0)
    # y >= p encodings: y = p + k, k = 0..18 (only these fit under 2^255)
    noncanon = []
    for k in range(19):
        y = E.P + k
        for sgn in (0, 1):
            noncanon.append(int.to_bytes(y | (sgn << 255), 32, "little"))
    ident = E.encode_point(E.IDENTITY)
    for a_enc in sorted(enc):
        for _ in range(6):
            msg = rng.randbytes(rng.randint(0, 64))
            add("small_order_a", a_enc, msg, ident + le(0))
            R = E.encode_point(rng.choice(so))
            add("small_order_a", a_enc, msg, R + le(0))
    # small-order A with nonzero S: pick S, guess j, R = [S]B - [j]A until h = j (mod ord A)
    for p in so[1:]:
        a_enc = E.encode_point(p)
        order = E.point_order_small(p)
        for _ in range(4):
            msg = rng.randbytes(rng.randint(0, 40))
            s = rng.randrange(E.L)
            for _try in range(200):
                j = rng.randrange(order)
                R = E.encode_point(E.point_add(E.scalar_mult(s, E.B), E.point_neg(E.scalar_mult(j, p))))
                h = E.sha512_modl(R, a_enc, msg)
                if h % order == j:
                    break
            add("small_order_a", a_enc, msg, R + le(s))
    for a_enc in noncanon:
        for _ in range(3):
            msg = rng.randbytes(rng.randint(0, 40))
            add("noncanon_a", a_enc, msg, ident + le(0))
            R = E.encode_point(rng.choice(so))
            add("noncanon_a", a_enc, msg, R + le(0))
        sk, pk = rng.choice(keys)
        msg = rng.randbytes(20)
        add("noncanon_a", a_enc, msg, signer.sign(sk, msg))

    # non-canonical R: identity as y = p + 1, identity with sign bit, y = p (order-4 point)
    for a_enc in sorted(enc):
        for r_enc in noncanon[:6] + [ident[:31] + b"\x80"]:
            msg = rng.randbytes(rng.randint(0, 40))
            add("noncanon_r", a_enc, msg, r_enc + le(0))

    # off-curve A: y values with no x
    off = 0
    y = 2
    while off < 40:
        if E.decode_point(le(y)) is None:
            msg = rng.randbytes(16)
            add("offcurve_a", le(y), msg, ident + le(0))
            sk, pk = rng.choice(keys)
            add("offcurve_a", le(y | (1 << 255)), msg, signer.sign(sk, msg))
            off += 1
        y += 1

    # mixed-order A = aB + T: "honest" signer with secret a; accept iff [h]T = 0
    for t in so[1:]:
        for _ in range(8):
            a = rng.randrange(1, E.L)
            Apt = E.point_add(E.scalar_mult(a, E.B), t)
            a_enc = E.encode_point(Apt)
            msg = rng.randbytes(rng.randint(0, 64))
            r = rng.randrange(1, E.L)
            R = E.encode_point(E.scalar_mult(r, E.B))
            h = E.sha512_modl(R, a_enc, msg)
            s = (r + h * a) % E.L
            add("mixed_order_a", a_enc, msg, R + le(s))

    out = os.path.join(HERE, "ed25519_vectors.bin")
    with open(out, "wb") as f:
        f.write(b"CBFTED25519V1\0\0\0" + struct.pack("<I", len(recs)))
        for cls, v, pk, sig, msg in recs:
            assert len(pk) == 32 and len(sig) == 64
            f.write(struct.pack("<IBBH", len(msg), v, cls, 0) + pk + sig + msg)
    acc = sum(r[1] for r in recs)
    print(f"wrote {len(recs)} vectors ({acc} accept, {len(recs) - acc} reject) -> {out}")
    by = {}
    for cls, v, *_ in recs:
        name = [k for k, c in CLASSES.items() if c == cls][0]
        by.setdefault(name, [0, 0])[v] += 1
    for k, (rej, ac) in sorted(by.items()):
        print(f"  {k:15s} accept {ac:4d} reject {rej:4d}")


if __name__ == "__main__":
    main()
