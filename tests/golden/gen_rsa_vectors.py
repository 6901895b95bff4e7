#!/usr/bin/env python3
"""Generate tests/golden/rsa_vectors.json — golden RSA-2048 PKCS#1 v1.5 / SHA-256 verify vectors.

The reference verifies replica and client signatures with Crypto++ 8.2.0
RSASS<PKCS1v15, SHA256> (util/src/crypto_utils.cpp:101-117,166).  Crypto++
is absent here, so verdicts are pinned against the container's OpenSSL 3.0.2 libcrypto
(EVP_DigestVerify, RSA_PKCS1_PADDING, SHA-256; accept iff rc == 1), which agrees with Crypto++ on
every signature of exactly modulus length with s < n.  Each vector carries both:
    "openssl": OpenSSL 3.0.2's verdict (ground truth, ctypes)
    "verdict": the reference's (Crypto++) verdict = oracle/rsa_ref.verify; equal to "openssl"
               except for the "s_plus_n" class (s >= n: Crypto++ reduces s mod n, OpenSSL
               rejects) — that difference is parity unpinned and flagged "pinned": false.

Keys: the reference's own replica test key (bftengine/tests/messages/helper.cpp:16-49, hex DER
PKCS#8 / X.509, e = 17) plus keys made here with `openssl genpkey` (e = 3, 17, 65537 x 2 and a
large odd 32-bit e).  Honest signatures come from OpenSSL EVP_DigestSign; malformed encodings
(wrong block type, missing separator, SHA-1 / parameter-less DigestInfo, ...) are forged with the
private exponent through oracle/rsa_ref.py.
Run:  python3 tests/golden/gen_rsa_vectors.py   (needs libcrypto.so.3 and the openssl CLI)
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import random
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rsa_ref as R  # noqa: E402

REF_HELPER = "/root/reference/bftengine/tests/messages/helper.cpp"


class OpenSSL:
    def __init__(self):
        L = self.lib = ctypes.CDLL("libcrypto.so.3")
        vp, cp, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
        L.d2i_AutoPrivateKey.restype = vp
        L.d2i_AutoPrivateKey.argtypes = [vp, ctypes.POINTER(cp), ctypes.c_long]
        L.d2i_PUBKEY.restype = vp
        L.d2i_PUBKEY.argtypes = [vp, ctypes.POINTER(cp), ctypes.c_long]
        L.i2d_PUBKEY.restype = ctypes.c_int
        L.i2d_PUBKEY.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p)]
        L.EVP_sha256.restype = vp
        L.EVP_MD_CTX_new.restype = vp
        L.EVP_MD_CTX_free.argtypes = [vp]
        L.EVP_PKEY_free.argtypes = [vp]
        L.EVP_DigestSignInit.argtypes = [vp, vp, vp, vp, vp]
        L.EVP_DigestSign.argtypes = [vp, cp, ctypes.POINTER(sz), cp, sz]
        L.EVP_DigestVerifyInit.argtypes = [vp, vp, vp, vp, vp]
        L.EVP_DigestVerify.argtypes = [vp, cp, sz, cp, sz]
        L.CRYPTO_free.argtypes = [vp, cp, ctypes.c_int]

    def priv(self, der: bytes):
        p = ctypes.c_char_p(der)
        k = self.lib.d2i_AutoPrivateKey(None, ctypes.byref(p), len(der))
        assert k, "d2i_AutoPrivateKey"
        return k

    def pub(self, der: bytes):
        p = ctypes.c_char_p(der)
        k = self.lib.d2i_PUBKEY(None, ctypes.byref(p), len(der))
        assert k, "d2i_PUBKEY"
        return k

    def pub_der_of(self, pkey) -> bytes:
        out = ctypes.c_void_p()
        n = self.lib.i2d_PUBKEY(pkey, ctypes.byref(out))
        data = ctypes.string_at(out, n)
        self.lib.CRYPTO_free(out, b"", 0)
        return data

    def sign(self, pkey, msg: bytes) -> bytes:
        L = self.lib
        ctx = L.EVP_MD_CTX_new()
        assert L.EVP_DigestSignInit(ctx, None, L.EVP_sha256(), None, pkey) == 1
        buf = ctypes.create_string_buffer(1024)
        ln = ctypes.c_size_t(1024)
        assert L.EVP_DigestSign(ctx, buf, ctypes.byref(ln), msg, len(msg)) == 1
        L.EVP_MD_CTX_free(ctx)
        return buf.raw[:ln.value]

    def verify(self, pkey, msg: bytes, sig: bytes) -> int:
        L = self.lib
        ctx = L.EVP_MD_CTX_new()
        assert L.EVP_DigestVerifyInit(ctx, None, L.EVP_sha256(), None, pkey) == 1
        rc = L.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg))
        L.EVP_MD_CTX_free(ctx)
        return int(rc == 1)


def reference_key():
    """The replica key pair of bftengine/tests/messages/helper.cpp (hex DER strings)."""
    src = open(REF_HELPER).read()

    def hexblock(name):
        m = re.search(name + r"[^=]*=\s*\{?((?:\s*\"[0-9A-Fa-f]*\")+)", src)
        return bytes.fromhex("".join(re.findall(r"\"([0-9A-Fa-f]*)\"", m.group(1))))

    return hexblock("replicaPrivateKey"), hexblock("pubKey")


def gen_key(e: int) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.der")
        subprocess.run(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt", "rsa_keygen_bits:2048",
                        "-pkeyopt", f"rsa_keygen_pubexp:{e}", "-outform", "DER", "-out", out],
                       check=True, capture_output=True)
        return open(out, "rb").read()


def main():
    rng = random.Random(0xC0FFEE)
    ossl = OpenSSL()
    priv_ref, pub_ref = reference_key()
    keys = []  # (n, e, d, openssl private handle, openssl public handle, source)
    n, e, d = R.parse_pkcs8_der(priv_ref)
    assert (n, e) == R.parse_spki_der(pub_ref)
    keys.append((n, e, d, ossl.priv(priv_ref), ossl.pub(pub_ref), "reference helper.cpp replica key", pub_ref))
    for ex in (65537, 65537, 3, 17, 0xC0000001):
        der = gen_key(ex)
        n, e, d = R.parse_pkcs8_der(der)
        assert e == ex and n.bit_length() == 2048
        pk = ossl.priv(der)
        pub_der = ossl.pub_der_of(pk)
        assert R.parse_spki_der(pub_der) == (n, e)
        keys.append((n, e, d, pk, ossl.pub(pub_der), f"openssl genpkey 2048, e={ex}", pub_der))

    vecs = []

    def add(ki, msg, sig, cls):
        n, e = keys[ki][0], keys[ki][1]
        v_ossl = ossl.verify(keys[ki][4], msg, sig)
        v_ref = int(R.verify(n, e, msg, sig))
        pinned = v_ossl == v_ref
        assert pinned or cls == "s_plus_n", (cls, ki, len(msg))
        assert v_ossl == int(R.verify_openssl_semantics(n, e, msg, sig)), cls
        vecs.append({"key": ki, "msg": msg.hex(), "sig": sig.hex(), "verdict": v_ref, "openssl": v_ossl,
                     "cls": cls, "pinned": pinned})

    def forge(ki, em: bytes) -> bytes:
        n, _, d = keys[ki][:3]
        return pow(int.from_bytes(em, "big"), d, n).to_bytes(256, "big")

    lengths = list(range(0, 130)) + [183, 184, 191, 192, 247, 248, 255, 256, 257, 1000, 4095, 4096]
    for i, ln in enumerate(lengths):
        ki = i % len(keys)
        msg = bytes(rng.getrandbits(8) for _ in range(ln))
        sig = ossl.sign(keys[ki][3], msg)
        assert sig == R.sign(keys[ki][0], keys[ki][2], msg)  # PKCS#1 v1.5 is deterministic
        add(ki, msg, sig, "valid")
    for ki in range(len(keys)):
        for t in range(10):
            msg = bytes(rng.getrandbits(8) for _ in range(rng.choice([32, 256, 300])))
            sig = ossl.sign(keys[ki][3], msg)
            bit = [0, 7, 8, 2047, 2040, 1024][t] if t < 6 else rng.randrange(2048)
            s = bytearray(sig)
            s[255 - bit // 8] ^= 1 << (bit % 8)
            add(ki, msg, bytes(s), "flip_sig")
            m2 = bytearray(msg)
            m2[rng.randrange(len(m2))] ^= 1 << rng.randrange(8)
            add(ki, bytes(m2), sig, "flip_msg")
            add((ki + 1 + t % (len(keys) - 1)) % len(keys), msg, sig, "wrong_key")
        n = keys[ki][0]
        msg = b"concord-bft rsa edge"
        for s_val, cls in ((0, "s_zero"), (1, "s_one"), (n - 1, "s_n_minus_1"), (n, "s_eq_n"),
                           ((1 << 2048) - 1, "s_max")):
            add(ki, msg, s_val.to_bytes(256, "big"), cls)
        # s + n (< 2^2048 for these moduli when s is small enough): Crypto++ accepts, OpenSSL rejects
        for t in range(4):
            m = bytes(rng.getrandbits(8) for _ in range(64))
            s = int.from_bytes(ossl.sign(keys[ki][3], m), "big")
            if s + n < (1 << 2048):
                add(ki, m, (s + n).to_bytes(256, "big"), "s_plus_n")
        # malformed encodings (forged with d)
        m = b"malformed encodings " + bytes([ki])
        h = hashlib.sha256(m).digest()
        di = R.SHA256_DIGESTINFO
        good = R.emsa_pkcs1_v15_sha256(m, 2048)
        assert forge(ki, good) == ossl.sign(keys[ki][3], m)
        bad = {
            "bt02": b"\x00\x02" + good[2:],
            "bt00": b"\x00\x00" + good[2:],
            "no_sep": good[:204] + b"\xff" + good[205:],
            "short_ps": b"\x00\x01" + b"\xff" * 7 + b"\x00" + bytes(195) + di + h,
            "sha1_info": b"\x00\x01" + b"\xff" * 218 + b"\x00" + bytes.fromhex("3021300906052b0e03021a05000414")
                         + hashlib.sha1(m).digest(),
            "no_null": b"\x00\x01" + b"\xff" * 204 + b"\x00" + bytes.fromhex("302f300b0609608648016503040201")
                       + b"\x04\x20" + h,
            "other_hash": good[:224] + hashlib.sha256(m + b"x").digest(),
            "lead_01": b"\x01" + good[1:],
            "ps_00": good[:100] + b"\x00" + good[101:],
            "raw_digest": b"\x00\x01" + b"\xff" * 221 + b"\x00" + h,
        }
        for cls, em in bad.items():
            assert len(em) == 256, cls
            if int.from_bytes(em, "big") < n:
                add(ki, m, forge(ki, em), "bad_" + cls)
    payload = {
        "format": "cbft rsa golden v1",
        "note": "RSA-2048 PKCS#1 v1.5 SHA-256; openssl = OpenSSL 3.0.2 EVP_DigestVerify verdict, "
                "verdict = Crypto++ 8.2.0 RSASS<PKCS1v15,SHA256> restated (oracle/rsa_ref.py)",
        "keys": [{"n": format(k[0], "x"), "e": k[1], "src": k[5], "spki_der": k[6].hex()} for k in keys],
        "vectors": vecs,
    }
    out = os.path.join(HERE, "rsa_vectors.json")
    with open(out, "w") as f:
        json.dump(payload, f, indent=0)
    acc = sum(v["verdict"] for v in vecs)
    print(f"wrote {out}: {len(vecs)} vectors ({acc} accept / {len(vecs) - acc} reject), "
          f"{sum(not v['pinned'] for v in vecs)} Crypto++-only")


if __name__ == "__main__":
    main()
