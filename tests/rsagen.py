"""Deterministic RSA-2048 test keys and signed batches for the RSA parity tests and bench.py.

Keys are generated once (seeded Miller-Rabin prime search, pure Python) and cached in
tests/golden/rsa_test_keys.json; signatures are PKCS#1 v1.5 / SHA-256 made with CRT (the same
encoding as oracle/rsa_ref.py, restated here so that bench.py's workload generation does not
import the oracle).  Workload / fixture generation only.
"""
from __future__ import annotations

import hashlib
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))

KEYS_PATH = os.path.join(HERE, "golden", "rsa_test_keys.json")
EXPONENTS = (65537, 17, 65537, 17, 3, 65537, 0xC0000001, 65537)


def _is_probable_prime(n: int, rng: random.Random) -> bool:
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for _ in range(24):
        a = rng.randrange(2, n - 2)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _prime(bits: int, e: int, rng: random.Random) -> int:
    while True:
        c = rng.getrandbits(bits) | (3 << (bits - 2)) | 1  # top two bits set: p*q has 2 * bits bits
        if c % e != 1 and _is_probable_prime(c, rng):
            from math import gcd
            if gcd(c - 1, e) == 1:
                return c


def make_keys():
    rng = random.Random(0x5EED_C0DE)
    keys = []
    for e in EXPONENTS:
        p = _prime(1024, e, rng)
        q = _prime(1024, e, rng)
        n = p * q
        assert n.bit_length() == 2048
        d = pow(e, -1, (p - 1) * (q - 1))
        keys.append({"n": format(n, "x"), "e": e, "d": format(d, "x"), "p": format(p, "x"), "q": format(q, "x")})
    with open(KEYS_PATH, "w") as f:
        json.dump({"note": "test-only RSA-2048 keys (tests/rsagen.py, seeded)", "keys": keys}, f, indent=0)


def load_keys():
    if not os.path.exists(KEYS_PATH):
        make_keys()
    raw = json.load(open(KEYS_PATH))["keys"]
    return [{k: (v if k == "e" else int(v, 16)) for k, v in key.items()} for key in raw]


def emsa_sha256_2048(msg: bytes) -> bytes:
    """EMSA-PKCS1-v1_5 for SHA-256 at 2048 bits: 00 01 FF*202 00 || DigestInfo || H(m)."""
    t = bytes.fromhex("3031300d060960864801650304020105000420") + hashlib.sha256(msg).digest()
    return b"\x00\x01" + b"\xff" * (256 - 3 - len(t)) + b"\x00" + t


def sign(key, msg: bytes) -> bytes:
    """PKCS#1 v1.5 / SHA-256 signature with CRT (equal to rsa_ref.sign)."""
    n, d, p, q = key["n"], key["d"], key["p"], key["q"]
    m = int.from_bytes(emsa_sha256_2048(msg), "big")
    sp = pow(m, d % (p - 1), p)
    sq = pow(m, d % (q - 1), q)
    h = (pow(q, -1, p) * (sp - sq)) % p
    return (sq + h * q).to_bytes(256, "big")


def signed_batch(n: int, nuniq: int = 512, msg_len=256, invalid_frac: float = 0.1, seed: int = 7, key_ids=None):
    """n (key_idx, sig, msg, expected) entries over load_keys(): nuniq distinct honest signatures
    tiled to n, then ~invalid_frac of the entries corrupted (bit flips in s or m, wrong key).
    key_ids restricts the signing keys (e.g. the e = 65537 client keys)."""
    keys = load_keys()
    ids = list(key_ids) if key_ids is not None else list(range(len(keys)))
    rng = random.Random(seed)
    uniq = []
    for u in range(nuniq):
        ki = ids[u % len(ids)]
        ln = msg_len if isinstance(msg_len, int) else rng.randint(*msg_len)
        msg = bytes(rng.getrandbits(8) for _ in range(ln))
        uniq.append((ki, sign(keys[ki], msg), msg))
    kidx, sigs, msgs, exp = [], [], [], []
    for i in range(n):
        ki, sig, msg = uniq[i % nuniq]
        ok = True
        if rng.random() < invalid_frac:
            kind = rng.randrange(3)
            if kind == 0:
                s = bytearray(sig)
                s[rng.randrange(256)] ^= 1 << rng.randrange(8)
                sig = bytes(s)
            elif kind == 1:
                m = bytearray(msg) if msg else bytearray(b"\0")
                m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
                msg = bytes(m)
            else:
                ki = (ki + 1) % len(keys)
            ok = None  # decided by the oracle
        kidx.append(ki)
        sigs.append(sig)
        msgs.append(msg)
        exp.append(ok)
    return keys, kidx, sigs, msgs, exp


if __name__ == "__main__":
    make_keys()
    print("wrote", KEYS_PATH)
