"""CPU tests of the RSA path's checker and host logic:
the Crypto++-semantics restatement (oracle/rsa_ref.py) against OpenSSL-pinned golden vectors, the
reference's own test key, and Python models of the GPU kernels' Montgomery arithmetic (the
one-lane FIOS rows over 32-bit limbs, R = 2^2048, and the lane-pair radix-2^28 column
accumulators, R' = 2^2072) checked against exact big-integer results, with every 64-bit
intermediate bound asserted."""
import json
import os
import random

import pytest

import rsa_ref as R
import rsagen

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "rsa_vectors.json")


def golden():
    g = json.load(open(GOLDEN))
    keys = [(int(k["n"], 16), k["e"]) for k in g["keys"]]
    return g, keys


def test_golden_vectors_oracle_matches_both_verdict_columns():
    g, keys = golden()
    vecs = g["vectors"]
    assert len(vecs) > 400
    for v in vecs:
        n, e = keys[v["key"]]
        msg, sig = bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])
        assert int(R.verify(n, e, msg, sig)) == v["verdict"], v["cls"]
        assert int(R.verify_openssl_semantics(n, e, msg, sig)) == v["openssl"], v["cls"]
        if v["pinned"]:
            assert v["verdict"] == v["openssl"]
    classes = {v["cls"] for v in vecs}
    for c in ("valid", "flip_sig", "flip_msg", "wrong_key", "s_zero", "s_eq_n", "s_plus_n", "bad_bt02",
              "bad_no_null", "bad_sha1_info", "bad_lead_01"):
        assert c in classes, c
    assert sum(v["verdict"] for v in vecs if v["cls"] == "valid") == sum(1 for v in vecs if v["cls"] == "valid")
    # the unpinned difference is exactly s >= n accepted by Crypto++
    assert all(v["verdict"] == 1 and v["openssl"] == 0 for v in vecs if not v["pinned"])


def test_reference_replica_key_is_in_fixture():
    g, keys = golden()
    assert g["keys"][0]["src"].startswith("reference helper.cpp")
    n, e = R.parse_spki_der(bytes.fromhex(g["keys"][0]["spki_der"]))
    assert (n, e) == keys[0] and e == 17 and n.bit_length() == 2048


def test_emsa_layout():
    em = R.emsa_pkcs1_v15_sha256(b"abc", 2048)
    assert len(em) == 256 and em[:2] == b"\x00\x01" and em[2:204] == b"\xff" * 202 and em[204] == 0
    assert em[205:224] == R.SHA256_DIGESTINFO


def test_signature_lengths_crypto_pp_semantics():
    k = rsagen.load_keys()[0]
    msg = b"short signature"
    sig = rsagen.sign(k, msg)
    stripped = sig.lstrip(b"\0")
    assert R.verify(k["n"], k["e"], msg, stripped)          # Integer(sig, len) ignores leading zeros
    assert R.verify(k["n"], k["e"], msg, b"\0" * 3 + sig)    # longer, zero-padded
    assert not R.verify_openssl_semantics(k["n"], k["e"], msg, b"\0" + sig)


# ---------------------------------------------------------------- kernel arithmetic model ----
M32 = (1 << 32) - 1


def limbs(x):
    return [(x >> (32 * i)) & M32 for i in range(64)]


def mont_mul_fios(a, b, n):
    """The kernel's mont_mul (concord-bft_amd/csrc/rsa_verify.hip): per row two carry chains,
    every intermediate checked to fit the 64-bit v_mad_u64_u32 result."""
    nl, al, bl = limbs(n), limbs(a), limbs(b)
    n0inv = (-pow(nl[0], -1, 1 << 32)) & M32
    t = [0] * 65
    for i in range(64):
        ai = al[i]
        X = ai * bl[0] + t[0]
        m = (X & M32) * n0inv & M32
        Y = m * nl[0] + (X & M32)
        assert Y & M32 == 0
        c1, c2 = X >> 32, Y >> 32
        for j in range(1, 64):
            X = ai * bl[j] + t[j] + c1
            Y = m * nl[j] + (X & M32) + c2
            assert X < 1 << 64 and Y < 1 << 64
            c1, c2 = X >> 32, Y >> 32
            t[j - 1] = Y & M32
        top = t[64] + c1 + c2
        t[63] = top & M32
        t[64] = top >> 32
        assert t[64] <= 1
    v = sum(x << (32 * i) for i, x in enumerate(t))
    assert v < 2 * n
    return v - n if v >= n else v


@pytest.mark.parametrize("seed", range(3))
def test_kernel_montgomery_model(seed):
    rng = random.Random(seed)
    keys = rsagen.load_keys()
    R_ = 1 << 2048
    for k in keys[:4]:
        n = k["n"]
        rinv = pow(R_, -1, n)
        cases = [(rng.randrange(n), rng.randrange(n)), (n - 1, n - 1), (R_ - 1, (R_ * R_) % n), (0, n - 1),
                 (1, 1)]
        for a, b in cases:
            assert mont_mul_fios(a, b, n) == a * b * rinv % n


def test_kernel_exponent_schedule_model():
    """The wave-uniform square-and-multiply schedule (masked multiplies, x starts at R mod n)
    gives s^e for lanes whose exponents differ in length."""
    keys = rsagen.load_keys()
    R_ = 1 << 2048
    rng = random.Random(5)
    n = keys[0]["n"]
    for e in (3, 17, 65537, 0xC0000001):
        s = rng.randrange(R_)  # s may exceed n (Crypto++ reduces it)
        top = 31  # wave top bit (some other lane holds e = 0xC0000001)
        sm = mont_mul_fios(s, R_ * R_ % n, n)
        x = R_ % n
        for bit in range(top, -1, -1):
            if bit != top:
                x = mont_mul_fios(x, x, n)
            if (e >> bit) & 1:
                x = mont_mul_fios(sm, x, n)
        x = mont_mul_fios(1, x, n)
        assert x == pow(s, e, n)


def mont_mul_pair_model(a, b, n):
    """The lane-pair radix-2^28 product of rsa_verify_pair_kernel: 74 limbs, R' = 2^2072, column
    accumulators split over an even (positions 0..37) and odd (38..75) lane, two rows per
    iteration then a two-column shift.  Checks every accumulator stays below 2^64 and returns
    the fully carried value (< 2n)."""
    M = (1 << 28) - 1
    NL, PC = 74, 38
    al = [(a >> (28 * i)) & M for i in range(NL)] + [0, 0]
    xs = [0] + [(b >> (28 * i)) & M for i in range(NL)] + [0] * 5          # slot 1 + j = limb j
    nl = [(n >> (28 * i)) & M for i in range(NL)]
    n0inv = (-pow(nl[0], -1, 1 << 28)) % (1 << 28)
    lanes = []
    for hi in (0, 1):
        P0 = PC if hi else 0
        nreg = [nl[P0 + k - 1] if 0 <= P0 + k - 1 < NL else 0 for k in range(PC + 1)]
        lanes.append({"P0": P0, "nreg": nreg, "A": [0] * PC})
    for i in range(0, NL, 2):
        for ln in lanes:
            ln["xv"] = [xs[ln["P0"] + k] for k in range(PC + 1)]
        L, H = lanes
        for h, ai in ((0, al[i]), (1, al[i + 1])):
            for ln in lanes:
                for c in range(PC):
                    ln["A"][c] += ai * ln["xv"][c + 1 - h]
            m = (L["A"][h] & 0xFFFFFFFF) * n0inv & M
            for ln in lanes:
                for c in range(PC):
                    ln["A"][c] += m * ln["nreg"][c + 1 - h]
                    assert ln["A"][c] < 1 << 64
            L["A"][h + 1] += L["A"][h] >> 28
        u0, u1 = H["A"][0], H["A"][1]
        for ln in lanes:
            ln["A"] = ln["A"][2:] + [0, 0]
        L["A"][PC - 2], L["A"][PC - 1] = u0, u1
    v = sum(x << (28 * c) for c, x in enumerate(lanes[0]["A"]))
    v += sum(x << (28 * (PC + c)) for c, x in enumerate(lanes[1]["A"]))
    assert v < 2 * n
    return v


@pytest.mark.parametrize("seed", range(2))
def test_kernel_pair_radix28_model(seed):
    rng = random.Random(100 + seed)
    keys = rsagen.load_keys()
    R = 1 << 2072
    for k in keys[:3]:
        n = k["n"]
        rinv = pow(R, -1, n)
        for a, b in [(rng.randrange(2 * n), rng.randrange(2 * n)), (2 * n - 1, 2 * n - 1),
                     ((1 << 2048) - 1, R * R % n), (1, n - 1)]:
            assert mont_mul_pair_model(a, b, n) % n == a * b * rinv % n
