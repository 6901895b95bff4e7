"""CPU restatement of the reference's RSA signature verify — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (libcbft_hipcrypto) never calls it.

What it restates:
  concord::util::crypto::RSAVerifier::verify  util/src/crypto_utils.cpp:101-117,166
      = Crypto++ 8.2.0 (thirdparty/cryptopp.cmake:3-18) RSASS<PKCS1v15, SHA256>::Verifier::
        VerifyMessage(data, len, sig, siglen)
Crypto++ is a network-fetched dependency absent from /root/reference, so its published
algorithm is restated here:
  * PK_Verifier::VerifyMessage -> TF_VerifierBase::InputSignature: the signature bytes are read
    as one big-endian Integer of ANY length (Integer(signature, signatureLength)), then
    RSAFunction::ApplyFunction = a_exp_b_mod_c(s, e, n) — no `s < n` check, so s is used mod n;
    if the result has more than MessageRepresentativeBitLength() = bits(n) - 1 bits it is
    replaced by 0; it is then encoded big-endian into MessageRepresentativeLength() =
    ceil((bits(n) - 1) / 8) bytes.
  * TF_VerifierBase::VerifyAndRestart -> PK_DeterministicSignatureMessageEncodingMethod::
    VerifyMessageRepresentative: recompute PKCS1v15_SignatureMessageEncodingMethod::
    ComputeMessageRepresentative(SHA-256 digest) — a leading 0x00 byte when (bits(n) - 1) % 8 != 0,
    then 0x01, 0xFF padding, 0x00, the SHA-256 DigestInfo prefix, the digest — and compare the
    two byte strings for equality.
For a 2048-bit modulus this is: accept iff (s mod n)^e mod n == 00 01 FF*202 00 || DigestInfo ||
SHA-256(m).  On every signature of exactly modulus length with s < n this coincides with OpenSSL
3.0.2's RSA_verify (RSA_PKCS1_PADDING, NID_sha256), and tests/golden/rsa_vectors.json pins it
there.  Where the two differ (s >= n, signatures of other lengths) the verdict is Crypto++'s and
is **parity unpinned** (Crypto++ is not available offline).
"""
from __future__ import annotations

import hashlib

# DER DigestInfo prefix for SHA-256 (PKCS #1 v2.2 §9.2 note 1; Crypto++ PKCS_DigestDecoration<SHA256>)
SHA256_DIGESTINFO = bytes.fromhex("3031300d060960864801650304020105000420")


def emsa_pkcs1_v15_sha256(msg: bytes, nbits: int) -> bytes:
    """PKCS1v15_SignatureMessageEncodingMethod::ComputeMessageRepresentative for SHA-256, as the
    bytes of the representative (length ceil((nbits - 1) / 8))."""
    rep_bits = nbits - 1
    rep_len = (rep_bits + 7) // 8
    t = SHA256_DIGESTINFO + hashlib.sha256(msg).digest()
    lead = b"\x00" if rep_bits % 8 else b""
    body_len = rep_len - len(lead)
    ps = body_len - 2 - len(t)
    if ps < 0:
        raise ValueError("modulus too short for SHA-256 PKCS#1 v1.5")
    return lead + b"\x01" + b"\xff" * ps + b"\x00" + t


def verify(n: int, e: int, msg: bytes, sig: bytes) -> bool:
    """RSAVerifier::verify(data, sig) with Crypto++ 8.2.0 semantics (see module docstring)."""
    nbits = n.bit_length()
    rep_bits = nbits - 1
    rep_len = (rep_bits + 7) // 8
    s = int.from_bytes(sig, "big")
    x = pow(s, e, n)
    if x.bit_length() > rep_bits:
        x = 0
    return x.to_bytes(rep_len, "big") == emsa_pkcs1_v15_sha256(msg, nbits)


def verify_openssl_semantics(n: int, e: int, msg: bytes, sig: bytes) -> bool:
    """OpenSSL 3.0.2 RSA_verify(NID_sha256) restated: the signature must be exactly the modulus
    length and s < n, then the same encoding comparison.  Used only to explain where the golden
    verdicts (OpenSSL) and Crypto++ differ."""
    k = (n.bit_length() + 7) // 8
    if len(sig) != k or int.from_bytes(sig, "big") >= n:
        return False
    return verify(n, e, msg, sig)


def sign(n: int, d: int, msg: bytes) -> bytes:
    """RSASS<PKCS1v15, SHA256>::Signer::SignMessage (deterministic): EM^d mod n, modulus length."""
    k = (n.bit_length() + 7) // 8
    em = int.from_bytes(emsa_pkcs1_v15_sha256(msg, n.bit_length()), "big")
    return pow(em, d, n).to_bytes(k, "big")


# ---------------------------------------------------------------- minimal DER key codecs ----
# The reference loads keys as hex-encoded DER (KeyFormat::HexaDecimalStrippedFormat: Crypto++
# X509PublicKey / PKCS8PrivateKey BER) or PEM (crypto_utils.cpp:142-176).  Only what the test
# fixtures need: SubjectPublicKeyInfo{rsaEncryption, RSAPublicKey{n, e}} and the integers of a
# PKCS#8 RSAPrivateKey.

def _der_read(buf: bytes, pos: int):
    tag = buf[pos]
    ln = buf[pos + 1]
    pos += 2
    if ln & 0x80:
        nb = ln & 0x7F
        ln = int.from_bytes(buf[pos:pos + nb], "big")
        pos += nb
    return tag, buf[pos:pos + ln], pos + ln


def _der_ints(seq: bytes):
    out, pos = [], 0
    while pos < len(seq):
        tag, val, pos = _der_read(seq, pos)
        if tag == 0x02:
            out.append(int.from_bytes(val, "big"))
    return out


def parse_spki_der(der: bytes):
    """SubjectPublicKeyInfo -> (n, e)."""
    _, spki, _ = _der_read(der, 0)
    _, _alg, pos = _der_read(spki, 0)
    tag, bitstr, _ = _der_read(spki, pos)
    assert tag == 0x03 and bitstr[0] == 0
    _, rsapub, _ = _der_read(bitstr[1:], 0)
    n, e = _der_ints(rsapub)[:2]
    return n, e


def parse_pkcs8_der(der: bytes):
    """PKCS#8 PrivateKeyInfo{RSAPrivateKey} or a bare PKCS#1 RSAPrivateKey -> (n, e, d)."""
    _, pki, _ = _der_read(der, 0)
    pos = 0
    _, _ver, pos = _der_read(pki, pos)
    tag, body, pos2 = _der_read(pki, pos)
    if tag == 0x02:  # PKCS#1: version, n, e, d, ...
        ints = _der_ints(pki)
        return ints[1], ints[2], ints[3]
    tag, octets, _ = _der_read(pki, pos2)
    assert tag == 0x04
    _, rsapriv, _ = _der_read(octets, 0)
    ints = _der_ints(rsapriv)
    return ints[1], ints[2], ints[3]
