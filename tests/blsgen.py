"""BLS test-set generation through the host build of the device code (tests/cpp/libbn254_shim.so)
and the Python oracle.  Keys: Shamir shares of a random sk (degree k-1), as BlsThresholdKeygen."""
import ctypes
import os
import random

import bn254_ref as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "cpp", "libbn254_shim.so")
_shim = None


def shim():
    global _shim
    if _shim is None:
        _shim = ctypes.CDLL(SHIM)
    return _shim


def be32(x: int) -> bytes:
    return x.to_bytes(32, "big")


def keyset(n: int, k: int, seed: int, threads: int = 8):
    """(sk, {i: sk_i}, pk65, [vk65_1..vk65_n]) with vk_i = sk_i g2."""
    sk, sks = B.keygen(n, k, seed)
    buf = b"".join(be32(sks[i]) for i in range(1, n + 1))
    out = ctypes.create_string_buffer(65 * n)
    shim().shim_g2_mul_gen_mt(buf, n, out, threads)
    vks = [out.raw[65 * i:65 * i + 65] for i in range(n)]
    pk = ctypes.create_string_buffer(65)
    shim().shim_g2_mul_gen(be32(sk), pk)
    return sk, sks, pk.raw, vks


def shares(sks: dict, ids, msg: bytes, threads: int = 8):
    ids = list(ids)
    buf = b"".join(be32(sks[i]) for i in ids)
    arr = (ctypes.c_uint32 * len(ids))(*ids)
    out = ctypes.create_string_buffer(37 * len(ids))
    shim().shim_sign_shares_mt(buf, arr, len(ids), msg, len(msg), out, threads)
    return [out.raw[37 * j:37 * j + 37] for j in range(len(ids))]


def doubled(share: bytes) -> bytes:
    """Bad share as in TestBlsBatchVerifier.cpp:84-90 (sig.Double())."""
    i, s = B.parse_share(share)
    return share[:4] + B.g1_to_bytes(B.ec_add(s, s, None))


def sign_point(sk: int, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(37)
    shim().shim_sign_share(be32(sk), 0, msg, len(msg), out)
    return out.raw[4:]
