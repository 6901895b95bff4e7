"""Synthetic signed-message sets for tests and bench (BASELINE.json configs), built with the
host OpenSSL (tools/cpu_baseline/libcbft_cpu_openssl.so).  Key i's seed is
SHA-512("cbft-key" || le32(i))[:32]; messages come from a seeded numpy PCG64.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
CPU_SO = os.path.join(ROOT, "tools", "cpu_baseline", "libcbft_cpu_openssl.so")
_cpu = None


def cpu_lib():
    global _cpu
    if _cpu is None:
        if not os.path.exists(CPU_SO):
            raise RuntimeError(f"{CPU_SO} missing: run `make cpu`")
        lib = ctypes.CDLL(CPU_SO)
        vp = ctypes.c_void_p
        lib.cbft_cpu_keys_new.restype = vp
        lib.cbft_cpu_keys_new.argtypes = [vp, ctypes.c_uint32]
        lib.cbft_cpu_keys_free.argtypes = [vp, ctypes.c_uint32]
        lib.cbft_cpu_verify.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
        lib.cbft_cpu_pubkey.argtypes = [vp, vp]
        lib.cbft_cpu_sign_many.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
        lib.cbft_cpu_rsa_keys_new.restype = vp
        lib.cbft_cpu_rsa_keys_new.argtypes = [vp, vp, ctypes.c_uint32]
        lib.cbft_cpu_rsa_verify.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
        _cpu = lib
    return _cpu


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def key_seeds(nkeys: int) -> np.ndarray:
    return np.frombuffer(b"".join(hashlib.sha512(b"cbft-key" + i.to_bytes(4, "little")).digest()[:32]
                                  for i in range(nkeys)), dtype=np.uint8).reshape(nkeys, 32).copy()


def pubkeys(sks: np.ndarray) -> np.ndarray:
    lib = cpu_lib()
    out = np.zeros_like(sks)
    for i in range(sks.shape[0]):
        assert lib.cbft_cpu_pubkey(_p(sks[i]), _p(out[i])) == 0
    return out


@dataclass
class SigSet:
    pk: np.ndarray        # nkeys x 32
    key_idx: np.ndarray   # n u32
    sig: np.ndarray       # n x 64
    blob: np.ndarray      # u8
    off: np.ndarray       # n u64
    len: np.ndarray       # n u32
    expected: np.ndarray  # n bool (OpenSSL verdicts)

    @property
    def n(self):
        return self.key_idx.shape[0]

    def msgs(self):
        b = self.blob.tobytes()
        return [b[o:o + l] for o, l in zip(self.off.tolist(), self.len.tolist())]

    def per_sig_pk(self) -> np.ndarray:
        return np.ascontiguousarray(self.pk[self.key_idx])


def make_sigset(n: int, nkeys: int = 4096, msg_len=256, seed: int = 0xC0FFEE, invalid_frac: float = 0.0,
                threads: int = 8, compute_expected: bool = True) -> SigSet:
    """msg_len: int (fixed) or (lo, hi) for log-uniform lengths in [lo, hi]."""
    rng = np.random.default_rng(seed)
    sks = key_seeds(nkeys)
    pk = pubkeys(sks)
    key_idx = (np.arange(n, dtype=np.uint64) % nkeys).astype(np.uint32)
    if isinstance(msg_len, tuple):
        lo, hi = msg_len
        lens = np.exp(rng.uniform(np.log(lo), np.log(hi + 1), size=n)).astype(np.uint32)
        lens = np.clip(lens, lo, hi).astype(np.uint32)
    else:
        lens = np.full(n, msg_len, dtype=np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    total = int(lens.sum())
    blob = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    sig = np.zeros((n, 64), dtype=np.uint8)
    lib = cpu_lib()
    lib.cbft_cpu_sign_many(_p(sks), nkeys, _p(key_idx), _p(blob), _p(off), _p(lens), n, _p(sig), threads)
    if invalid_frac > 0:
        bad = rng.random(n) < invalid_frac
        kinds = rng.integers(0, 5, size=n)
        L = 2**252 + 27742317777372353535851937790883648493
        for i in np.nonzero(bad)[0]:
            k = kinds[i]
            if k == 0:      # flip a bit of R
                sig[i, rng.integers(0, 32)] ^= 1 << int(rng.integers(0, 8))
            elif k == 1:    # flip a bit of S
                sig[i, 32 + rng.integers(0, 31)] ^= 1 << int(rng.integers(0, 8))
            elif k == 2:    # S + L
                s = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
                sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), dtype=np.uint8)
            elif k == 3 and lens[i] > 0:  # flip a message byte
                blob[int(off[i]) + int(rng.integers(0, int(lens[i])))] ^= 0x5A
            else:           # wrong key
                key_idx[i] = (key_idx[i] + 1) % nkeys
    ss = SigSet(pk, key_idx, sig, blob, off, lens, np.zeros(n, dtype=bool))
    if compute_expected:
        ss.expected = cpu_verify(ss, threads=threads).astype(bool)
    return ss


def cpu_verify(ss: SigSet, threads: int = 8, keycache=None) -> np.ndarray:
    lib = cpu_lib()
    own = keycache is None
    if own:
        keycache = lib.cbft_cpu_keys_new(_p(ss.pk), ss.pk.shape[0])
    out = np.zeros(ss.n, dtype=np.uint8)
    lib.cbft_cpu_verify(keycache, _p(ss.key_idx), _p(ss.sig), _p(ss.blob), _p(ss.off), _p(ss.len), ss.n, _p(out),
                        threads)
    if own:
        lib.cbft_cpu_keys_free(keycache, ss.pk.shape[0])
    return out


# ------------------------------------------------------------------ BLS BN-P254 (config #4)
# Host build of the library's own BN-P254 code (tests/cpp/libbn254_shim.so, `make shim`): used
# here only to generate key sets and shares, and as the labelled "not RELIC" CPU baseline.
BN_R = 0x2523648240000001BA344D8000000007FF9F800000000010A10000000000000D
SHIM_SO = os.path.join(ROOT, "tests", "cpp", "libbn254_shim.so")
_shim = None


def bn_lib():
    global _shim
    if _shim is None:
        if not os.path.exists(SHIM_SO):
            raise RuntimeError(f"{SHIM_SO} missing: run `make shim`")
        _shim = ctypes.CDLL(SHIM_SO)
    return _shim


@dataclass
class BlsCert:
    n: int
    k: int
    pk: bytes          # 65-byte group public key
    vks: list          # n x 65-byte share verification keys
    msg: bytes         # 32-byte digest
    shares: list       # 37-byte shares (id || G1), some "doubled" (bad)
    bad: set           # indices into shares
    expected_sig: bytes
    sign_probe: tuple = None  # (id, sk, share) of one good share: signing is checked against it


def make_bls_cert(n: int = 1024, k: int = 683, extra: int = 0, bad_frac: float = 0.0, seed: int = 2024,
                  threads: int = 8) -> BlsCert:
    """Shamir key set (degree k-1 polynomial, as BlsThresholdKeygen), shares of k + extra
    random signers over a 32-byte digest; bad shares are sigma doubled (TestBlsBatchVerifier.cpp:84-90)."""
    import random
    rng = random.Random(seed)
    coeffs = [rng.randrange(1, BN_R) for _ in range(k)]

    def f(x):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % BN_R
        return acc

    lib = bn_lib()
    sks = {i: f(i) for i in range(1, n + 1)}
    buf = b"".join(sks[i].to_bytes(32, "big") for i in range(1, n + 1))
    out = ctypes.create_string_buffer(65 * n)
    lib.shim_g2_mul_gen_mt(buf, n, out, threads)
    vks = [out.raw[65 * i:65 * i + 65] for i in range(n)]
    pkb = ctypes.create_string_buffer(65)
    lib.shim_g2_mul_gen(coeffs[0].to_bytes(32, "big"), pkb)
    msg = bytes(rng.randrange(256) for _ in range(32))
    ids = sorted(rng.sample(range(1, n + 1), k + extra))
    sbuf = b"".join(sks[i].to_bytes(32, "big") for i in ids)
    arr = (ctypes.c_uint32 * len(ids))(*ids)
    so = ctypes.create_string_buffer(37 * len(ids))
    lib.shim_sign_shares_mt(sbuf, arr, len(ids), msg, len(msg), so, threads)
    shares = [so.raw[37 * j:37 * j + 37] for j in range(len(ids))]
    bad = set(rng.sample(range(len(shares)), int(round(bad_frac * len(shares)))))
    two = (2).to_bytes(32, "big")
    for j in bad:
        d = ctypes.create_string_buffer(33)
        lib.shim_g1_mul(shares[j][4:], two, d)
        shares[j] = shares[j][:4] + d.raw
    es = ctypes.create_string_buffer(37)
    lib.shim_sign_share(coeffs[0].to_bytes(32, "big"), 0, msg, len(msg), es)
    good = min(j for j in range(len(shares)) if j not in bad)
    probe = (ids[good], sks[ids[good]], shares[good])
    return BlsCert(n, k, pkb.raw, vks, msg, shares, bad, es.raw[4:], probe)


def cpu_bls_verify_shares(cert: BlsCert, h33: bytes, threads: int = 16) -> np.ndarray:
    lib = bn_lib()
    k = len(cert.shares)
    out = np.zeros(k, dtype=np.uint8)
    lib.shim_verify_shares_mt(h33, b"".join(cert.vks), cert.n, b"".join(cert.shares), k, _p(out), threads)
    return out
