"""Parity gate run by bench.py (before anything is timed) and by __graft_entry__.smoke(): every
verdict class the GPU tests cover, checked against committed golden DATA only (no oracle import;
the fixtures were produced by the scripts under tests/golden/).  Any mismatch raises
ParityError, and bench.py exits non-zero, so a driver-run bench proves parity on its own even when
the separate GPU test run is lost.

Classes:
  ed25519  tests/golden/ed25519_vectors.bin — 1,145 OpenSSL 3.0.2 verdicts: RFC 8032 §7.1, honest
           signatures over SHA-512 block boundaries, R/S/A/M bit flips, S + L, high S bits, wrong
           key, small-order / non-canonical / off-curve / mixed-order A, non-canonical R.  Through
           per-signature keys (cbft_ed25519_verify_batch_pk) AND the key table
           (cbft_ed25519_load_keys + cbft_ed25519_verify_batch), per class.
  relic    tests/golden/relic_bls_keys.json (RELIC output held by the reference's key files
           tests/simpleKVBC/scripts/set{A,B}_replica_*) + tests/golden/relic_bls_vectors.json
           (oracle/bn254_ref.py bytes): sk_i*g2 == vk_i (40/40), decode -> encode of every vk,
           multisig sum of vks == group key, GPU-signed shares == oracle shares, share verdicts
           with a doubled share, threshold combinations / multisig aggregates == the oracle's
           bytes and verifying under the file's group key.
  rsa      tests/golden/rsa_vectors.json — 417 verdicts (Crypto++ semantics, OpenSSL-pinned):
           honest, bit flips, wrong key, s in {0, 1, n-1, n, 2^2048-1}, forged encodings.
"""
from __future__ import annotations

import json
import os
import struct
from collections import Counter, defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

ED_CLASSES = {0: "rfc8032", 1: "valid", 2: "flip_r", 3: "flip_s", 4: "s_plus_l", 5: "s_high_bits", 6: "flip_msg",
              7: "wrong_key", 8: "small_order_a", 9: "noncanon_a", 10: "noncanon_r", 11: "offcurve_a",
              12: "mixed_order_a", 13: "flip_a", 14: "long_msg"}


class ParityError(SystemExit):
    pass


def _bools(bitmap: bytes, n: int) -> np.ndarray:
    return np.unpackbits(np.frombuffer(bitmap, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def load_ed25519():
    data = open(os.path.join(GOLDEN, "ed25519_vectors.bin"), "rb").read()
    if data[:16] != b"CBFTED25519V1\0\0\0":
        raise ParityError("ed25519_vectors.bin: bad header")
    (n,) = struct.unpack_from("<I", data, 16)
    off, out = 20, []
    for _ in range(n):
        mlen, v, cls, _ = struct.unpack_from("<IBBH", data, off)
        off += 8
        out.append((cls, bool(v), data[off:off + 32], data[off + 32:off + 96], data[off + 96:off + 96 + mlen]))
        off += 96 + mlen
    return out


def _per_class(classes, exp, got, names):
    rec = defaultdict(lambda: {"n": 0, "accept": 0, "mismatch": 0})
    for c, e, g in zip(classes, exp, got):
        r = rec[names(c)]
        r["n"] += 1
        r["accept"] += int(e)
        r["mismatch"] += int(e != g)
    return dict(sorted(rec.items()))


def gate_ed25519(ctx) -> dict:
    vecs = load_ed25519()
    cls = [v[0] for v in vecs]
    exp = np.array([v[1] for v in vecs])
    pks, sigs, msgs = [v[2] for v in vecs], [v[3] for v in vecs], [v[4] for v in vecs]
    got_pk = _bools(ctx.verify_pk(pks, sigs, msgs), len(vecs))
    keys = sorted(set(pks))
    index = {k: i for i, k in enumerate(keys)}
    tid = ctx.load_keys(keys)
    try:
        got_tab = _bools(ctx.verify(tid, [index[p] for p in pks], sigs, msgs), len(vecs))
    finally:
        ctx.unload_keys(tid)
    out = {"vectors": len(vecs), "accept": int(exp.sum()), "distinct_keys": len(keys),
           "per_signature_keys_mismatch": int((got_pk != exp).sum()),
           "key_table_mismatch": int((got_tab != exp).sum()),
           "classes": _per_class(cls, exp, got_pk, ED_CLASSES.get)}
    for c, r in _per_class(cls, exp, got_tab, ED_CLASSES.get).items():
        out["classes"][c]["mismatch_key_table"] = r["mismatch"]
    if out["per_signature_keys_mismatch"] or out["key_table_mismatch"]:
        raise ParityError(f"parity gate: Ed25519 golden vectors differ: {out}")
    return out


def _bitmap(ids) -> bytes:
    b = bytearray(256)
    for i in ids:
        b[(i - 1) // 8] |= 1 << ((i - 1) % 8)
    return bytes(b)


def gate_relic(ctx) -> dict:
    keys = json.load(open(os.path.join(GOLDEN, "relic_bls_keys.json")))
    vecs = {s["name"]: s for s in json.load(open(os.path.join(GOLDEN, "relic_bls_vectors.json")))["systems"]}
    c = Counter()
    fails = []
    for sname, systems in sorted(keys["sets"].items()):
        for cname, r in sorted(systems.items()):
            name = f"{sname}/{cname}"
            n, thr = r["n"], r["threshold"]
            multisig = r["type"] == "multisig-bls" or thr == n
            pk = bytes.fromhex(r["public_key"])
            vks = [bytes.fromhex(h) for h in r["verification_keys"]]
            sks = {int(i): int(v) for i, v in r["secret_shares"].items()}
            v = vecs[name]
            msg = bytes.fromhex(v["msg"])
            for i, sk in sks.items():  # sk_i * g2 == the RELIC-written vk_i
                c["vk_from_sk"] += 1
                if ctx.bls_public_key(sk) != vks[i - 1]:
                    fails.append(f"{name}: sk_{i}*g2 != vk_{i}")
            if ctx.bls_hash_to_g1(msg).hex() != v["h_g1"]:
                fails.append(f"{name}: hash_to_g1 differs from the oracle")
            c["hash_to_g1"] += 1
            kid = ctx.bls_load_keys(pk, vks)
            try:
                if not all(ctx.bls_key_status(kid, n)):
                    fails.append(f"{name}: a RELIC vk failed to decode")
                for i in range(1, n + 1):  # decode -> encode round trip of every vk
                    c["vk_roundtrip"] += 1
                    if ctx.bls_sum_keys(kid, _bitmap([i])) != vks[i - 1]:
                        fails.append(f"{name}: vk_{i} does not re-encode")
                if multisig:
                    c["group_key_sum"] += 1
                    if ctx.bls_sum_keys(kid, _bitmap(range(1, n + 1))) != pk:
                        fails.append(f"{name}: sum of vks != group key")
                shares = [ctx.bls_sign(sks[i], i, msg) for i in range(1, n + 1)]
                exp_sh = [bytes.fromhex(h) for h in v["shares"]]
                c["shares_signed"] += n
                for i, (a, b) in enumerate(zip(shares, exp_sh), 1):
                    if a != b:
                        fails.append(f"{name}: share {i} differs from the oracle")
                bad = bytes.fromhex(v["bad_share"])
                ver = ctx.bls_verify_shares(kid, msg, exp_sh + [bad]).tolist()
                c["share_verdicts"] += n + 1
                if ver != [True] * n + [False]:
                    fails.append(f"{name}: share verdicts {ver}")
                combined = bytes.fromhex(v["combined"])
                if multisig:
                    agg = ctx.bls_combine(exp_sh, multisig=True)
                    c["combined"] += 1
                    if agg != combined or not ctx.bls_verify_multisig(kid, msg, agg, _bitmap(range(1, n + 1))) \
                            or not ctx.bls_verify(kid, msg, agg):
                        fails.append(f"{name}: multisig aggregate")
                else:
                    for ids in v["subsets"]:
                        c["combined"] += 1
                        comb = ctx.bls_combine([exp_sh[i - 1] for i in ids])
                        if comb != combined or not ctx.bls_verify(kid, msg, comb):
                            fails.append(f"{name}: combination of {ids}")
                    # the certificate policy with share 1 replaced by its doubled form: the
                    # optimistic combine fails, per-share verification flags exactly share 1, and
                    # the other n - 1 >= threshold shares combine to the same signature
                    sig, ok, badv = ctx.bls_combine_threshold(kid, msg, [bad] + exp_sh[1:], optimistic=True)
                    c["combine_threshold"] += 1
                    if not ok or sig != combined or badv.tolist() != [True] + [False] * (n - 1):
                        fails.append(f"{name}: combine_threshold ok={ok} bad={badv.tolist()}")
                c["reject_wrong_msg"] += 1
                if ctx.bls_verify(kid, msg[::-1], combined):
                    fails.append(f"{name}: verified under the wrong digest")
            finally:
                ctx.bls_unload_keys(kid)
            c["systems"] += 1
    if fails:
        raise ParityError("parity gate: RELIC fixture: " + "; ".join(fails[:10]))
    return dict(c)


def gate_rsa(ctx) -> dict:
    g = json.load(open(os.path.join(GOLDEN, "rsa_vectors.json")))
    keys = [(int(k["n"], 16), k["e"]) for k in g["keys"]]
    tid = ctx.rsa_load_keys(keys)
    try:
        if not ctx.rsa_key_status(tid, len(keys)).all():
            raise ParityError("parity gate: an RSA golden key failed to load")
        vecs = g["vectors"]
        got = _bools(ctx.rsa_verify(tid, [v["key"] for v in vecs], [bytes.fromhex(v["sig"]) for v in vecs],
                                    [bytes.fromhex(v["msg"]) for v in vecs]), len(vecs))
    finally:
        ctx.rsa_unload_keys(tid)
    exp = np.array([bool(v["verdict"]) for v in vecs])
    out = {"vectors": len(vecs), "accept": int(exp.sum()), "reject": int((~exp).sum()),
           "mismatch": int((got != exp).sum()),
           "classes": _per_class([v["cls"] for v in vecs], exp, got, lambda x: x)}
    if out["mismatch"]:
        raise ParityError(f"parity gate: RSA golden vectors differ: {out}")
    return out


def run(ctx, rsa: bool = True, relic: bool = True) -> dict:
    out = {"ed25519_golden": gate_ed25519(ctx)}
    if relic:
        out["relic_bls_fixture"] = gate_relic(ctx)
    if rsa:
        out["rsa_golden"] = gate_rsa(ctx)
    return out
