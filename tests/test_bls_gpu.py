"""GPU parity tests of the BLS BN-P254 path (threshsign) through the C ABI, against the Python
oracle (oracle/bn254_ref.py) and the host build of the same code.  RELIC parity itself is
unpinned; verdicts and combined signatures are fixed by the mathematics."""
import random

import numpy as np
import pytest

import bn254_ref as B
import blsgen
import cbft_hipcrypto as cb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = cb.Context(device=0)
    yield c
    c.close()


def test_hash_to_g1_matches_oracle(ctx):
    for m in (b"", b"abc", bytes(32), bytes(range(32)), b"\xff" * 100):
        assert ctx.bls_hash_to_g1(m) == B.g1_to_bytes(B.g1_map(m))


def test_share_verification_verdicts(ctx):
    n, k = 16, 11
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=11)
    msg = bytes(range(100, 132))
    good = blsgen.shares(sks, range(1, n + 1), msg)
    cases = list(good)
    cases.append(blsgen.doubled(good[2]))                       # Double() -> invalid
    cases.append((4).to_bytes(4, "big") + good[2][4:])          # sk_3's point labelled id 4
    cases.append(b"\x00\x00\x00\x00" + good[0][4:])             # id 0
    cases.append((17).to_bytes(4, "big") + good[0][4:])         # id > n
    cases.append(good[5][:4] + b"\x05" + good[5][5:])           # bad prefix
    cases.append(good[5][:4] + b"\x02" + B.P.to_bytes(32, "big"))  # x >= p
    # x^3 + 2 not a square (no point), under both prefixes
    x = next(x for x in range(1, 100) if pow((x ** 3 + 2) % B.P, (B.P - 1) // 2, B.P) != 1)
    cases.append(good[6][:4] + b"\x02" + x.to_bytes(32, "big"))
    cases.append(good[6][:4] + b"\x03" + x.to_bytes(32, "big"))
    cases.append(good[7][:4] + bytes(33))                          # infinity: e(O, g2) != e(H, vk)
    cases.append(good[7][:4] + b"\x00" + b"\x01" + bytes(31))     # bad infinity encoding
    cases.append(good[8][:4] + bytes([good[8][4] ^ 1]) + good[8][5:])  # the other root's prefix
    kid = ctx.bls_load_keys(pk, vks)
    try:
        assert all(ctx.bls_key_status(kid, n))
        got = ctx.bls_verify_shares(kid, msg, cases)
    finally:
        ctx.bls_unload_keys(kid)
    H = B.g1_map(msg)
    exp = []
    for s in cases:
        i = int.from_bytes(s[:4], "big")
        try:
            p = B.g1_from_bytes(s[4:])
        except ValueError:
            exp.append(False)
            continue
        exp.append(1 <= i <= n and B.verify_share(H, p, B.g2_from_bytes(vks[i - 1])))
    assert got.tolist() == exp
    assert sum(exp) == n


@pytest.mark.parametrize("n,k", [(1, 1), (4, 3), (7, 5), (16, 11), (16, 16)])
def test_threshold_combine_byte_identical(ctx, n, k):
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=n * 100 + k)
    msg = bytes([n, k]) * 16
    rng = random.Random(n + k)
    ids = sorted(rng.sample(range(1, n + 1), k))
    sh = blsgen.shares(sks, ids, msg)
    comb = ctx.bls_combine(sh)
    want = B.g1_to_bytes(B.combine_threshold({i: B.parse_share(s)[1] for i, s in zip(ids, sh)}))
    assert comb == want == blsgen.sign_point(sk, msg)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        assert ctx.bls_verify(kid, msg, comb)
        assert not ctx.bls_verify(kid, msg + b"x", comb)
        assert not ctx.bls_verify(kid, msg, blsgen.doubled(b"\0\0\0\1" + comb)[4:])
    finally:
        ctx.bls_unload_keys(kid)


def test_multisig_combine_and_verify(ctx):
    n = 10
    sk, sks, pk, vks = blsgen.keyset(n, n, seed=5)
    msg = b"multisig digest 0123456789abcdef"
    ids = [1, 2, 4, 5, 7, 9, 10]
    sh = blsgen.shares(sks, ids, msg)
    comb = ctx.bls_combine(sh, multisig=True)
    acc = None
    for s in sh:
        acc = B.ec_add(acc, B.parse_share(s)[1], None)
    assert comb == B.g1_to_bytes(acc)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        assert ctx.bls_verify_multisig(kid, msg, comb, B.signers_bitmap(ids))
        assert not ctx.bls_verify_multisig(kid, msg, comb, B.signers_bitmap(ids[:-1]))
        assert not ctx.bls_verify_multisig(kid, b"other digest", comb, B.signers_bitmap(ids))
        # no signer: PK = infinity, the key wave releases the Miller-loop wave without lines
        assert not ctx.bls_verify_multisig(kid, msg, comb, bytes(256))
        assert ctx.bls_verify_multisig(kid, msg, comb, B.signers_bitmap(ids))  # context still sound
    finally:
        ctx.bls_unload_keys(kid)


def test_combine_rejects_duplicate_ids(ctx):
    sk, sks, pk, vks = blsgen.keyset(4, 3, seed=1)
    sh = blsgen.shares(sks, [1, 2], b"m" * 32)
    with pytest.raises(cb.CbftError):
        ctx.bls_combine([sh[0], sh[0], sh[1]])


def test_full_size_commit_certificate(ctx):
    # BASELINE config #4: n = 1024 replicas, k = 2f+1 = 683, 10% of the shares doubled
    n, k = 1024, 683
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=2024)
    msg = bytes(range(32))
    rng = random.Random(7)
    ids = sorted(rng.sample(range(1, n + 1), 760))
    sh = blsgen.shares(sks, ids, msg)
    bad = set(rng.sample(range(len(sh)), 76))
    for j in bad:
        sh[j] = blsgen.doubled(sh[j])
    kid = ctx.bls_load_keys(pk, vks)
    try:
        valid = ctx.bls_verify_shares(kid, msg, sh)
        assert valid.tolist() == [j not in bad for j in range(len(sh))]
        use = [s for j, s in enumerate(sh) if valid[j]][:k]
        comb = ctx.bls_combine(use)
        assert comb == blsgen.sign_point(sk, msg)
        assert ctx.bls_verify(kid, msg, comb)
    finally:
        ctx.bls_unload_keys(kid)


@pytest.mark.parametrize("optimistic", [True, False])
def test_combine_threshold_policy(ctx, optimistic):
    """cbft_bls_combine_threshold = SignaturesProcessingJob (CollectorOfThresholdSignatures.hpp:
    363-406): all-good shares combine optimistically with an empty bad set; with doubled shares
    the call falls back to per-share verification, reports exactly the bad ones and combines the
    valid ones; later duplicates of an id are ignored; too few valid shares -> not ok."""
    n, t = 16, 11
    sk, sks, pk, vks = blsgen.keyset(n, t, seed=33)
    msg = b"combine_threshold digest 0123456"
    rng = random.Random(3)
    ids = sorted(rng.sample(range(1, n + 1), 14))
    sh = blsgen.shares(sks, ids, msg)
    want = blsgen.sign_point(sk, msg)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        sig, ok, bad = ctx.bls_combine_threshold(kid, msg, sh, optimistic)
        assert ok and sig == want and not bad.any()
        badset = {1, 5, 9}
        mixed = [blsgen.doubled(s) if j in badset else s for j, s in enumerate(sh)]
        mixed.append(sh[0])  # a later duplicate of an id: ignored, not reported
        sig, ok, bad = ctx.bls_combine_threshold(kid, msg, mixed, optimistic)
        assert ok and sig == want
        assert bad.tolist() == [j in badset for j in range(len(mixed))]
        few = [blsgen.doubled(s) if j >= 9 else s for j, s in enumerate(sh)]  # 9 valid < t = 11
        sig, ok, bad = ctx.bls_combine_threshold(kid, msg, few, optimistic)
        assert not ok and bad.tolist() == [j >= 9 for j in range(len(few))]
        assert not ctx.bls_combine_threshold(kid, msg + b"x", sh, optimistic)[1]
    finally:
        ctx.bls_unload_keys(kid)


def test_sign_matches_oracle(ctx):
    # IThresholdSigner::signData: id (4 B big-endian) || sk * g1_map(msg) (BlsThresholdSigner.cpp:32-47)
    rng = random.Random(5)
    for sid, msg in ((1, b""), (7, bytes(32)), (2048, b"commit digest" * 3)):
        sk = rng.randrange(1, B.R)
        assert ctx.bls_sign(sk, sid, msg) == B.sign_share(sk, sid, msg)


def test_sum_keys_is_multisig_pk(ctx):
    # n-of-n multisig PK = sum of vk_i (BlsMultisigVerifier.cpp:33-38)
    n, k = 9, 9
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=21)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        for ids in (range(1, n + 1), [2, 5, 9], [4]):
            acc = None
            for i in ids:
                acc = B.ec_add(acc, B.g2_from_bytes(vks[i - 1]), None)
            assert ctx.bls_sum_keys(kid, B.signers_bitmap(ids)) == B.g2_to_bytes(acc)
    finally:
        ctx.bls_unload_keys(kid)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_combine_equals_combine(ctx, world):
    """cbft_bls_combine_partial over each rank's slice + cbft_bls_combine_finish == one combine
    (the multi-GPU path of cbft_multigpu.bls_combine_sharded, ranks simulated on one GPU)."""
    import cbft_multigpu as mg

    n, k = 24, 17
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=23)
    msg = bytes(range(40, 72))
    ids = random.Random(world).sample(range(1, n + 1), k)
    shares = blsgen.shares(sks, ids, msg)
    whole = ctx.bls_combine(shares)
    assert whole == blsgen.sign_point(sk, msg)
    parts = [ctx.bls_combine_partial(shares, *mg.share_slice(k, world, r)) for r in range(world)]
    assert all(len(p) == cb.BLS_G1_PARTIAL_BYTES for p in parts)
    assert ctx.bls_combine_finish(parts) == whole
    # multisig (unit scalars): sum of the shares
    parts_ms = [ctx.bls_combine_partial(shares, *mg.share_slice(k, world, r), multisig=True) for r in range(world)]
    assert ctx.bls_combine_finish(parts_ms) == ctx.bls_combine(shares, multisig=True)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_multisig_key_sum(ctx, world):
    import cbft_multigpu as mg

    n = 20
    sk, sks, pk, vks = blsgen.keyset(n, n, seed=29)
    msg = bytes(range(7, 39))
    signers = [1, 2, 5, 6, 7, 11, 13, 17, 19, 20]
    shares = blsgen.shares(sks, signers, msg)
    sig = ctx.bls_combine(shares, multisig=True)
    bm = B.signers_bitmap(signers)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        assert ctx.bls_verify_multisig(kid, msg, sig, bm)
        parts = [ctx.bls_sum_keys_partial(kid, bm, *mg.id_slice(n, world, r)) for r in range(world)]
        assert all(len(p) == cb.BLS_G2_PARTIAL_BYTES for p in parts)
        assert ctx.bls_verify_multisig_partials(msg, sig, parts)
        assert not ctx.bls_verify_multisig_partials(bytes(32), sig, parts)
        # a signer missing from the key sum -> reject
        bm2 = B.signers_bitmap(signers[:-1])
        parts2 = [ctx.bls_sum_keys_partial(kid, bm2, *mg.id_slice(n, world, r)) for r in range(world)]
        assert not ctx.bls_verify_multisig_partials(msg, sig, parts2)
    finally:
        ctx.bls_unload_keys(kid)


def _bad_g2_keys():
    """Encodings bls_keys_wave_kernel must reject exactly as g2_decompress does (the one-lane
    kernel and the oracle): bad prefix, x >= p, an x off E', a point of E'(Fp2) outside the
    order-r subgroup, and infinity (decodes, but a threshold key of infinity is unusable)."""
    x = 1
    while B.f2_sqrt(B.F2(x, 1) * B.F2(x, 1) * B.F2(x, 1) + B.B2) is not None:  # x^3 + b' a non-square: off the curve
        x += 1
    off_curve = b"\x02" + x.to_bytes(32, "big") + (1).to_bytes(32, "big")
    x = 1
    while True:  # a twist point: E'(Fp2) has order r * h2, so [r]Q != O for this x
        y = B.f2_sqrt(B.F2(x, 2) * B.F2(x, 2) * B.F2(x, 2) + B.B2)
        if y is not None:
            pt = (B.F2(x, 2), y)
            if B.ec_mul(B.R, pt) is not None:
                break
        x += 1
    return {"prefix": b"\x05" + bytes(64), "x_ge_p": b"\x02" + B.P.to_bytes(32, "big") + bytes(32),
            "off_curve": off_curve, "not_in_g2": B.g2_to_bytes(pt), "infinity": bytes(65)}


def test_key_decoding_edge_cases_and_lines(ctx):
    """Key status of a set mixing valid and invalid verification keys equals the oracle's decode
    (infinity excepted: unusable), and the lines built for the valid ones verify their shares
    while every share under an invalid key is rejected."""
    n, k = 12, 8
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=29)
    bad = _bad_g2_keys()
    slots = {2: "prefix", 5: "x_ge_p", 7: "off_curve", 9: "not_in_g2", 11: "infinity"}
    vks = list(vks)
    for i, name in slots.items():
        vks[i - 1] = bad[name]
    for name, enc in bad.items():
        if name == "infinity":
            assert B.g2_from_bytes(enc) is None
        else:
            with pytest.raises(ValueError):
                B.g2_from_bytes(enc)
    msg = bytes(range(7, 39))
    good = blsgen.shares(sks, range(1, n + 1), msg)
    kid = ctx.bls_load_keys(pk, vks)
    try:
        status = ctx.bls_key_status(kid, n)
        got = ctx.bls_verify_shares(kid, msg, good)
    finally:
        ctx.bls_unload_keys(kid)
    assert status[0] == 1  # the group key
    assert [bool(s) for s in status[1:]] == [i not in slots for i in range(1, n + 1)]
    assert got.tolist() == [i not in slots for i in range(1, n + 1)]


def test_generator_and_key_lines_verify_full_keyset(ctx):
    """A 1,024-key set (the config #4 size, one wave pair per key): all keys decode, and a share
    of every 64th signer verifies while a doubled one does not."""
    n, k = 1024, 683
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=31)
    msg = bytes(32)
    ids = list(range(1, n + 1, 64)) + [n]
    good = blsgen.shares(sks, ids, msg)
    cases = good + [blsgen.doubled(good[0]), blsgen.doubled(good[-1])]
    kid = ctx.bls_load_keys(pk, vks)
    try:
        assert all(ctx.bls_key_status(kid, n))
        got = ctx.bls_verify_shares(kid, msg, cases)
    finally:
        ctx.bls_unload_keys(kid)
    assert got.tolist() == [True] * len(good) + [False, False]


def test_sum_keys_exceptional_cases(ctx):
    """The wave key sum's exact group law: a key repeated (the addition turns into a doubling),
    a key and its negation (the partial sum hits infinity, then continues), a sum that ends at
    infinity, a selected key that did not decode (sum unusable), over 1,024 keys so the sum
    runs over several blocks and levels."""
    n = 1024
    sk, sks, pk, vks = blsgen.keyset(n, 2, seed=37)
    vks = list(vks)
    neg = lambda e: bytes([e[0] ^ 1]) + e[1:]  # noqa: E731  (-P: the y sign bit flipped)
    vks[3] = vks[2]            # id 4 = id 3
    vks[5] = neg(vks[4])       # id 6 = -id 5
    vks[700] = neg(vks[699])   # id 701 = -id 700, in another block
    vks[900] = b"\x05" + bytes(64)  # id 901 does not decode
    pts = [B.g2_from_bytes(v) if i != 900 else None for i, v in enumerate(vks)]
    kid = ctx.bls_load_keys(pk, vks)
    try:
        cases = [[3, 4], [5, 6], [3, 4, 5, 6, 7], [700, 701], list(range(1, 17)), list(range(1, 901)),
                 [i for i in range(1, n + 1) if i % 3 and i != 901], list(range(2, 700, 7))]
        for ids in cases:
            acc = None
            for i in ids:
                acc = B.ec_add(acc, pts[i - 1], None)
            assert ctx.bls_sum_keys(kid, B.signers_bitmap(ids)) == B.g2_to_bytes(acc), ids[:8]
        bm = B.signers_bitmap([1, 2, 901])
        assert ctx.bls_sum_keys(kid, bm) == bytes(65)  # a selected key that did not decode
    finally:
        ctx.bls_unload_keys(kid)


@pytest.mark.parametrize("devices", [[0, 0], [0] * 4])
def test_multi_device_share_verification(ctx, devices):
    """cbft_open_devices: the key set on every device, the shares cut into one contiguous slice
    per device and verified concurrently -- the merged bitmap equals the single-device one
    (on one GPU the devices repeat, each child with its own streams)."""
    n, k = 40, 27
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=41)
    msg = bytes(range(3, 35))
    good = blsgen.shares(sks, range(1, n + 1), msg)
    cases = list(good)
    for j in (0, 7, 13, 21, 39):
        cases[j] = blsgen.doubled(good[j])  # bad shares spread over the slices
    cases.append((n + 1).to_bytes(4, "big") + good[1][4:])  # id out of range
    kid = ctx.bls_load_keys(pk, vks)
    try:
        want = ctx.bls_verify_shares(kid, msg, cases)
    finally:
        ctx.bls_unload_keys(kid)
    with cb.Context(devices=devices) as g:
        gk = g.bls_load_keys(pk, vks)
        try:
            assert all(g.bls_key_status(gk, n))
            got = g.bls_verify_shares(gk, msg, cases)
            assert got.tolist() == want.tolist()
            assert sum(want) == n - 5
            sig, ok, bad = g.bls_combine_threshold(gk, msg, cases, optimistic=True)
            assert ok and sig == blsgen.sign_point(sk, msg)
        finally:
            g.bls_unload_keys(gk)


def test_keyset_rotation_per_checkpoint_window(ctx):
    """Per-checkpoint-window threshold systems (CryptoManager.hpp:62-78,116-141): get(sn) picks the
    system of the last checkpoint <= (sn-1)/W.  Window w+1's key set is loaded while window w's
    certificates are being verified and combined on another thread, and window w-1's is unloaded
    once its certificates are done.  Every certificate must verify, report exactly its doubled
    shares and combine to sk_w * H(m) under its own window's keys, and fail under the next one."""
    import hashlib
    import threading
    from concurrent.futures import ThreadPoolExecutor

    W, n, k, windows = 150, 64, 43, 4
    systems = [blsgen.keyset(n, k, seed=900 + w) for w in range(windows)]
    certs = []
    for w, (sk, sks, pk, vks) in enumerate(systems):
        rng = random.Random(w)
        cw = []
        for j in range(5):
            sn = w * W + 1 + 30 * j
            msg = hashlib.sha256(b"cert %d" % sn).digest()
            sh = blsgen.shares(sks, sorted(rng.sample(range(1, n + 1), k + 4)), msg)
            bad = set(rng.sample(range(len(sh)), 2))
            sh = [blsgen.doubled(s) if i in bad else s for i, s in enumerate(sh)]
            cw.append((sn, msg, sh, bad, blsgen.sign_point(sk, msg)))
        certs.append(cw)

    lock = threading.Lock()
    loaded = {0: ctx.bls_load_keys(systems[0][2], systems[0][3])}
    ready = [threading.Event() for _ in range(windows)]
    started = [threading.Event() for _ in range(windows)]
    done = [threading.Event() for _ in range(windows)]
    ready[0].set()

    def get(sn):
        chk = (sn - 1) // W
        with lock:
            c = max(c for c in loaded if c <= chk)
            return c, loaded[c]

    def loader():
        for w in range(1, windows):
            assert started[w - 1].wait(120)  # window w-1's certificates are in flight
            kid = ctx.bls_load_keys(systems[w][2], systems[w][3])
            assert all(ctx.bls_key_status(kid, n))
            with lock:
                loaded[w] = kid
            ready[w].set()
            if w >= 2:
                assert done[w - 2].wait(120)
                with lock:
                    old = loaded.pop(w - 2)
                ctx.bls_unload_keys(old)

    def certify(w):
        assert ready[w].wait(120)
        for j, (sn, msg, sh, bad, want) in enumerate(certs[w]):
            c, kid = get(sn)
            assert c == w
            valid = ctx.bls_verify_shares(kid, msg, sh)
            assert valid.tolist() == [i not in bad for i in range(len(sh))]
            sig, ok, badmask = ctx.bls_combine_threshold(kid, msg, sh, optimistic=j % 2 == 0)
            assert ok and sig == want and set(np.flatnonzero(badmask).tolist()) == bad
            assert ctx.bls_verify(kid, msg, sig)
            started[w].set()
        if w + 1 < windows:  # the next window's keys reject this window's shares and signature
            assert ready[w + 1].wait(120)
            with lock:
                nxt = loaded[w + 1]
            sn, msg, sh, bad, want = certs[w][0]
            assert not ctx.bls_verify_shares(nxt, msg, sh).any()
            assert not ctx.bls_verify(nxt, msg, want)
        done[w].set()

    try:
        with ThreadPoolExecutor(max_workers=windows + 1) as ex:
            futs = [ex.submit(loader)] + [ex.submit(certify, w) for w in range(windows)]
            for f in futs:
                f.result(timeout=300)
        assert sorted(loaded) == [windows - 2, windows - 1]
    finally:
        for kid in loaded.values():
            ctx.bls_unload_keys(kid)


def test_sign_row_ladder_edge_scalars(ctx):
    """The row-parallel signature (GLV halves, odd-digit windows, selects instead of branches)
    equals the oracle's sk * g1_map(msg) on scalars that stress the decomposition: 1, 2, 3, r - 1,
    r - 2, 2^127 +- 1, 2^128, both nontrivial cube roots w of unity mod r and w +- 1 (a GLV half
    is 0 or +-1), and random keys (even and odd halves of both signs)."""
    g = 2
    while pow(g, (B.R - 1) // 3, B.R) == 1:
        g += 1
    w = pow(g, (B.R - 1) // 3, B.R)
    assert (w * w + w + 1) % B.R == 0
    scal = [1, 2, 3, B.R - 1, B.R - 2, (1 << 127) - 1, 1 << 127, (1 << 127) + 1, 1 << 128, (1 << 200) + 12345]
    for lam in (w, w * w % B.R):
        scal += [lam, lam + 1, lam - 1, (2 * lam) % B.R, B.R - lam]
    rng = random.Random(99)
    scal += [rng.randrange(1, B.R) for _ in range(24)]
    msgs = [b"", b"x" * 70, bytes(range(32))]
    for i, sk in enumerate(scal):
        m = msgs[i % 3]
        assert ctx.bls_sign(sk, 1 + i, m) == B.sign_share(sk, 1 + i, m), (i, hex(sk))
    # keys outside [1, r): reduced mod r (sk * H has order r), 0 mod r refused
    for sk in (B.R + 1, B.R + 2, 2 * B.R - 1, (1 << 256) - 1):
        assert ctx.bls_sign(sk, 7, b"m") == B.sign_share(sk % B.R, 7, b"m"), hex(sk)
    for sk in (0, B.R, 2 * B.R):
        with pytest.raises(cb.CbftError):
            ctx.bls_sign(sk, 7, b"m")


def test_public_key_comb_edge_scalars(ctx):
    """vk = sk * g2 by the fixed-base comb (odd digits, selects): equal to the oracle's sk * g2 for
    scalars at the recoding's edges (1, 2, 15, 16, 17, 2^252, r - 1, r - 2, even and odd) and random
    keys, and the same key twice gives the same bytes (the lazily built table is reused)."""
    rng = random.Random(123)
    scal = [1, 2, 3, 15, 16, 17, 255, 256, 1 << 252, (1 << 253) + 1, B.R - 1, B.R - 2, B.R - 16]
    scal += [rng.randrange(1, B.R) for _ in range(12)]
    for sk in scal:
        exp = B.g2_to_bytes(B.ec_mul(sk, B.G2_GEN))
        assert ctx.bls_public_key(sk) == exp, hex(sk)
    assert ctx.bls_public_key(scal[-1]) == B.g2_to_bytes(B.ec_mul(scal[-1], B.G2_GEN))
    for sk in (B.R + 1, B.R + 16, 5 * B.R + 3, (1 << 256) - 1):
        assert ctx.bls_public_key(sk) == B.g2_to_bytes(B.ec_mul(sk % B.R, B.G2_GEN)), hex(sk)
    for sk in (0, B.R, 3 * B.R):
        with pytest.raises(cb.CbftError):
            ctx.bls_public_key(sk)
