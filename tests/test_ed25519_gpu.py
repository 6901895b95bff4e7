"""GPU parity tests: libcbft_hipcrypto (HIP, gfx950) against the golden OpenSSL verdicts, the
plain-C oracle and the host OpenSSL, through the C ABI.  Bit-exact verdicts are the bar."""
import ctypes
import os

import numpy as np
import pytest

import cbft_hipcrypto as cb
from golden_io import load_ed25519_vectors
import workload as sigsets

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    c = cb.Context(device=0, max_batch=1 << 16)
    yield c
    c.close()


@pytest.fixture(scope="module")
def golden():
    return load_ed25519_vectors()


def _bools(bitmap, n):
    return cb.bitmap_to_bools(bitmap, n)


def test_golden_per_signature_keys(ctx, golden):
    n = len(golden)
    got = _bools(ctx.verify_pk([v.pk for v in golden], [v.sig for v in golden], [v.msg for v in golden]), n)
    exp = np.array([bool(v.verdict) for v in golden])
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first: {[(int(i), golden[i].cls) for i in bad[:10]]}"


def test_golden_key_table(ctx, golden):
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    tid = ctx.load_keys(keys)
    try:
        n = len(golden)
        got = _bools(ctx.verify(tid, [index[v.pk] for v in golden], [v.sig for v in golden],
                                [v.msg for v in golden]), n)
        exp = np.array([bool(v.verdict) for v in golden])
        assert np.array_equal(got, exp)
    finally:
        ctx.unload_keys(tid)


@pytest.mark.parametrize("radix", [8, 9, 10, 12, 13, 14, 15])
def test_golden_key_table_radix(ctx, golden, radix):
    """Every comb radix gives the golden verdicts (the default radix is covered above)."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    tid = ctx.load_keys(keys, radix=radix)
    try:
        n = len(golden)
        got = _bools(ctx.verify(tid, [index[v.pk] for v in golden], [v.sig for v in golden],
                                [v.msg for v in golden]), n)
        exp = np.array([bool(v.verdict) for v in golden])
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    finally:
        ctx.unload_keys(tid)


@pytest.mark.parametrize("b_radix", [16, 17, 20, 24, 26])
@pytest.mark.parametrize("radix", [8, 13])
def test_golden_base_table_radix(golden, b_radix, radix):
    """B's comb radix (CBFT_OPT_B_RADIX; the default 22 is covered above): the ladder's lane split
    changes with it (radix-2^13 keys: 9 additions per lane at B radix 16, 9 at 17, 9 at 20, 8 at 22,
    8 at 24, 8 at 26; radix 26 is a 42.9 GB table of 10 positions)."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    with cb.Context(device=0) as c:
        c.set_option(cb.OPT_B_RADIX, b_radix)
        tid = c.load_keys(keys, radix=radix)
        n = len(golden)
        got = _bools(c.verify(tid, [index[v.pk] for v in golden], [v.sig for v in golden],
                              [v.msg for v in golden]), n)
    exp = np.array([bool(v.verdict) for v in golden])
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("b_radix", [24, 26])
def test_pair_ladder_wide_base_table(b_radix):
    """The pair ladder (batches from 32K) over B radix 2^24 / 2^26: 31 / 30 additions dealt to two
    lanes (16 / 15 each), 10 % invalid signatures, verdicts equal to OpenSSL's."""
    ss = sigsets.make_sigset(40000, nkeys=64, msg_len=256, seed=0xB26 + b_radix, invalid_frac=0.1)
    with cb.Context(device=0, max_batch=40000) as c:
        c.set_option(cb.OPT_B_RADIX, b_radix)
        tid = c.load_keys(ss.pk, radix=13)
        got = _bools(c.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), 40000)
    assert np.array_equal(got, ss.expected), np.nonzero(got != ss.expected)[0][:10]


def test_load_keys_bad_radix(ctx):
    lib = ctx.lib
    tid = ctypes.c_uint32()
    key = (ctypes.c_uint8 * 32)()
    for r in (7, 16, -1):
        assert lib.cbft_ed25519_load_keys_ex(ctx.handle, key, 1, r, ctypes.byref(tid)) == -22


@pytest.mark.parametrize("n", [1, 7, 63, 64, 65, 200, 1000])
def test_ragged_batch_sizes(ctx, golden, n):
    vs = [golden[i % len(golden)] for i in range(n)]
    bm = ctx.verify_pk([v.pk for v in vs], [v.sig for v in vs], [v.msg for v in vs])
    assert len(bm) == (n + 7) // 8
    got = _bools(bm, n)
    assert np.array_equal(got, np.array([bool(v.verdict) for v in vs]))
    if n % 8:
        assert bm[-1] >> (n % 8) == 0  # bits past n are zero


@pytest.mark.parametrize("n", [8191, 8192, 8193, 20000])
def test_host_staging_boundary(ctx, n):
    # host-buffer batches whose pageable inputs fit CBFT_PACK_MAX go through one packed pinned
    # staging copy, larger ones through per-array copies (cbft_hipcrypto.cpp): both sides of it,
    # key-table and per-signature keys, mixed lengths with 10 % invalid
    ss = sigsets.make_sigset(n, nkeys=97, msg_len=(1, 700), seed=n, invalid_frac=0.10)
    tid = ctx.load_keys(ss.pk)
    try:
        got = _bools(ctx.verify(tid, ss.key_idx, ss.sig, ss.msgs()), n)
    finally:
        ctx.unload_keys(tid)
    assert np.array_equal(got, ss.expected)
    got2 = _bools(ctx.verify_pk(ss.per_sig_pk(), ss.sig, ss.msgs()), n)
    assert np.array_equal(got2, ss.expected)


def test_empty_batch(ctx):
    assert ctx.verify_pk([], [], []) == b""


def test_verdict_independent_of_batch_composition(ctx, golden):
    vs = golden[:300]
    full = _bools(ctx.verify_pk([v.pk for v in vs], [v.sig for v in vs], [v.msg for v in vs]), len(vs))
    rev = _bools(ctx.verify_pk([v.pk for v in vs[::-1]], [v.sig for v in vs[::-1]], [v.msg for v in vs[::-1]]),
                 len(vs))
    assert np.array_equal(full, rev[::-1])


def test_mixed_lengths_with_invalid_vs_openssl_and_oracle(ctx):
    # config #3 shape (SigManager mixed batch), reduced: 64..4096 B, 10 % adversarially invalid
    ss = sigsets.make_sigset(3000, nkeys=257, msg_len=(64, 4096), seed=7, invalid_frac=0.10)
    tid = ctx.load_keys(ss.pk)
    try:
        got = _bools(ctx.verify(tid, ss.key_idx, ss.sig, ss.msgs()), ss.n)
    finally:
        ctx.unload_keys(tid)
    assert np.array_equal(got, ss.expected)
    assert (~ss.expected).sum() > 200
    # the plain-C oracle agrees on a sample
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "libcbft_oracle.so"))
    out = np.zeros(200, dtype=np.uint8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib.cbft_oracle_ed25519_verify_many(p(ss.pk), p(ss.key_idx), p(ss.sig), p(ss.blob), p(ss.off), p(ss.len),
                                        ctypes.c_size_t(200), p(out))
    assert np.array_equal(out.astype(bool), ss.expected[:200])


def test_full_size_64k_key_table_and_per_sig(ctx):
    # config #2 at full size: 64K sigs x 256 B, 4096 keys; every 97th signature corrupted
    ss = sigsets.make_sigset(65536, nkeys=4096, msg_len=256, seed=11)
    bad = np.arange(0, ss.n, 97)
    ss.sig[bad, 40] ^= 0x01
    ss.expected = sigsets.cpu_verify(ss).astype(bool)
    assert (~ss.expected).sum() == bad.size
    tid = ctx.load_keys(ss.pk)
    try:
        got = _bools(ctx.verify(tid, ss.key_idx, ss.sig, ss.msgs()), ss.n)
    finally:
        ctx.unload_keys(tid)
    assert np.array_equal(got, ss.expected)
    got2 = _bools(ctx.verify_pk(ss.per_sig_pk(), ss.sig, ss.msgs()), ss.n)
    assert np.array_equal(got2, ss.expected)


def test_invalid_arguments(ctx):
    lib = cb.load_library()
    assert lib.cbft_ed25519_unload_keys(ctx.handle, 123456) == -22
    out = (ctypes.c_uint8 * 1)()
    rc = lib.cbft_ed25519_verify_batch(ctx.handle, 999, None, None, None, None, None, 1, out)
    assert rc == -22
    tid = ctx.load_keys([bytes(32)])
    try:
        idx = np.array([5], dtype=np.uint32)  # out of range key index
        sig = np.zeros(64, dtype=np.uint8)
        off = np.zeros(1, dtype=np.uint64)
        ln = np.zeros(1, dtype=np.uint32)
        blob = np.zeros(1, dtype=np.uint8)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = lib.cbft_ed25519_verify_batch(ctx.handle, tid, p(idx), p(sig), p(blob), p(off), p(ln), 1, out)
        assert rc == -22
    finally:
        ctx.unload_keys(tid)


def test_fresh_context_without_presizing(golden):
    # regression: buffers sized lazily on the first call (max_batch = 0)
    with cb.Context(device=0) as c:
        vs = golden[:256]
        got = _bools(c.verify_pk([v.pk for v in vs], [v.sig for v in vs], [v.msg for v in vs]), len(vs))
        assert np.array_equal(got, np.array([bool(v.verdict) for v in vs]))
        vs = golden  # grow
        got = _bools(c.verify_pk([v.pk for v in vs], [v.sig for v in vs], [v.msg for v in vs]), len(vs))
        assert np.array_equal(got, np.array([bool(v.verdict) for v in vs]))


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 127, 128, 129, 1145])
def test_finish_tree_both_forms(golden, k, n):
    # The tree finish: one inversion per block of 64 lanes x K signatures (Montgomery's trick over
    # an LDS product tree, the root inverted on the scalar unit); rejected items (S >= L,
    # undecodable A) enter the product as 1.  Both K (1 below 16K signatures, 2 from 16K) on the
    # golden set and its prefixes: partial blocks, a lone lane, a block boundary +- 1.
    sub = golden[:n]
    with cb.Context(device=0) as c:
        c.set_option(cb.OPT_FINISH_K, k)
        got = _bools(c.verify_pk([v.pk for v in sub], [v.sig for v in sub], [v.msg for v in sub]), len(sub))
    assert np.array_equal(got, np.array([bool(v.verdict) for v in sub]))


def test_finish_k2_full_golden(golden):
    with cb.Context(device=0) as c:
        c.set_option(cb.OPT_FINISH_K, 2)
        got = _bools(c.verify_pk([v.pk for v in golden], [v.sig for v in golden], [v.msg for v in golden]),
                     len(golden))
    assert np.array_equal(got, np.array([bool(v.verdict) for v in golden]))


class _Hip:
    """Device buffers and streams from the HIP runtime libcbft_hipcrypto itself links (torch ships
    its own HIP runtime; a second runtime in the same process sees no GPUs once the first owns it)."""

    def __init__(self):
        cb.load_library()
        self.lib = ctypes.CDLL("libamdhip64.so.7")  # the soname libcbft_hipcrypto loaded
        self.bufs, self.streams = [], []

    def _ok(self, rc, what):
        assert rc == 0, f"{what}: hipError {rc}"

    def to_dev(self, a: np.ndarray) -> int:
        p = ctypes.c_void_p()
        self._ok(self.lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(a.nbytes, 1))), "hipMalloc")
        self.bufs.append(p.value)
        a = np.ascontiguousarray(a)
        self._ok(self.lib.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1), "hipMemcpy")
        return p.value

    def from_dev(self, ptr: int, nbytes: int) -> bytes:
        out = np.zeros(nbytes, dtype=np.uint8)
        self._ok(self.lib.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes),
                                    2), "hipMemcpy")
        return out.tobytes()

    def stream(self) -> int:
        s = ctypes.c_void_p()
        self._ok(self.lib.hipStreamCreate(ctypes.byref(s)), "hipStreamCreate")
        self.streams.append(s.value)
        return s.value

    def sync(self):
        self._ok(self.lib.hipDeviceSynchronize(), "hipDeviceSynchronize")

    def close(self):
        self.sync()
        for s in self.streams:
            self.lib.hipStreamDestroy(ctypes.c_void_p(s))
        for b in self.bufs:
            self.lib.hipFree(ctypes.c_void_p(b))


@pytest.mark.parametrize("order", ["1", "0"])
def test_device_path_two_streams_stage_order(order):
    # the bench's schedule: device-resident batches alternating over two streams, the library's
    # cross-batch stage order (hash after hash, ladder after ladder) and two rotating work slots.
    # Batches with different corruption patterns must each keep their own verdicts.
    hip = _Hip()
    n = 65536
    nwords = (n + 63) // 64
    base = sigsets.make_sigset(n, nkeys=512, msg_len=256, seed=23)
    variants = []
    for v in range(3):
        sig = base.sig.copy()
        bad = np.arange(v, n, 89 + 10 * v)
        sig[bad, 33 + v] ^= 0x40
        exp = np.ones(n, dtype=bool)
        exp[bad] = False
        variants.append((hip.to_dev(sig.reshape(-1)), exp))
    try:
        with cb.Context(device=0, max_batch=n) as c:
            c.set_option(cb.OPT_STAGE_ORDER, int(order))
            tid = c.load_keys(base.pk)
            d_kidx = hip.to_dev(base.key_idx)
            d_blob = hip.to_dev(base.blob)
            d_off = hip.to_dev(base.off)
            d_len = hip.to_dev(base.len)
            streams = [hip.stream(), hip.stream()]
            outs = [hip.to_dev(np.zeros(nwords, dtype=np.uint64)) for _ in range(6)]
            for b in range(6):
                c.verify_device(tid, 0, d_kidx, variants[b % 3][0], d_blob, d_off, d_len, n, outs[b], streams[b % 2])
            hip.sync()
            for b in range(6):
                got = _bools(hip.from_dev(outs[b], nwords * 8), n)
                assert np.array_equal(got, variants[b % 3][1]), f"batch {b}"
            c.unload_keys(tid)
    finally:
        hip.close()


@pytest.mark.parametrize("streams,slots,early", [(4, 4, "1"), (4, 4, "0"), (3, 2, "1"), (2, 4, "1")])
def test_device_path_mixed_lengths_many_streams(streams, slots, early):
    # config #3's device-resident schedule: variable-length batches (sorted hash, long-message
    # tail on the slot's aux stream) over several streams and work slots; with
    # CBFT_OPT_HASH_ORDER_EARLY the next batch's hash waits only for this batch's short hashes.  Every
    # batch keeps its own verdicts (different corruption per batch, a slot reused while the
    # previous tail may still run).
    hip = _Hip()
    n = 16384
    nwords = (n + 63) // 64
    base = sigsets.make_sigset(n, nkeys=256, msg_len=(64, 4096), seed=31, invalid_frac=0.05)
    variants = []
    for v in range(3):
        sig = base.sig.copy()
        bad = np.arange(v, n, 61 + 7 * v)
        sig[bad, 40 + v] ^= 0x10
        exp = base.expected.copy()
        exp[bad] = False
        variants.append((hip.to_dev(sig.reshape(-1)), exp))
    try:
        with cb.Context(device=0, max_batch=n) as c:
            c.set_option(cb.OPT_WORK_SLOTS, slots).set_option(cb.OPT_HASH_ORDER_EARLY, int(early))
            tid = c.load_keys(base.pk)
            d_kidx = hip.to_dev(base.key_idx)
            d_blob = hip.to_dev(base.blob)
            d_off = hip.to_dev(base.off)
            d_len = hip.to_dev(base.len)
            ss = [hip.stream() for _ in range(streams)]
            nb = 9
            outs = [hip.to_dev(np.zeros(nwords, dtype=np.uint64)) for _ in range(nb)]
            for b in range(nb):
                c.verify_device(tid, 0, d_kidx, variants[b % 3][0], d_blob, d_off, d_len, n, outs[b], ss[b % streams])
            hip.sync()
            for b in range(nb):
                got = _bools(hip.from_dev(outs[b], nwords * 8), n)
                assert np.array_equal(got, variants[b % 3][1]), f"batch {b}"
            c.unload_keys(tid)
    finally:
        hip.close()


def test_per_batch_profiling_ring(golden):
    # cbft_set_profiling(ctx, 2): each verify keeps its own stage events; the average covers
    # exactly the batches since enabling, and verdicts are unchanged by the instrumentation
    with cb.Context(device=0) as c:
        vs = golden[:512]
        exp = np.array([bool(v.verdict) for v in vs])
        c.set_profiling(True, per_batch=True)
        for _ in range(3):
            got = _bools(c.verify_pk([v.pk for v in vs], [v.sig for v in vs], [v.msg for v in vs]), len(vs))
            assert np.array_equal(got, exp)
        stage, cnt = c.stage_times_avg_ms()
        assert cnt == 3
        assert all(v > 0 for v in stage.values())
        c.set_profiling(False)
        with pytest.raises(cb.CbftError):
            c.stage_times_avg_ms()
        lib = cb.load_library()
        assert lib.cbft_set_profiling(c.handle, 3) == -22


@pytest.mark.parametrize("radix,b_radix", [(8, 22), (11, 22), (13, 16), (13, 22), (15, 22), (14, 24)])
def test_pair_ladder_golden_geometries(golden, radix, b_radix):
    """The pair ladder over the golden set at several key / B comb geometries: each lane's first
    addition is a point set from the identity, whichever table (a key position or B) and digit
    sign (including the identity entry of a zero digit) it starts on."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    with cb.Context(device=0) as c:
        c.set_option(cb.OPT_LADDER_LANES, 2).set_option(cb.OPT_B_RADIX, b_radix)
        tid = c.load_keys(keys, radix=radix)
        got = _bools(c.verify(tid, [index[v.pk] for v in golden], [v.sig for v in golden],
                              [v.msg for v in golden]), len(golden))
    exp = np.array([bool(v.verdict) for v in golden])
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("lanes", ["2", "4"])
def test_ladder_layouts_both_sizes(golden, lanes):
    """Each comb-ladder layout (CBFT_OPT_LADDER_LANES) at the sizes the default does not pick it
    for: the pair ladder on the small golden batch, the quad ladder on a 64K batch."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    with cb.Context(device=0, max_batch=1 << 16) as c:
        c.set_option(cb.OPT_LADDER_LANES, int(lanes))
        tid = c.load_keys(keys)
        got = _bools(c.verify(tid, [index[v.pk] for v in golden], [v.sig for v in golden],
                              [v.msg for v in golden]), len(golden))
        assert np.array_equal(got, np.array([bool(v.verdict) for v in golden]))
        ss = sigsets.make_sigset(1 << 16, nkeys=64, msg_len=256, seed=77, threads=16, invalid_frac=0.05)
        tid2 = c.load_keys(ss.pk)
        got = _bools(c.verify_packed(tid2, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), 1 << 16)
        assert np.array_equal(got, ss.expected)


def test_config3_full_shape(ctx):
    """BASELINE config #3 at full size: 65,536 signatures from 4,096 clients, message lengths
    log-uniform in 64..4,096 B (variable-length SHA-512: 2..33 blocks), 10 % adversarially invalid;
    verdicts equal host OpenSSL's on every signature."""
    ss = sigsets.make_sigset(65536, nkeys=4096, msg_len=(64, 4096), seed=3, invalid_frac=0.10, threads=16)
    tid = ctx.load_keys(ss.pk)
    try:
        got = _bools(ctx.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), ss.n)
    finally:
        ctx.unload_keys(tid)
    assert np.array_equal(got, ss.expected)
    assert 0.05 < (~ss.expected).mean() < 0.15


@pytest.mark.parametrize("chunk", [1, 15, 16, 17, 64, 65, 300, 1024])
def test_golden_small_batches_fused_kernel(ctx, golden, chunk):
    """Key-table batches up to 1,024 signatures run as ONE fused launch (ed25519_small3_kernel:
    hash + quad comb + R decode on four waves, 8 signatures per block, 8-bit verdict pieces): the
    golden set in batches of `chunk` gives the golden verdicts, equal to the three-kernel path
    (CBFT_OPT_SMALL_MAX = 0) batch for batch, including partial words and tail quads."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    exp = np.array([bool(v.verdict) for v in golden])
    three = cb.Context(device=0).set_option(cb.OPT_SMALL_MAX, 0)
    tid, tid3 = ctx.load_keys(keys), three.load_keys(keys)
    try:
        for lo in range(0, len(golden), chunk):
            part = golden[lo:lo + chunk]
            args = ([index[v.pk] for v in part], [v.sig for v in part], [v.msg for v in part])
            got = _bools(ctx.verify(tid, *args), len(part))
            ref = _bools(three.verify(tid3, *args), len(part))
            assert np.array_equal(got, exp[lo:lo + chunk]), f"fused kernel, batch at {lo}"
            assert np.array_equal(ref, got), f"three-kernel path disagrees at {lo}"
    finally:
        ctx.unload_keys(tid)
        three.unload_keys(tid3)
        three.close()


@pytest.mark.parametrize("n,msg_len", [(1, 256), (9, 256), (17, 256), (47, 256), (64, 256), (65, 256), (130, 256),
                                       (5000, 256), (5000, (1, 2048)), (5000, 2048), (13000, 2048)])
def test_device_path_small_batch_whole_words(n, msg_len):
    """cbft_ed25519_verify_batch_device writes ceil(n/64) WHOLE 64-bit verdict words, bits past n
    = 0, also when the batch runs as the fused small kernel (8-signature pieces per block): the
    buffer is pre-filled with 0xFF, so a piece no block covers would show up as stray accept bits.
    n = 5,000: the three-kernel path with the device-side hash sort (one block count for all
    messages: the uniform flag keeps the identity order; random lengths: the permutation); 2,048-B
    messages are long (ed25519_hash_long_kernel): all of 5,000, or the last 64 x 192 of 13,000."""
    hip = _Hip()
    nwords = (n + 63) // 64
    ss = sigsets.make_sigset(n, nkeys=7, msg_len=msg_len, seed=900 + n, invalid_frac=0.2)
    try:
        with cb.Context(device=0) as c:
            tid = c.load_keys(ss.pk)
            d_kidx, d_sig = hip.to_dev(ss.key_idx), hip.to_dev(ss.sig.reshape(-1))
            d_blob, d_off, d_len = hip.to_dev(ss.blob), hip.to_dev(ss.off), hip.to_dev(ss.len)
            out = hip.to_dev(np.full(nwords + 1, 0xFFFFFFFFFFFFFFFF, dtype=np.uint64))
            c.verify_device(tid, 0, d_kidx, d_sig, d_blob, d_off, d_len, n, out, None)
            hip.sync()
            words = np.frombuffer(hip.from_dev(out, (nwords + 1) * 8), dtype=np.uint64)
            bits = np.unpackbits(words[:nwords].view(np.uint8), bitorder="little").astype(bool)
            assert np.array_equal(bits[:n], ss.expected)
            assert not bits[n:].any(), "stale bits past n in the last verdict word"
            assert words[nwords] == np.uint64(0xFFFFFFFFFFFFFFFF), "wrote past ceil(n/64) words"
            c.unload_keys(tid)
    finally:
        hip.close()


@pytest.mark.parametrize("n", [1, 9, 1000, 5000])
def test_fixed_device_path(n):
    """cbft_ed25519_verify_fixed_device (message i at d_msg + i * L) gives the verdicts of the
    variable-length device call and of OpenSSL, on the fused small kernel (n <= 1,024) and the
    three-kernel path, whole verdict words."""
    hip = _Hip()
    nwords = (n + 63) // 64
    L = 200
    ss = sigsets.make_sigset(n, nkeys=5, msg_len=L, seed=4200 + n, invalid_frac=0.2)
    assert np.array_equal(ss.off, np.arange(n, dtype=ss.off.dtype) * L)
    try:
        with cb.Context(device=0) as c:
            tid = c.load_keys(ss.pk)
            d_kidx, d_sig = hip.to_dev(ss.key_idx), hip.to_dev(ss.sig.reshape(-1))
            d_blob, d_off, d_len = hip.to_dev(ss.blob), hip.to_dev(ss.off), hip.to_dev(ss.len)
            outs = []
            for fixed in (True, False):
                out = hip.to_dev(np.full(nwords, 0xFFFFFFFFFFFFFFFF, dtype=np.uint64))
                if fixed:
                    c.verify_fixed_device(tid, 0, d_kidx, d_sig, d_blob, L, n, out, None)
                else:
                    c.verify_device(tid, 0, d_kidx, d_sig, d_blob, d_off, d_len, n, out, None)
                hip.sync()
                words = np.frombuffer(hip.from_dev(out, nwords * 8), dtype=np.uint64)
                bits = np.unpackbits(words.view(np.uint8), bitorder="little").astype(bool)
                assert not bits[n:].any()
                outs.append(bits[:n])
            assert np.array_equal(outs[0], ss.expected)
            assert np.array_equal(outs[1], ss.expected)
            c.unload_keys(tid)
    finally:
        hip.close()


@pytest.mark.parametrize("streams", [3, 2])
def test_fixed_device_64k_streams_planted_invalid(streams):
    """The headline's exact schedule: cbft_ed25519_verify_fixed_device at 64K,
    distinct signed batches with 1 % planted invalid signatures (R / S / message bit flips, S + L,
    wrong key) cycled over three (and two) streams, a verdict buffer per step pre-filled with a
    pattern no batch can produce; every step's words equal its own batch's OpenSSL verdicts."""
    hip = _Hip()
    n, L, nb, steps = 65536, 256, 3, 9
    nwords = n // 64
    sets = [sigsets.make_sigset(n, nkeys=512, msg_len=L, seed=77 + b, invalid_frac=0.01) for b in range(nb)]
    assert all(int((~s.expected).sum()) > 300 for s in sets)
    for s in sets[1:]:
        assert np.array_equal(s.pk, sets[0].pk)
    try:
        with cb.Context(device=0, max_batch=n) as c:
            tid = c.load_keys(sets[0].pk)
            dev = [(hip.to_dev(s.key_idx), hip.to_dev(s.sig.reshape(-1)), hip.to_dev(s.blob)) for s in sets]
            ss = [hip.stream() for _ in range(streams)]
            fill = np.full(nwords, 0x5A5A5A5A5A5A5A5A, dtype=np.uint64)
            outs = [hip.to_dev(fill) for _ in range(steps)]
            for j in range(steps):
                d_kidx, d_sig, d_blob = dev[j % nb]
                c.verify_fixed_device(tid, 0, d_kidx, d_sig, d_blob, L, n, outs[j], ss[j % streams])
            hip.sync()
            for j in range(steps):
                got = _bools(hip.from_dev(outs[j], nwords * 8), n)
                bad = np.nonzero(got != sets[j % nb].expected)[0]
                assert bad.size == 0, f"step {j} (batch {j % nb}): {bad.size} mismatches, first {bad[:8]}"
            c.unload_keys(tid)
    finally:
        hip.close()


@pytest.mark.parametrize("n", [1, 100, 257, 5000])
def test_hash_block_count_sort(golden, n):
    """Variable-length batches hash in order of their SHA-512 block count (a counting sort into a
    permutation before K1; a batch whose messages share one block count keeps the identity order):
    verdicts equal OpenSSL's and the unsorted path's for every signature, across ragged sizes and
    lengths straddling block boundaries (0..4,096 B, golden lengths too)."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    vs = [golden[i % len(golden)] for i in range(n)]
    args = ([index[v.pk] for v in vs], [v.sig for v in vs], [v.msg for v in vs])
    exp = np.array([bool(v.verdict) for v in vs])
    out = {}
    for label, sort_min in (("sorted", 1), ("unsorted", 0)):
        with cb.Context(device=0) as c:
            # the three-kernel path, where the sort runs
            c.set_option(cb.OPT_SMALL_MAX, 0).set_option(cb.OPT_SHA_SORT_MIN, sort_min)
            tid = c.load_keys(keys)
            out[label] = _bools(c.verify(tid, *args), n)
            # a second batch through the same work slot: the bucket counters were reset
            out[label + "2"] = _bools(c.verify(tid, *args), n)
    for k, v in out.items():
        assert np.array_equal(v, exp), k
    # random lengths, then one length for all (every signature in one bucket: the identity order)
    for msg_len in ((1, 4096), 200):
        ss = sigsets.make_sigset(n, nkeys=16, msg_len=msg_len, seed=77 + n, invalid_frac=0.1)
        with cb.Context(device=0) as c:
            c.set_option(cb.OPT_SMALL_MAX, 0).set_option(cb.OPT_SHA_SORT_MIN, 1)
            tid = c.load_keys(ss.pk)
            got = _bools(c.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), n)
            got2 = _bools(c.verify_packed(tid, ss.key_idx, ss.sig, ss.blob, ss.off, ss.len), n)
        assert np.array_equal(got, ss.expected), msg_len
        assert np.array_equal(got2, ss.expected), msg_len


@pytest.mark.parametrize("chunk", [1, 17, 300, 1024])
def test_golden_small_batches_three_wave_kernel(golden, chunk):
    """The fused kernel with [S]B on its own wave beside the hash and [h](-A) wave and the R-decode
    waves gives the golden verdicts batch for batch, partial words and tail quads included."""
    keys = sorted({v.pk for v in golden})
    index = {k: i for i, k in enumerate(keys)}
    exp = np.array([bool(v.verdict) for v in golden])
    with cb.Context(device=0) as c:
        tid = c.load_keys(keys)
        for lo in range(0, len(golden), chunk):
            part = golden[lo:lo + chunk]
            got = _bools(c.verify(tid, [index[v.pk] for v in part], [v.sig for v in part], [v.msg for v in part]),
                         len(part))
            assert np.array_equal(got, exp[lo:lo + chunk]), f"batch at {lo}"


@pytest.mark.parametrize("lens", [
    (943, 0, 47, 48, 111, 112, 941, 942),     # every message fits 8 SHA-512 blocks: the split hash
    (944, 0, 47, 48, 111, 112, 941, 942),     # one 9-block message: the block hashes on wave 0 alone
    (1, 2, 3, 4, 5, 6, 7, 8),                  # one block each
])
def test_split_hash_block_boundaries(lens):
    """The three-wave fused kernel's two-wave SHA-512 (message schedules of blocks 1.. written to
    LDS by the [S]B wave) against OpenSSL, for one 8-signature block mixing lengths at the block
    boundaries and at the split's 8-block limit (64 + 943 + 17 = 1,024 B), honest and corrupted
    signatures alike."""
    parts = [sigsets.make_sigset(2, nkeys=2, msg_len=L, seed=7000 + j, invalid_frac=0.5) for j, L in enumerate(lens)]
    pk = np.concatenate([p.pk for p in parts])
    kidx, sigs, msgs, exp = [], [], [], []
    for j, p in enumerate(parts):
        for t in range(2):
            kidx.append(2 * j + int(p.key_idx[t]))
            sigs.append(bytes(p.sig[t]))
            msgs.append(bytes(p.blob[int(p.off[t]): int(p.off[t]) + int(p.len[t])]))
            exp.append(bool(p.expected[t]))
    order = list(range(0, 16, 2)) + list(range(1, 16, 2))  # one block holds all eight lengths
    with cb.Context(device=0) as c:
        tid = c.load_keys(pk)
        got = _bools(c.verify(tid, [kidx[k] for k in order], [sigs[k] for k in order], [msgs[k] for k in order]), 16)
    assert np.array_equal(got, np.array([exp[k] for k in order]))
