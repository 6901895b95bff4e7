"""GPU tests of the host-buffer pipeline and the multi-GPU context (include/cbft_hipcrypto.h):

* cbft_ed25519_verify_batch_async / _fixed_async + cbft_wait: more batches in flight than the
  context has slots, waited out of order, pinned (cbft_host_alloc) and pageable inputs mixed,
  blob offsets that do not start at 0 — every batch keeps its own exact verdicts;
* concurrent blocking callers on one context (the reference calls verifiers from 40 + 24 pool
  threads, ReplicaConfig.hpp:202-212);
* the device path never reads past a key table: an out-of-range key index (or an absurd message
  length) verifies false;
* cbft_open_devices: BASELINE config #5's geometry — 1,048,576 signatures as 8 contiguous shards
  of 131,072 (here 8 shard contexts on one GPU) — gives the bitmap of one big batch.
Verdicts are checked against the host OpenSSL (tools/workload.py)."""
import ctypes
import threading

import numpy as np
import pytest

import cbft_hipcrypto as cb
import workload as sigsets
from test_ed25519_gpu import _Hip

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base():
    return sigsets.make_sigset(65536, nkeys=1024, msg_len=256, seed=0x5EED)


@pytest.fixture(scope="module")
def ctx():
    c = cb.Context(device=0, max_batch=1 << 16)
    yield c
    c.close()


def _variant(ss, v):
    sig = ss.sig.copy()
    bad = np.arange(v % 7, ss.n, 61 + 6 * v)
    sig[bad, 32 + (v % 31)] ^= 0x10
    exp = ss.expected.copy()
    exp[bad] = False
    return sig, exp


def _pinned_copy(ctx, a: np.ndarray, dtype) -> np.ndarray:
    raw = ctx.host_alloc(max(a.nbytes, 1))
    view = raw[: a.nbytes].view(dtype).reshape(a.shape)
    view[...] = a
    return raw, view


def test_async_more_batches_than_slots(ctx, base):
    tid = ctx.load_keys(base.pk, radix=8)
    pins = []
    try:
        subs = []
        for v in range(11):
            sig, exp = _variant(base, v)
            kidx, blob = base.key_idx, base.blob
            if v % 2:  # odd batches from pinned memory, even ones pageable
                r1, sig = _pinned_copy(ctx, sig, np.uint8)
                r2, kidx = _pinned_copy(ctx, base.key_idx, np.uint32)
                r3, blob = _pinned_copy(ctx, base.blob, np.uint8)
                pins += [r1, r2, r3]
            out = np.zeros(base.n // 8, dtype=np.uint8)
            if v % 3 == 0:
                t = ctx.verify_async(tid, kidx, sig, blob, out, msg_len=256)
            else:
                t = ctx.verify_async(tid, kidx, sig, blob, out, offs=base.off, lens=base.len)
            subs.append((t, out, exp, sig, kidx, blob))
        for t, out, exp, *_ in reversed(subs):
            ctx.wait(t)
            ctx.wait(t)  # a second wait is a no-op
            assert np.array_equal(cb.bitmap_to_bools(out.tobytes(), base.n), exp)
    finally:
        ctx.unload_keys(tid)
        for r in pins:
            ctx.host_free(r)


def test_async_offsets_not_from_zero(ctx):
    ss = sigsets.make_sigset(3000, nkeys=64, msg_len=(1, 900), seed=99, invalid_frac=0.1)
    pad = 1 << 20
    blob = np.concatenate([np.full(pad, 0xEE, dtype=np.uint8), ss.blob])
    offs = ss.off + np.uint64(pad)
    tid = ctx.load_keys(ss.pk)
    try:
        out = np.zeros((ss.n + 7) // 8, dtype=np.uint8)
        t = ctx.verify_async(tid, ss.key_idx, ss.sig, blob, out, offs=offs, lens=ss.len)
        ctx.wait(t)
    finally:
        ctx.unload_keys(tid)
    assert np.array_equal(cb.bitmap_to_bools(out.tobytes(), ss.n), ss.expected)


def test_concurrent_blocking_callers(ctx, base):
    tid = ctx.load_keys(base.pk, radix=8)
    errors = []
    msgs = base.msgs()

    def worker(w):
        try:
            for rep in range(6):
                lo = ((w * 7 + rep) * 997) % (base.n - 700)
                n = 1 + (w * 131 + rep * 17) % 700
                bm = ctx.verify(tid, base.key_idx[lo:lo + n], base.sig[lo:lo + n], msgs[lo:lo + n])
                if not np.array_equal(cb.bitmap_to_bools(bm, n), base.expected[lo:lo + n]):
                    errors.append((w, rep))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    try:
        th = [threading.Thread(target=worker, args=(w,)) for w in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th)
    finally:
        ctx.unload_keys(tid)
    assert not errors, errors[:5]


def test_device_path_key_index_out_of_range_verifies_false(ctx):
    ss = sigsets.make_sigset(4096, nkeys=16, msg_len=256, seed=5)
    kidx = ss.key_idx.copy()
    bad = np.arange(3, ss.n, 17)
    kidx[bad] = np.array([16, 17, 1 << 20, 0xFFFFFFFF], dtype=np.uint32)[np.arange(bad.size) % 4]
    lens = ss.len.copy()
    lens[5] = 0xFFFFFFFF  # absurd length: never read, verifies false
    exp = ss.expected.copy()
    exp[bad] = False
    exp[5] = False
    hip = _Hip()
    try:
        tid = ctx.load_keys(ss.pk)
        d_v = hip.to_dev(np.zeros((ss.n + 63) // 64, dtype=np.uint64))
        ctx.verify_device(tid, 0, hip.to_dev(kidx), hip.to_dev(ss.sig.reshape(-1)), hip.to_dev(ss.blob),
                          hip.to_dev(ss.off), hip.to_dev(lens), ss.n, d_v)
        ctx.sync()
        got = cb.bitmap_to_bools(hip.from_dev(d_v, ss.n // 8), ss.n)
        ctx.unload_keys(tid)
    finally:
        hip.close()
    assert np.array_equal(got, exp)


def test_sharded_context_config5_geometry(base):
    """1,048,576 signatures in one call on an 8-shard context (contiguous 131,072 per shard, as
    config #5 splits them over 8 GPUs) == the same batch on one plain context == OpenSSL."""
    reps = 16
    n = base.n * reps
    kidx = np.tile(base.key_idx, reps)
    sig = np.tile(base.sig, (reps, 1))
    blob = np.tile(base.blob, reps)
    exp = np.tile(base.expected, reps)
    bad = np.arange(11, n, 1013)
    sig[bad, 40] ^= 0x02
    exp[bad] = False
    with cb.Context(devices=[0] * 8, max_batch=n) as g:
        assert g.devices() == [0] * 8
        tid = g.load_keys(base.pk, radix=8)
        out = np.zeros(n // 8, dtype=np.uint8)
        t = g.verify_async(tid, kidx, sig, blob, out, msg_len=256)
        g.wait(t)
        got8 = cb.bitmap_to_bools(out.tobytes(), n)
        # a ragged total (not a multiple of the shard word size) as well
        m = n - 1000 - 37
        out2 = np.zeros((m + 7) // 8, dtype=np.uint8)
        offs = np.arange(m, dtype=np.uint64) * np.uint64(256)
        lens = np.full(m, 256, dtype=np.uint32)
        t = g.verify_async(tid, kidx[:m], sig[:m], blob, out2, offs=offs, lens=lens)
        g.wait(t)
        got_r = cb.bitmap_to_bools(out2.tobytes(), m)
        g.unload_keys(tid)
    with cb.Context(device=0, max_batch=n) as c:
        tid = c.load_keys(base.pk, radix=8)
        out1 = np.zeros(n // 8, dtype=np.uint8)
        t = c.verify_async(tid, kidx, sig, blob, out1, msg_len=256)
        c.wait(t)
        c.unload_keys(tid)
    assert np.array_equal(out, out1)
    assert np.array_equal(got8, exp)
    assert np.array_equal(got_r, exp[:m])


def test_single_dma_batch_layout(ctx, base):
    """A batch built in one pinned block at cbft_ed25519_batch_layout's offsets (one DMA)."""
    n = 5000 + 13
    blk, kidx, sig, msgs = ctx.batch_views(n, 256)
    try:
        kidx[:] = base.key_idx[:n]
        sig[:] = base.sig[:n]
        msgs[:] = base.blob[: n * 256]
        sig[7, 3] ^= 1
        exp = base.expected[:n].copy()
        exp[7] = False
        tid = ctx.load_keys(base.pk, radix=8)
        out = np.zeros((n + 7) // 8, dtype=np.uint8)
        t = ctx.verify_async(tid, kidx, sig, msgs, out, msg_len=256, n=n)
        ctx.wait(t)
        ctx.unload_keys(tid)
        assert np.array_equal(cb.bitmap_to_bools(out.tobytes(), n), exp)
    finally:
        ctx.host_free(blk)


def test_append_keys_incremental_and_concurrent(ctx):
    """Keys appended to a live table (chunk boundaries at 256 keys) get the next indices; the
    loaded keys are not rebuilt and batches against them run while appends build new tables."""
    ss = sigsets.make_sigset(6000, nkeys=1100, msg_len=(32, 300), seed=77, invalid_frac=0.1)
    tid = ctx.load_keys(ss.pk[:300], radix=8)
    assert ctx.table_size(tid) == (300, 8)
    old = ss.key_idx < 300
    msgs = ss.msgs()
    errors, stop = [], threading.Event()

    def hammer():  # verifies against the first 300 keys while appends run
        idx = np.nonzero(old)[0][:800]
        try:
            while not stop.is_set():
                bm = ctx.verify(tid, ss.key_idx[idx], ss.sig[idx], [msgs[i] for i in idx])
                if not np.array_equal(cb.bitmap_to_bools(bm, idx.size), ss.expected[idx]):
                    errors.append("mismatch during append")
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=hammer)
    th.start()
    try:
        firsts = [ctx.append_keys(tid, ss.pk[a:b]) for a, b in ((300, 301), (301, 700), (700, 1100))]
    finally:
        stop.set()
        th.join(timeout=60)
    assert firsts == [300, 301, 700] and not errors, errors[:3]
    assert ctx.table_size(tid)[0] == 1100
    got = cb.bitmap_to_bools(ctx.verify(tid, ss.key_idx, ss.sig, msgs), ss.n)
    ctx.unload_keys(tid)
    assert np.array_equal(got, ss.expected)


def test_append_to_empty_table_and_index_bounds(ctx):
    ss = sigsets.make_sigset(500, nkeys=40, msg_len=64, seed=78)
    tid = ctx.load_keys(np.zeros((0, 32), dtype=np.uint8), radix=8)
    try:
        assert ctx.table_size(tid)[0] == 0
        with pytest.raises(cb.CbftError):  # index 0 is not loaded yet
            ctx.verify(tid, ss.key_idx[:1], ss.sig[:1], ss.msgs()[:1])
        assert ctx.append_keys(tid, ss.pk) == 0
        got = cb.bitmap_to_bools(ctx.verify(tid, ss.key_idx, ss.sig, ss.msgs()), ss.n)
        assert np.array_equal(got, ss.expected)
    finally:
        ctx.unload_keys(tid)


def test_append_past_budget_rebuilds_at_lower_radix(monkeypatch):
    """appends check the HBM budget in whole 256-key chunks (what the table really
    allocates: 2.69 GB per chunk at radix 13, 0.77 GB at 11, 0.135 GB at 8).  With a 1 GB budget
    a radix-13 table does not fit at all, radix 11 holds one chunk (256 keys) and radix 8 seven
    (1,792 keys); appending past each limit rebuilds the whole table once at the next radix with
    the same key indices, and past radix 8 the append fails with CBFT_ENOMEM leaving the table
    usable."""
    monkeypatch.setenv("CBFT_COMB_BUDGET_GB", "1.0")
    ss = sigsets.make_sigset(2000, nkeys=40, msg_len=(16, 300), seed=81, invalid_frac=0.1)
    msgs = ss.msgs()
    rng = np.random.default_rng(5)
    pk = np.concatenate([ss.pk, rng.integers(0, 256, size=(1800 - 40, 32), dtype=np.uint8)])
    with cb.Context(device=0) as c:
        tid = c.load_keys(pk[:1], radix=13)  # explicit radix: the budget is not consulted
        assert c.table_size(tid) == (1, 13)
        seen = []
        for a, b in ((1, 2), (2, 256), (256, 257), (257, 1792)):
            assert c.append_keys(tid, pk[a:b]) == a
            seen.append(c.table_size(tid))
            use = np.nonzero(ss.key_idx < b)[0]
            got = cb.bitmap_to_bools(c.verify(tid, ss.key_idx[use], ss.sig[use], [msgs[i] for i in use]), use.size)
            assert np.array_equal(got, ss.expected[use]), (a, b)
        assert seen == [(2, 11), (256, 11), (257, 8), (1792, 8)]
        with pytest.raises(cb.CbftError) as e:
            c.append_keys(tid, pk[1792:1793])
        assert e.value.code == -12  # CBFT_ENOMEM
        assert c.table_size(tid) == (1792, 8)
        got = cb.bitmap_to_bools(c.verify(tid, ss.key_idx, ss.sig, msgs), ss.n)
        assert np.array_equal(got, ss.expected)
        c.unload_keys(tid)


def test_replace_key_slot(ctx):
    """cbft_ed25519_replace_keys: a slot rebuilt with another key verifies that key's signatures
    and no longer the old key's; the other slots are untouched."""
    ss = sigsets.make_sigset(512, nkeys=8, msg_len=64, seed=83)
    msgs = ss.msgs()
    tid = ctx.load_keys(ss.pk[:6], radix=8)
    try:
        use = np.nonzero(ss.key_idx < 6)[0]
        ctx.replace_keys(tid, [2], ss.pk[7:8])  # slot 2 now holds key 7
        kidx = ss.key_idx[use].copy()
        got = cb.bitmap_to_bools(ctx.verify(tid, kidx, ss.sig[use], [msgs[i] for i in use]), use.size)
        exp = ss.expected[use] & (kidx != 2)
        assert np.array_equal(got, exp)
        seven = np.nonzero(ss.key_idx == 7)[0]
        got7 = cb.bitmap_to_bools(ctx.verify(tid, np.full(seven.size, 2, np.uint32), ss.sig[seven],
                                             [msgs[i] for i in seven]), seven.size)
        assert got7.all()
        with pytest.raises(cb.CbftError):
            ctx.replace_keys(tid, [6], ss.pk[7:8])  # not a loaded slot
    finally:
        ctx.unload_keys(tid)


def test_async_pageable_inputs_reusable_on_return(ctx, base):
    """a pageable batch too large for the pinned pack (64K x 256 B = 16 MB of
    messages) is copied before the _async call returns, so the caller may overwrite its buffers
    at once and the verdicts still belong to the original inputs."""
    tid = ctx.load_keys(base.pk, radix=8)
    try:
        sig, blob = base.sig.copy(), base.blob.copy()
        out = np.zeros(base.n // 8, dtype=np.uint8)
        t = ctx.verify_async(tid, base.key_idx, sig, blob, out, offs=base.off, lens=base.len)
        sig[:] = 0xA5
        blob[:] = 0x5A
        ctx.wait(t)
        assert np.array_equal(cb.bitmap_to_bools(out.tobytes(), base.n), base.expected)
    finally:
        ctx.unload_keys(tid)
