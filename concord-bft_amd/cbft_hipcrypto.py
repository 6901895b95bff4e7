"""Python binding of libcbft_hipcrypto (ctypes over the C ABI in include/cbft_hipcrypto.h).

This is the binding a maintainer would add next to the reference's own Python tooling (the
ctypes stub shown in INTEGRATION.md); tests and bench.py drive the GPU through it.  The product
path has no CPU fallback: if the HIP library is missing or no GPU is visible, every entry point
raises.

    ctx = Context(device=0)
    tid = ctx.load_keys(pks)                       # pks: list of 32-byte keys
    bitmap = ctx.verify(tid, key_idx, sigs, msgs)  # -> bytes, bit i = signature i accepted
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CBFT_LIB") or os.path.join(HERE, "libcbft_hipcrypto.so")  # CBFT_LIB: variant builds

CBFT_NO_KEY_TABLE = 0xFFFFFFFF
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)

# (name, restype, argtypes) for every symbol include/cbft_hipcrypto.h declares
ABI = [
    ("cbft_device_count", ctypes.c_int, []),
    ("cbft_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("cbft_last_error", ctypes.c_char_p, []),
    ("cbft_open", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t]),
    ("cbft_open_mask", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_size_t]),
    ("cbft_open_devices", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t]),
    ("cbft_device_of", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("cbft_close", None, [ctypes.c_void_p]),
    ("cbft_set_option", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]),
    ("cbft_host_alloc", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("cbft_host_free", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("cbft_ed25519_verify_batch_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("cbft_ed25519_verify_fixed_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("cbft_wait", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    ("cbft_ed25519_batch_layout", ctypes.c_int,
     [ctypes.c_size_t, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    ("cbft_ed25519_load_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, _u32p]),
    ("cbft_ed25519_load_keys_ex", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, _u32p]),
    ("cbft_ed25519_unload_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("cbft_ed25519_append_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                                _u32p]),
    ("cbft_ed25519_replace_keys", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    ("cbft_ed25519_table_size", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, _u32p,
                                               ctypes.POINTER(ctypes.c_int)]),
    ("cbft_ed25519_verify_batch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("cbft_ed25519_verify_batch_pk", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_size_t, ctypes.c_void_p]),
    ("cbft_ed25519_verify_batch_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    ("cbft_ed25519_verify_fixed_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    ("cbft_sync", ctypes.c_int, [ctypes.c_void_p]),
    ("cbft_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("cbft_stage_times_ms", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    ("cbft_stage_times_avg_ms", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("cbft_rsa_load_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, _u32p]),
    ("cbft_rsa_unload_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("cbft_rsa_key_status", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_rsa_verify_batch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("cbft_rsa_verify_batch_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    ("cbft_rsa_kernel_ms", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    ("cbft_bls_load_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, _u32p]),
    ("cbft_bls_unload_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("cbft_bls_key_status", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_bls_hash_to_g1", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_bls_verify_shares", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
      ctypes.c_void_p]),
    ("cbft_bls_combine", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int,
                                        ctypes.c_void_p]),
    ("cbft_bls_verify", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                       ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    ("cbft_bls_combine_threshold", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    ("cbft_bls_verify_multisig", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p,
      ctypes.POINTER(ctypes.c_int)]),
    ("cbft_bls_sum_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_void_p]),
    ("cbft_bls_sign", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                     ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_bls_public_key", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]),
    ("cbft_bls_combine_partial", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
      ctypes.c_void_p]),
    ("cbft_bls_combine_finish", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_bls_sum_keys_partial", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    ("cbft_bls_verify_multisig_partials", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32,
      ctypes.POINTER(ctypes.c_int)]),
]

# cbft_set_option options (include/cbft_hipcrypto.h, "tuning")
OPT_LADDER_LANES = 1
OPT_B_RADIX = 2
OPT_WORK_SLOTS = 3
OPT_SMALL_MAX = 4
OPT_SHA_SORT_MIN = 5
OPT_STAGE_ORDER = 6
OPT_HASH_ORDER_EARLY = 7
OPT_FINISH_K = 8

BLS_G1_PARTIAL_BYTES = 108
BLS_G2_PARTIAL_BYTES = 220

_lib = None


class CbftError(RuntimeError):
    def __init__(self, code: int, what: str):
        lib = load_library()
        detail = lib.cbft_last_error().decode(errors="replace")
        super().__init__(f"{what}: {lib.cbft_strerror(code).decode()} ({code}) {detail}")
        self.code = code


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the HIP library (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run `make lib` (or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    for name, res, args in ABI:
        if os.environ.get("CBFT_LIB") and not hasattr(lib, name):
            continue  # an older A/B build ($CBFT_LIB) without a later entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        raise CbftError(rc, what)


def pack_messages(msgs: Sequence[bytes]):
    """Concatenate messages into (blob, offsets u64, lengths u32) as the ABI expects."""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=len(msgs))
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs) > 1:
        np.cumsum(lens[:-1], out=offs[1:])
    blob = b"".join(msgs)
    return np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8), offs, lens


def bitmap_to_bools(bitmap: bytes, n: int) -> np.ndarray:
    return np.unpackbits(np.frombuffer(bitmap, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Context:
    """One GPU context (cbft_open / cbft_close)."""

    def __init__(self, device: int = 0, max_batch: int = 0, device_mask: int = 0,
                 devices: Optional[Sequence[int]] = None):
        """device_mask != 0: one context over every GPU in the mask (cbft_open_mask); devices: an
        explicit shard list, repeats allowed (cbft_open_devices)."""
        self.lib = load_library()
        self.handle = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            _check(self.lib.cbft_open_devices(ctypes.byref(self.handle), arr, len(devices), max_batch),
                   f"cbft_open_devices({list(devices)})")
            device = devices[0]
        elif device_mask:
            _check(self.lib.cbft_open_mask(ctypes.byref(self.handle), device_mask, max_batch),
                   f"cbft_open_mask({device_mask:#x})")
            device = (device_mask & -device_mask).bit_length() - 1
        else:
            _check(self.lib.cbft_open(ctypes.byref(self.handle), device, max_batch), f"cbft_open(device={device})")
        self.device = device

    def set_option(self, option: int, value: int):
        """cbft_set_option: a per-context geometry / scheduling switch (OPT_*)."""
        _check(self.lib.cbft_set_option(self.handle, option, int(value)), f"cbft_set_option({option}, {value})")
        return self

    def devices(self) -> List[int]:
        out = (ctypes.c_int * 32)()
        n = self.lib.cbft_device_of(self.handle, out, 32)
        if n < 0:
            raise CbftError(n, "cbft_device_of")
        return list(out[:n])

    # ------------------------------------------------------------------ pinned host memory
    def host_alloc(self, nbytes: int) -> np.ndarray:
        """A uint8 numpy view of cbft_host_alloc memory (free with host_free(view))."""
        p = ctypes.c_void_p()
        _check(self.lib.cbft_host_alloc(self.handle, nbytes, ctypes.byref(p)), "cbft_host_alloc")
        buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
        return np.frombuffer(buf, dtype=np.uint8)

    def host_free(self, view: np.ndarray):
        _check(self.lib.cbft_host_free(self.handle, ctypes.c_void_p(view.ctypes.data)), "cbft_host_free")

    # ------------------------------------------------------------------ async host-buffer verify
    def verify_async(self, tid: int, key_idx: np.ndarray, sigs: np.ndarray, blob: np.ndarray, out: np.ndarray,
                     offs: Optional[np.ndarray] = None, lens: Optional[np.ndarray] = None,
                     msg_len: Optional[int] = None, n: Optional[int] = None) -> int:
        """Queue a batch; returns the ticket.  Either (offs, lens) or a fixed msg_len.  `out`
        (uint8, >= ceil(n/8)) receives the bitmap by the time wait(ticket) returns; inputs and
        out must stay alive until then."""
        t = ctypes.c_uint64()
        if msg_len is not None:
            n = int(key_idx.shape[0]) if n is None else n
            _check(self.lib.cbft_ed25519_verify_fixed_async(self.handle, tid, _ptr(key_idx), _ptr(sigs), _ptr(blob),
                                                            msg_len, n, _ptr(out), ctypes.byref(t)),
                   "cbft_ed25519_verify_fixed_async")
        else:
            n = int(lens.shape[0]) if n is None else n
            _check(self.lib.cbft_ed25519_verify_batch_async(self.handle, tid, _ptr(key_idx), _ptr(sigs), _ptr(blob),
                                                            _ptr(offs), _ptr(lens), n, _ptr(out), ctypes.byref(t)),
                   "cbft_ed25519_verify_batch_async")
        return t.value

    def batch_views(self, n: int, msg_len: int):
        """One pinned block laid out as cbft_ed25519_batch_layout says: returns (block, key_idx
        u32[n], sig u8[n, 64], msgs u8[n * msg_len]) views; fill them and submit with
        verify_async(..., msg_len=msg_len) for a single-DMA batch.  Free with host_free(block)."""
        o = [ctypes.c_size_t() for _ in range(4)]
        _check(self.lib.cbft_ed25519_batch_layout(n, msg_len, *[ctypes.byref(x) for x in o]),
               "cbft_ed25519_batch_layout")
        ok, osig, omsg, total = (x.value for x in o)
        blk = self.host_alloc(total)
        return (blk, blk[ok:ok + 4 * n].view(np.uint32), blk[osig:osig + 64 * n].reshape(n, 64),
                blk[omsg:omsg + n * msg_len])

    def wait(self, ticket: int):
        _check(self.lib.cbft_wait(self.handle, ticket), "cbft_wait")

    def close(self):
        if self.handle:
            self.lib.cbft_close(self.handle)
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ keys
    def load_keys(self, pks: Iterable[bytes] | np.ndarray, radix: int = 0) -> int:
        """Upload a key table; radix = comb radix 2^radix of the per-key tables (8..15, 0 = default)."""
        arr = _as_rows(pks, 32)
        tid = ctypes.c_uint32()
        _check(self.lib.cbft_ed25519_load_keys_ex(self.handle, _ptr(arr), arr.shape[0], radix, ctypes.byref(tid)),
               "cbft_ed25519_load_keys_ex")
        return tid.value

    def append_keys(self, tid: int, pks) -> int:
        """Append keys to a loaded table; returns the first new key index."""
        arr = _as_rows(pks, 32)
        first = ctypes.c_uint32()
        _check(self.lib.cbft_ed25519_append_keys(self.handle, tid, _ptr(arr), arr.shape[0], ctypes.byref(first)),
               "cbft_ed25519_append_keys")
        return first.value

    def replace_keys(self, tid: int, idx, pks):
        """Rebuild loaded key slots idx with new keys (cbft_ed25519_replace_keys)."""
        arr = _as_rows(pks, 32)
        ix = np.ascontiguousarray(np.asarray(idx, dtype=np.uint32))
        assert ix.shape[0] == arr.shape[0]
        _check(self.lib.cbft_ed25519_replace_keys(self.handle, tid, _ptr(ix), _ptr(arr), ix.shape[0]),
               "cbft_ed25519_replace_keys")

    def table_size(self, tid: int):
        n, r = ctypes.c_uint32(), ctypes.c_int()
        _check(self.lib.cbft_ed25519_table_size(self.handle, tid, ctypes.byref(n), ctypes.byref(r)),
               "cbft_ed25519_table_size")
        return n.value, r.value

    def unload_keys(self, tid: int):
        _check(self.lib.cbft_ed25519_unload_keys(self.handle, tid), "cbft_ed25519_unload_keys")

    # ------------------------------------------------------------------ verify
    def verify(self, tid: int, key_idx, sigs, msgs: Sequence[bytes]) -> bytes:
        n = len(msgs)
        kidx = np.ascontiguousarray(np.asarray(key_idx, dtype=np.uint32))
        s = _as_rows(sigs, 64)
        assert kidx.shape[0] == n and s.shape[0] == n
        blob, offs, lens = pack_messages(msgs)
        out = np.zeros(max(1, (n + 7) // 8), dtype=np.uint8)
        _check(self.lib.cbft_ed25519_verify_batch(self.handle, tid, _ptr(kidx), _ptr(s), _ptr(blob), _ptr(offs),
                                                   _ptr(lens), n, _ptr(out)), "cbft_ed25519_verify_batch")
        return out.tobytes()[: (n + 7) // 8]

    def verify_packed(self, tid: int, key_idx: np.ndarray, sigs: np.ndarray, blob: np.ndarray, offs: np.ndarray,
                      lens: np.ndarray) -> bytes:
        """verify() with messages already packed as (blob, offsets u64, lengths u32)."""
        n = int(lens.shape[0])
        out = np.zeros(max(1, (n + 7) // 8), dtype=np.uint8)
        _check(self.lib.cbft_ed25519_verify_batch(self.handle, tid, _ptr(key_idx), _ptr(sigs), _ptr(blob), _ptr(offs),
                                                   _ptr(lens), n, _ptr(out)), "cbft_ed25519_verify_batch")
        return out.tobytes()[: (n + 7) // 8]

    def verify_pk(self, pks, sigs, msgs: Sequence[bytes]) -> bytes:
        n = len(msgs)
        p = _as_rows(pks, 32)
        s = _as_rows(sigs, 64)
        assert p.shape[0] == n and s.shape[0] == n
        blob, offs, lens = pack_messages(msgs)
        out = np.zeros(max(1, (n + 7) // 8), dtype=np.uint8)
        _check(self.lib.cbft_ed25519_verify_batch_pk(self.handle, _ptr(p), _ptr(s), _ptr(blob), _ptr(offs),
                                                      _ptr(lens), n, _ptr(out)), "cbft_ed25519_verify_batch_pk")
        return out.tobytes()[: (n + 7) // 8]

    def verify_device(self, tid: int, d_pk: int, d_key_idx: int, d_sig: int, d_msg: int, d_off: int, d_len: int,
                      n: int, d_verdict_words: int, stream: int = 0):
        """All arguments are raw device addresses (e.g. torch tensor .data_ptr())."""
        _check(self.lib.cbft_ed25519_verify_batch_device(
            self.handle, tid, ctypes.c_void_p(d_pk), ctypes.c_void_p(d_key_idx), ctypes.c_void_p(d_sig),
            ctypes.c_void_p(d_msg), ctypes.c_void_p(d_off), ctypes.c_void_p(d_len), n,
            ctypes.c_void_p(d_verdict_words), ctypes.c_void_p(stream)), "cbft_ed25519_verify_batch_device")

    def verify_fixed_device(self, tid: int, d_pk: int, d_key_idx: int, d_sig: int, d_msg: int, msg_len: int,
                            n: int, d_verdict_words: int, stream: int = 0):
        """Fixed-length messages (message i at d_msg + i * msg_len); raw device addresses."""
        _check(self.lib.cbft_ed25519_verify_fixed_device(
            self.handle, tid, ctypes.c_void_p(d_pk), ctypes.c_void_p(d_key_idx), ctypes.c_void_p(d_sig),
            ctypes.c_void_p(d_msg), msg_len, n, ctypes.c_void_p(d_verdict_words), ctypes.c_void_p(stream)),
            "cbft_ed25519_verify_fixed_device")

    def sync(self):
        _check(self.lib.cbft_sync(self.handle), "cbft_sync")

    # ------------------------------------------------------------------ RSA-2048 PKCS#1 v1.5 / SHA-256
    def rsa_load_keys(self, keys: Sequence[tuple]) -> int:
        """keys: (n, e) integer pairs (2048-bit moduli, 32-bit exponents)."""
        mods = np.frombuffer(b"".join(int(n).to_bytes(256, "big") for n, _ in keys), dtype=np.uint8) \
            if keys else np.zeros(1, np.uint8)
        exps = np.array([int(e) for _, e in keys] or [0], dtype=np.uint32)
        tid = ctypes.c_uint32()
        _check(self.lib.cbft_rsa_load_keys(self.handle, _ptr(mods), _ptr(exps), len(keys), ctypes.byref(tid)),
               "cbft_rsa_load_keys")
        return tid.value

    def rsa_unload_keys(self, tid: int):
        _check(self.lib.cbft_rsa_unload_keys(self.handle, tid), "cbft_rsa_unload_keys")

    def rsa_key_status(self, tid: int, nkeys: int) -> np.ndarray:
        out = np.zeros(max(1, nkeys), dtype=np.uint8)
        _check(self.lib.cbft_rsa_key_status(self.handle, tid, _ptr(out)), "cbft_rsa_key_status")
        return out[:nkeys].astype(bool)

    def rsa_verify(self, tid: int, key_idx, sigs, msgs: Sequence[bytes]) -> bytes:
        n = len(msgs)
        kidx = np.ascontiguousarray(np.asarray(key_idx, dtype=np.uint32))
        s = _as_rows(sigs, 256)
        assert kidx.shape[0] == n and s.shape[0] == n
        blob, offs, lens = pack_messages(msgs)
        out = np.zeros(max(1, (n + 7) // 8), dtype=np.uint8)
        _check(self.lib.cbft_rsa_verify_batch(self.handle, tid, _ptr(kidx), _ptr(s), _ptr(blob), _ptr(offs),
                                               _ptr(lens), n, _ptr(out)), "cbft_rsa_verify_batch")
        return out.tobytes()[: (n + 7) // 8]

    def rsa_verify_device(self, tid: int, d_key_idx: int, d_sig: int, d_msg: int, d_off: int, d_len: int, n: int,
                          d_verdict_words: int, stream: int = 0):
        _check(self.lib.cbft_rsa_verify_batch_device(
            self.handle, tid, ctypes.c_void_p(d_key_idx), ctypes.c_void_p(d_sig), ctypes.c_void_p(d_msg),
            ctypes.c_void_p(d_off), ctypes.c_void_p(d_len), n, ctypes.c_void_p(d_verdict_words),
            ctypes.c_void_p(stream)), "cbft_rsa_verify_batch_device")

    def rsa_kernel_ms(self) -> float:
        out = ctypes.c_float()
        _check(self.lib.cbft_rsa_kernel_ms(self.handle, ctypes.byref(out)), "cbft_rsa_kernel_ms")
        return out.value

    # ------------------------------------------------------------------ BLS BN-P254
    def bls_load_keys(self, pk65: bytes, vks65: Sequence[bytes]) -> int:
        kid = ctypes.c_uint32()
        _check(self.lib.cbft_bls_load_keys(self.handle, pk65, b"".join(vks65), len(vks65), ctypes.byref(kid)),
               "cbft_bls_load_keys")
        return kid.value

    def bls_unload_keys(self, kid: int):
        _check(self.lib.cbft_bls_unload_keys(self.handle, kid), "cbft_bls_unload_keys")

    def bls_key_status(self, kid: int, n: int) -> bytes:
        out = ctypes.create_string_buffer(n + 1)
        _check(self.lib.cbft_bls_key_status(self.handle, kid, out), "cbft_bls_key_status")
        return out.raw

    def bls_hash_to_g1(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(33)
        _check(self.lib.cbft_bls_hash_to_g1(self.handle, msg, len(msg), out), "cbft_bls_hash_to_g1")
        return out.raw

    def bls_verify_shares(self, kid: int, msg: bytes, shares: Sequence[bytes]) -> np.ndarray:
        k = len(shares)
        out = ctypes.create_string_buffer(max(1, (k + 7) // 8))
        _check(self.lib.cbft_bls_verify_shares(self.handle, kid, msg, len(msg), b"".join(shares), k, out),
               "cbft_bls_verify_shares")
        return bitmap_to_bools(out.raw, k)

    def bls_combine(self, shares: Sequence[bytes], multisig: bool = False) -> bytes:
        out = ctypes.create_string_buffer(33)
        _check(self.lib.cbft_bls_combine(self.handle, b"".join(shares), len(shares), 1 if multisig else 0, out),
               "cbft_bls_combine")
        return out.raw

    def bls_combine_threshold(self, kid: int, msg: bytes, shares: Sequence[bytes], optimistic: bool = True):
        """The certificate policy in one call (cbft_bls_combine_threshold): returns (sig33, ok,
        bad) with bad[j] = share j failed share verification."""
        k = len(shares)
        sig = ctypes.create_string_buffer(33)
        bad = ctypes.create_string_buffer(max(1, (k + 7) // 8))
        ok = ctypes.c_int()
        _check(self.lib.cbft_bls_combine_threshold(self.handle, kid, msg, len(msg), b"".join(shares), k,
                                                    1 if optimistic else 0, sig, bad, ctypes.byref(ok)),
               "cbft_bls_combine_threshold")
        return sig.raw, bool(ok.value), bitmap_to_bools(bad.raw, k)

    def bls_verify(self, kid: int, msg: bytes, sig33: bytes) -> bool:
        ok = ctypes.c_int()
        _check(self.lib.cbft_bls_verify(self.handle, kid, msg, len(msg), sig33, ctypes.byref(ok)), "cbft_bls_verify")
        return bool(ok.value)

    def bls_verify_multisig(self, kid: int, msg: bytes, sig33: bytes, signers256: bytes) -> bool:
        ok = ctypes.c_int()
        _check(self.lib.cbft_bls_verify_multisig(self.handle, kid, msg, len(msg), sig33, signers256,
                                                  ctypes.byref(ok)), "cbft_bls_verify_multisig")
        return bool(ok.value)

    def bls_sum_keys(self, kid: int, signers256: bytes) -> bytes:
        out = ctypes.create_string_buffer(65)
        _check(self.lib.cbft_bls_sum_keys(self.handle, kid, signers256, out), "cbft_bls_sum_keys")
        return out.raw

    # sharded combine / multisig key sum (partials are exchanged between ranks, cbft_multigpu)
    def bls_combine_partial(self, shares: Sequence[bytes], lo: int, hi: int, multisig: bool = False) -> bytes:
        out = ctypes.create_string_buffer(BLS_G1_PARTIAL_BYTES)
        _check(self.lib.cbft_bls_combine_partial(self.handle, b"".join(shares), len(shares), lo, hi,
                                                  1 if multisig else 0, out), "cbft_bls_combine_partial")
        return out.raw

    def bls_combine_finish(self, partials: Sequence[bytes]) -> bytes:
        out = ctypes.create_string_buffer(33)
        _check(self.lib.cbft_bls_combine_finish(self.handle, b"".join(partials), len(partials), out),
               "cbft_bls_combine_finish")
        return out.raw

    def bls_sum_keys_partial(self, kid: int, signers256: bytes, lo_id: int, hi_id: int) -> bytes:
        out = ctypes.create_string_buffer(BLS_G2_PARTIAL_BYTES)
        _check(self.lib.cbft_bls_sum_keys_partial(self.handle, kid, signers256, lo_id, hi_id, out),
               "cbft_bls_sum_keys_partial")
        return out.raw

    def bls_verify_multisig_partials(self, msg: bytes, sig33: bytes, key_partials: Sequence[bytes]) -> bool:
        ok = ctypes.c_int()
        _check(self.lib.cbft_bls_verify_multisig_partials(self.handle, msg, len(msg), sig33, b"".join(key_partials),
                                                           len(key_partials), ctypes.byref(ok)),
               "cbft_bls_verify_multisig_partials")
        return bool(ok.value)

    def bls_sign(self, sk: int, share_id: int, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(37)
        _check(self.lib.cbft_bls_sign(self.handle, sk.to_bytes(32, "big"), share_id, msg, len(msg), out),
               "cbft_bls_sign")
        return out.raw

    def bls_public_key(self, sk: int) -> bytes:
        """sk * g2, 65 compressed bytes (the signer's share verification key)."""
        out = ctypes.create_string_buffer(65)
        _check(self.lib.cbft_bls_public_key(self.handle, sk.to_bytes(32, "big"), out), "cbft_bls_public_key")
        return out.raw

    def set_profiling(self, on: bool = True, per_batch: bool = False):
        mode = (2 if per_batch else 1) if on else 0
        _check(self.lib.cbft_set_profiling(self.handle, mode), "cbft_set_profiling")

    def stage_times_avg_ms(self):
        """Mean {hash, ladder, finish} stage times (ms) over the batches since
        set_profiling(per_batch=True), and the batch count."""
        out = (ctypes.c_float * 3)()
        cnt = ctypes.c_int(0)
        _check(self.lib.cbft_stage_times_avg_ms(self.handle, out, 3, ctypes.byref(cnt)), "cbft_stage_times_avg_ms")
        return {"hash": out[0], "ladder": out[1], "finish": out[2]}, cnt.value

    def stage_times_ms(self):
        """{hash, ladder, finish} kernel times (ms) of the last verify (needs set_profiling)."""
        out = (ctypes.c_float * 3)()
        _check(self.lib.cbft_stage_times_ms(self.handle, out, 3), "cbft_stage_times_ms")
        return {"hash": out[0], "ladder": out[1], "finish": out[2]}


def _as_rows(x, width: int) -> np.ndarray:
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x, dtype=np.uint8).reshape(-1, width)
    else:
        rows = list(x)
        for r in rows:
            if len(r) != width:
                raise ValueError(f"expected {width}-byte items, got {len(r)}")
        a = np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(-1, width) if rows else np.zeros((0, width),
                                                                                                   np.uint8)
    return np.ascontiguousarray(a)


def device_count() -> int:
    return load_library().cbft_device_count()
