"""CPU-side checks of the drop-in boundary: the library builds, loads, and exports every
symbol include/cbft_hipcrypto.h declares (no compute calls without a GPU)."""
import os
import re

import pytest

import cbft_hipcrypto as cb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "cbft_hipcrypto.h")).read()
    return sorted(set(re.findall(r"\b(cbft_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    syms = declared_symbols()
    assert "cbft_ed25519_verify_batch" in syms and "cbft_open" in syms
    assert sorted(n for n, _, _ in cb.ABI) == syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(cb.LIB_PATH):
        pytest.skip("libcbft_hipcrypto.so not built")
    lib = cb.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_strerror_and_codes():
    if not os.path.exists(cb.LIB_PATH):
        pytest.skip("libcbft_hipcrypto.so not built")
    lib = cb.load_library()
    assert lib.cbft_strerror(0) == b"ok"
    assert lib.cbft_strerror(-22) == b"invalid argument"


def test_pack_messages_layout():
    blob, off, ln = cb.pack_messages([b"ab", b"", b"xyz"])
    assert blob.tobytes() == b"abxyz"
    assert off.tolist() == [0, 2, 2] and ln.tolist() == [2, 0, 3]
    assert cb.bitmap_to_bools(bytes([0b101]), 3).tolist() == [True, False, True]
