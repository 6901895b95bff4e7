"""Row-parallel GF(2^255 - 19) (concord-bft_amd/csrc/fe25519_row.h) on the host SIMD emulation
(tests/cpp/libfe_row_shim.so, the same templates the small-batch kernels' R decode runs on
gfx950), against Python integers mod p, with operands at the bounds the header states:
row-reduced limbs <= 2^29 + 2^23, row-lazy limbs <= 2^30 + 2^24, lanes 9..15 zero.
"""
import ctypes
import os
import random

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "cpp", "libfe_row_shim.so")
P = 2**255 - 19
MASK = (1 << 29) - 1
REDUCED = (1 << 29) + (1 << 23)
LAZY = (1 << 30) + (1 << 24)

U36 = ctypes.c_uint32 * 36
U64 = ctypes.c_uint32 * 64


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(SHIM):
        pytest.skip("tests/cpp/libfe_row_shim.so not built (make fe_row_shim)")
    return ctypes.CDLL(SHIM)


def val(limbs):
    return sum(int(x) << (29 * i) for i, x in enumerate(limbs))


def rows(elems):
    a = U36()
    for r, e in enumerate(elems):
        for i in range(9):
            a[9 * r + i] = e[i]
    return a


def out_rows(out):
    res = []
    for r in range(4):
        lanes = [out[16 * r + l] for l in range(16)]
        assert lanes[9:] == [0] * 7, "lanes 9..15 must stay zero"
        assert all(x <= REDUCED for x in lanes[:9]), "output not row-reduced"
        res.append(lanes[:9])
    return res


def rand_limbs(rng, bound):
    kind = rng.randrange(4)
    if kind == 0:
        return [bound] * 9  # every limb at the bound
    if kind == 1:
        return [rng.choice((0, bound, bound - 1, MASK)) for _ in range(9)]
    if kind == 2:
        x = rng.randrange(P)
        return [(x >> (29 * i)) & MASK for i in range(9)]
    return [rng.randrange(bound + 1) for _ in range(9)]


@pytest.mark.parametrize("bound", [REDUCED, LAZY])
def test_mul_sq_bounds(lib, bound):
    rng = random.Random(0xFE25519 + bound)
    for _ in range(200):
        a = [rand_limbs(rng, bound) for _ in range(4)]
        b = [rand_limbs(rng, bound) for _ in range(4)]
        out = U64()
        lib.fe_row_mul(rows(a), rows(b), out)
        for r, o in enumerate(out_rows(out)):
            assert val(o) % P == val(a[r]) * val(b[r]) % P
        lib.fe_row_sq(rows(a), out)
        for r, o in enumerate(out_rows(out)):
            assert val(o) % P == val(a[r]) ** 2 % P


def test_sub_carry(lib):
    rng = random.Random(7)
    for _ in range(200):
        a = [rand_limbs(rng, LAZY) for _ in range(4)]
        b = [rand_limbs(rng, LAZY) for _ in range(4)]
        out = U64()
        lib.fe_row_sub(rows(a), rows(b), out)
        for r, o in enumerate(out_rows(out)):
            assert val(o) % P == (val(a[r]) - val(b[r])) % P
        c = [[rng.randrange(1 << 31) for _ in range(9)] for _ in range(4)]
        lib.fe_row_carry(rows(c), out)
        for r, o in enumerate(out_rows(out)):
            assert val(o) % P == val(c[r]) % P


def test_pow22523(lib):
    rng = random.Random(11)
    cases = [0, 1, 2, P - 1, P - 2, 2**255 - 20 - 2**200, rng.randrange(P), rng.randrange(P)]
    for k in range(0, len(cases), 4):
        elems = [[(x >> (29 * i)) & MASK for i in range(9)] for x in cases[k:k + 4]]
        out = U64()
        lib.fe_row_pow22523(rows(elems), out)
        for r, o in enumerate(out_rows(out)):
            assert val(o) % P == pow(cases[k + r], (P - 5) // 8, P)
