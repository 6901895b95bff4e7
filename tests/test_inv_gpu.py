"""The wave-cooperative variable-time inversion (safegcd30.h: sg_inv30_var_wave) on gfx950, through
the test-only harness tests/hip/libinv_selftest.so: one wave per value, both moduli the library
inverts with it (BN-P254's p: the pairing checks' Fp12 inversion; 2^255 - 19: the Ed25519 finish
root), adversarial and random values, against Python's pow(x, p - 2, p) and against the one-lane
form on the same device."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "hip", "libinv_selftest.so")
U = -(2**62 + 2**55 + 1)
P_BN = 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1
P_ED = 2**255 - 19


def _limbs30(x):
    return [(x >> (30 * j)) & (2**30 - 1) for j in range(9)]


def _val30(v):
    return sum(int(l) << (30 * j) for j, l in enumerate(v))


def _values(p, seed):
    rng = random.Random(seed)
    xs = [0, 1, 2, 3, 19, p - 1, p - 2, (p - 1) // 2, (p + 1) // 2, 2**128 - 1, 2**128, 2**253 % p, 2**254 % p]
    xs += [(1 << k) % p for k in range(0, 255, 5)] + [p - (1 << k) for k in range(0, 250, 7)]
    xs += [(2**30 - 1) << (30 * j) for j in range(8)]  # full limbs: carries across the limb splits
    xs += [rng.randrange(p) for _ in range(1500)]
    return [x % p for x in xs]


@pytest.mark.gpu
@pytest.mark.parametrize("which,p", [(0, P_BN), (1, P_ED)])
def test_wave_inversion_on_gpu(which, p):
    if not os.path.exists(LIB):
        pytest.fail("tests/hip/libinv_selftest.so not built (make selftest)")
    lib = ctypes.CDLL(LIB)
    xs = _values(p, 0xA11 + which)
    n = len(xs)
    inp = np.array([_limbs30(x) for x in xs], dtype=np.int32)
    wave = np.zeros_like(inp)
    lane = np.zeros_like(inp)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.inv_selftest(ptr(inp), ptr(wave), ptr(lane), ctypes.c_int(n), ctypes.c_int(which))
    assert rc == 0, f"HIP error {rc}"
    for x, w, l in zip(xs, wave, lane):
        want = pow(x, p - 2, p) if x else 0
        assert _val30(w) == want and all(0 <= int(v) < 2**30 for v in w), hex(x)
        assert _val30(l) == want, hex(x)
