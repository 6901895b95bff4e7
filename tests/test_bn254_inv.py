"""CPU check of the variable-time Fp inversion (safegcd divsteps, bn254_field.h: fp_inv_var) that
the final exponentiations use, through the host build of the device code
(tests/cpp/libbn254_shim.so): equal to x^(p-2) mod p and to the constant-time Fermat fp_inv."""
import ctypes
import os
import random

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "cpp", "libbn254_shim.so")
U = -(2**62 + 2**55 + 1)
P = 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1


@pytest.fixture(scope="module")
def shim():
    if not os.path.exists(SHIM):
        pytest.skip("tests/cpp/libbn254_shim.so not built (make shim)")
    return ctypes.CDLL(SHIM)


def test_fp_inv_var_matches_fermat(shim):
    rng = random.Random(0xB15)
    xs = [0, 1, 2, 3, 19, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2**253, 2**254 % P, 2**128, 2**128 - 1]
    xs += [(1 << k) % P for k in range(0, 254, 7)] + [rng.randrange(P) for _ in range(2000)]
    for x in xs:
        o1, o2 = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        agree = shim.shim_fp_inv(x.to_bytes(32, "big"), o1, o2)
        want = pow(x, P - 2, P)
        assert int.from_bytes(o1.raw, "big") == want, hex(x)
        assert int.from_bytes(o2.raw, "big") == want, hex(x)
        assert agree == 1


def test_fp_addsub_matches_add_and_sub(shim):
    """f_addsub (one signed pass, per-lane add or subtract) gives the same reduced limbs as f_add /
    f_sub, and the right values, including operands whose top limbs tie."""
    rng = random.Random(0xADD5)
    xs = [0, 1, P - 1, P - 2, (P - 1) // 2, 2**253, 2**232, 2**232 - 1] + [rng.randrange(P) for _ in range(600)]
    for i, a in enumerate(xs):
        b = xs[(i * 7 + 3) % len(xs)]
        out = ctypes.create_string_buffer(128)
        same = shim.shim_fp_addsub(a.to_bytes(32, "big"), b.to_bytes(32, "big"), out)
        vals = [int.from_bytes(out.raw[32 * k:32 * k + 32], "big") for k in range(4)]
        assert vals == [(a + b) % P, (a - b) % P, (a + b) % P, (a - b) % P]
        assert same == 1
