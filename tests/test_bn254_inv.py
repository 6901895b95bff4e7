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


def _limbs(x, n=9):
    return [(x >> (29 * i)) & (2**29 - 1) for i in range(n - 1)] + [x >> 232]


def _val(l):
    return sum(int(v) << (29 * i) for i, v in enumerate(l))


def test_fp_reduce64_edges(shim):
    """fp_reduce64 (bn254_cycsq.h): x mod q below 2q for every 0 <= x < 64q, including the values
    on each side of every multiple of q (where the top-limb estimate of the multiple is off by one)."""
    rng = random.Random(0x64)
    xs = [0, 1, 64 * P - 1] + [k * P + d for k in range(1, 64) for d in (-2, -1, 0, 1)]
    xs += [rng.randrange(64 * P) for _ in range(3000)] + [(k * P) | (2**232 - 1) for k in range(1, 63)]
    arr = ctypes.c_uint32 * 9
    for x in xs:
        if not 0 <= x < 64 * P:
            continue
        limbs = _limbs(x)
        out = arr()
        ok = shim.shim_fp_reduce64(arr(*limbs), out)
        assert ok == 1, hex(x)
        r = _val(out)
        assert r % P == x % P and r < 2 * P, hex(x)
    # low limbs up to 2^29 + 7 (the carried form of the squaring's last stage)
    for _ in range(2000):
        lo = [2**29 + rng.randrange(8) if rng.random() < 0.5 else rng.randrange(2**29) for _ in range(8)]
        top = rng.randrange((60 * P - _val(lo + [0])) >> 232)
        limbs = lo + [top]
        out = arr()
        assert shim.shim_fp_reduce64(arr(*limbs), out) == 1
        assert _val(out) % P == _val(limbs) % P


def test_fp_mul_raw_operand_bounds(shim):
    """f_mul with the squaring's unreduced operands (bn254_cycsq.h: cs_operands): U with every low
    limb up to 2^31 - 1 and value < 8q, V normalised < 8q -> U V 2^-261 mod q, below 1.3q."""
    rng = random.Random(0x31)
    arr = ctypes.c_uint32 * 9
    RINV = pow(2**261, -1, P)
    for it in range(1500):
        lo = [rng.randrange(2**31 - 2**29, 2**31) if it % 2 else 2**31 - 1 for _ in range(8)]
        low = _val(lo + [0])
        top_max = (8 * P - 1 - low) >> 232
        u = lo + [rng.randrange(top_max + 1) if it % 3 else top_max]
        v = rng.randrange(8 * P) if it % 5 else 8 * P - 1
        out = arr()
        assert shim.shim_fp_mul_raw(arr(*u), arr(*_limbs(v)), out) == 1
        r = _val(out)
        assert r % P == _val(u) * v * RINV % P
        assert r < 13 * P // 10


def test_cyclotomic_square_lane_emulation(shim):
    """p36_cyc_sqr's lane stages (cs_pre, cs_operands, f_mul, cs_combine, cs_finish) over an
    emulated 36-lane wave, 186 squarings deep (the three x^u chains of a final exponentiation)
    from random cyclotomic elements, equal fp12_sqr; every lane stays reduced, replicas agree."""
    shim.shim_cyc_sqr_emul.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in range(1, 9):
        assert shim.shim_cyc_sqr_emul(seed, 186 if seed < 3 else 20) == 1, seed


def test_fp12_mul_lane_emulation(shim):
    """p36_mul's lane stages (cm_terms, cm_xi, cm_sum3) over an emulated 36-lane wave, chained
    60 multiplications deep from random (non-cyclotomic) elements, equal fp12_mul."""
    shim.shim_p36_mul_emul.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in range(1, 9):
        assert shim.shim_p36_mul_emul(seed, 60 if seed < 3 else 5) == 1, seed


def test_fp12_sqr_lane_emulation(shim):
    """p36_sqr's lane stages (sq_operands + the cm_* stages) over an emulated 36-lane wave, 64
    squarings deep (a Miller loop's worth) from random elements, equal fp12_sqr."""
    shim.shim_p36_sqr_emul.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in range(1, 9):
        assert shim.shim_p36_sqr_emul(seed, 64 if seed < 3 else 5) == 1, seed


def test_g1_lazy_doubling_matches(shim):
    """g1q_dbl's lazy stages (g1d_et, g1d_x3w, g1d_y3; bn254_cycsq.h) as one lane's doubling,
    300 doublings deep from hashed points, equal g1_dbl as affine points; coordinates reduced."""
    shim.shim_g1_dbl_lazy.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in range(1, 7):
        assert shim.shim_g1_dbl_lazy(seed, 300 if seed < 3 else 30) == 1, seed


def test_fp_mul_raw_both_operands(shim):
    """f_mul with BOTH operands unreduced as the G2 line rounds build them (bn254_g2wave.h:
    g2w_mul_ops / g2w_sqr_ops): a + b (limbs < 2^30) times a - b + 2q (limbs < 1.5 2^30), both
    values < 4q, including every low limb at its maximum -> the product mod q, below 2q."""
    rng = random.Random(0x2B)
    arr = ctypes.c_uint32 * 9
    RINV = pow(2**261, -1, P)
    for it in range(1500):
        hi = it % 4 == 0
        lo_u = [2**30 - 1 if hi else rng.randrange(2**30) for _ in range(8)]
        lo_v = [3 * 2**29 - 1 if hi else rng.randrange(3 * 2**29) for _ in range(8)]
        u = lo_u + [rng.randrange(((4 * P - 1 - _val(lo_u + [0])) >> 232) + 1)]
        v = lo_v + [rng.randrange(((4 * P - 1 - _val(lo_v + [0])) >> 232) + 1)]
        assert _val(u) < 4 * P and _val(v) < 4 * P
        out = arr()
        assert shim.shim_fp_mul_raw(arr(*u), arr(*v), out) == 1
        assert _val(out) % P == _val(u) * _val(v) * RINV % P


def test_fp_lin3_combinations(shim):
    """fp_lin3 (bn254_cycsq.h), the one-reduction linear combinations of the G2 line steps:
    3a, a - 2b, 2a - 2b - 2c, a - 4b, a - b - c mod p, including inputs at 0 and p - 1."""
    rng = random.Random(0x13)
    xs = [0, 1, P - 1, P - 2] + [rng.randrange(P) for _ in range(400)]
    for i, a in enumerate(xs):
        b, c = xs[(3 * i + 1) % len(xs)], xs[(7 * i + 2) % len(xs)]
        out = ctypes.create_string_buffer(160)
        assert shim.shim_fp_lin3(a.to_bytes(32, "big"), b.to_bytes(32, "big"), c.to_bytes(32, "big"), out) == 1
        got = [int.from_bytes(out.raw[32 * k:32 * k + 32], "big") for k in range(5)]
        a2 = 2 * a
        assert got == [3 * a2 % P, (a2 - 2 * b) % P, (2 * a2 - 2 * b - 2 * c) % P, (a2 - 4 * b) % P,
                       (a2 - b - c) % P]


def test_secret_scalar_ladders_match_double_and_add(shim):
    """g1_mul_ct / g2_mul_ct (Montgomery ladder over k + 2r, masked swaps: used for signing and
    sk*g2) equal the double-and-add forms for edge and random scalars k < r."""
    import random

    r = 0x2523648240000001BA344D8000000007FF9F800000000010A10000000000000D
    rng = random.Random(5)
    ks = [0, 1, 2, 3, r - 1, r - 2, (r - 1) // 2, 1 << 252, (1 << 253) - 1] + [rng.randrange(r) for _ in range(24)]
    h = ctypes.create_string_buffer(33)
    shim.shim_g1_map(b"ladder", 6, h)
    for k in ks:
        kb = k.to_bytes(32, "big")
        a, b = ctypes.create_string_buffer(33), ctypes.create_string_buffer(33)
        shim.shim_g1_mul(h.raw, kb, a)
        shim.shim_g1_mul_ct(h.raw, kb, b)
        assert a.raw == b.raw, hex(k)
        c, d = ctypes.create_string_buffer(65), ctypes.create_string_buffer(65)
        shim.shim_g2_mul_gen(kb, c)
        shim.shim_g2_mul_gen_ct(kb, d)
        assert c.raw == d.raw, hex(k)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_row_fp_and_g1_emulation(shim, seed):
    """Row-parallel Fp (bn254_row.h) and G1 (bn254_g1row.h) over the host SIMD emulation of the
    gfx950 DPP / ds_bpermute moves, against the one-lane field and group code (0 = no mismatch)."""
    for fn, iters in ((shim.shim_rf_check, 4000), (shim.shim_g1r_check, 60)):
        fn.argtypes = [ctypes.c_uint64, ctypes.c_int]
        assert fn(seed, iters) == 0, fn.__name__


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_row_g2_emulation(shim, seed):
    """Row-parallel G2 (bn254_g2row.h) against the one-lane G2 code: doubling and mixed addition
    with their Miller-loop lines (line_dbl_j / line_add_j values), full Jacobian addition incl.
    T + T and T + (-T), flag-carrying accumulation chains, and the NAF subgroup check against
    r Q == O on points of G2 and twist points off it; every row product's operands are checked
    against rf_mul's bounds (row-normal limbs, (a/q)(b/q) < 221)."""
    shim.shim_g2r_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert shim.shim_g2r_check(seed, 24) == 0


def test_row_g2_subgroup_on_cofactor_torsion():
    """bls_keys_row_kernel's subgroup test (g2r_in_subgroup: psi(Q) = [6u^2]Q) == r Q == O
    (g2_in_subgroup) on points of G2 ([h2] T) and of the cofactor's order-13 and order-96757
    subgroups ([r][h2 / ell] T), T random twist points; host emulation of the row code."""
    import bn254_ref as B
    lib = ctypes.CDLL(SHIM)
    lib.shim_g2r_subgroup_scaled.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_int)]
    h2 = 2 * B.P - B.R

    def words(x):
        return (ctypes.c_uint32 * 8)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)])

    for k1, k2, want in ((h2, 1, 8), (B.R, h2 // 13, 6), (B.R, h2 // 96757, 7), (1, 1, 8)):
        tested = ctypes.c_int(0)
        bad = lib.shim_g2r_subgroup_scaled(k1 * 7 + k2, 8, words(k1), words(k2), ctypes.byref(tested))
        assert bad == 0
        assert tested.value >= want - 1  # a point may have no component in the target subgroup


def test_row_sqrt_power_matches_one_lane(shim):
    """rf_pow_sw (bn254_row.h), the row-parallel square-root power of g1_map_row, on four emulated
    DPP rows: x^((p+1)/4) mod p, equal to the one-lane f_pow_sw, every product within its bounds."""
    rng = random.Random(0x5A27)
    xs = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, 2**253, 2**254 % P] + [rng.randrange(P) for _ in range(63)]
    xs += [1] * (-len(xs) % 4)
    for k in range(0, len(xs), 4):
        buf = b"".join(x.to_bytes(32, "big") for x in xs[k:k + 4])
        out = ctypes.create_string_buffer(128)
        assert shim.shim_rf_sqrt_pow(buf, out) == 1
        for r in range(4):
            assert int.from_bytes(out.raw[32 * r:32 * r + 32], "big") == pow(xs[k + r], (P + 1) // 4, P)


def test_sha256_key_msg_matches_hashlib(shim):
    """sha256_key_msg (sha256.h), the register-resident SHA-256 of the BLS signing / key blinds:
    SHA-256(key bytes ^ x || msg[:m]) for m = 0..64 (one and two blocks, every padding boundary)."""
    import hashlib
    import struct

    rng = random.Random(0x256)
    for m in range(65):
        key = [rng.getrandbits(32) for _ in range(8)]
        x = rng.choice((0, 0x5C))
        msg = bytes(rng.getrandbits(8) for _ in range(m))
        out = ctypes.create_string_buffer(32)
        shim.shim_sha256_key_msg((ctypes.c_uint32 * 8)(*key), x, msg, m, out)
        kb = bytes(b ^ x for b in struct.pack("<8I", *key))
        assert out.raw == hashlib.sha256(kb + msg).digest(), m


@pytest.mark.parametrize("which,p", [(0, P), (1, 2**255 - 19)])
def test_wave_inversion_emulated(shim, which, p):
    """safegcd30.h's wave form (sg_inv30_var_wave: scalar divsteps, lane-parallel limb updates in
    redundant limbs, exact zero test, sg_canon30) over an emulated 64-lane wave, for BN-P254's p
    (the pairing checks' Fp inversion) and 2^255 - 19 (the Ed25519 finish root): equal to x^(p-2),
    0 -> 0, within the batch bound, and the redundant-limb case actually exercised."""
    shim.shim_sg_wave_inv.restype = ctypes.c_long
    rng = random.Random(0x5A7E + which)
    xs = [0, 1, 2, 3, 19, p - 1, p - 2, (p - 1) // 2, (p + 1) // 2, 2**253 % p, 2**128, 2**128 - 1]
    xs += [(1 << k) % p for k in range(0, 255, 3)] + [p - (1 << k) for k in range(0, 250, 9)]
    xs += [rng.randrange(p) for _ in range(3000)]
    red_total = 0
    for x in xs:
        out, red = ctypes.create_string_buffer(32), ctypes.c_long()
        nb = shim.shim_sg_wave_inv(which, x.to_bytes(32, "big"), out, ctypes.byref(red))
        assert int.from_bytes(out.raw, "big") == (pow(x, p - 2, p) if x else 0), hex(x)
        assert 1 <= nb <= 25
        red_total += red.value
    assert red_total > 0
