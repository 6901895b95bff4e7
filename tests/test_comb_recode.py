"""CPU check of the signed radix-2^w comb recoding the key-table ladder uses
(concord-bft_amd/csrc/ed25519_verify.hip: ed25519_comb_ladder_kernel; geometry in
csrc/ed25519_verify.h: cbft_comb_npos).

For s < L: s' = s + 2^(w-1) * sum_{j < npos-1} 2^(w j); d_j = chunk_j(s') - 2^(w-1) below the
top position, d_top = chunk_top(s').  Then sum_j d_j 2^(w j) == s, every |d_j| <= 2^(w-1) (the
table has entries 0 .. 2^(w-1)), and npos is the least position count for which that holds."""
import random

import pytest

L = 2**252 + 27742317777372353535851937790883648493
NPOS = {8: 32, 9: 29, 10: 26, 11: 23, 12: 22, 13: 20, 14: 19, 15: 17, 16: 16, 17: 15, 18: 15, 19: 14, 20: 13,
        21: 13, 22: 12, 23: 11, 24: 11, 25: 11, 26: 10}
B_RADICES = (16, 22, 24, 26)  # B's table: CBFT_COMB_B_RADIX (22) and cbft_set_option(CBFT_OPT_B_RADIX) alternatives


def offset(w, npos):
    return sum(1 << (w * j + w - 1) for j in range(npos - 1))


def recode(s, w, npos):
    sp = (s + offset(w, npos)) % (1 << 256)
    half = 1 << (w - 1)
    ds = []
    for j in range(npos):
        ch = (sp >> (w * j)) & ((1 << w) - 1)
        ds.append(ch if j == npos - 1 else ch - half)
    return ds


def edge_scalars():
    rng = random.Random(0xC0FFEE)
    xs = [0, 1, 2, L - 1, L - 2, 2**252, 2**252 - 1, (L - 1) // 2]
    xs += [rng.randrange(L) for _ in range(300)]
    # scalars whose low chunks all sit at the signed-digit boundaries
    for w in NPOS:
        xs.append(sum(((1 << (w - 1)) - 1) << (w * j) for j in range(256 // w)) % L)
        xs.append(sum((1 << (w - 1)) << (w * j) for j in range(256 // w)) % L)
    return xs


@pytest.mark.parametrize("w", sorted(NPOS))
def test_recode_sums_and_ranges(w):
    npos = NPOS[w]
    half = 1 << (w - 1)
    for s in edge_scalars():
        ds = recode(s, w, npos)
        assert sum(d << (w * j) for j, d in enumerate(ds)) == s
        assert all(-half <= d <= half - 1 for d in ds[:-1])
        assert 0 <= ds[-1] <= half
        assert -(1 << 25) <= min(ds) and max(ds) <= 1 << 25  # the ladders' digits (int32 in LDS / registers)


@pytest.mark.parametrize("w", sorted(NPOS))
def test_npos_is_minimal(w):
    npos = NPOS[w]
    # with one position fewer, the largest scalar's top digit leaves the table
    ds = recode(L - 1, w, npos - 1)
    assert ds[-1] > (1 << (w - 1)) or sum(d << (w * j) for j, d in enumerate(ds)) != L - 1


def test_lane_split_covers_all_positions():
    # additions dealt to the 4 lanes of a quad: lane q takes q*nper .. q*nper+nper-1
    for wa in range(8, 14):
        for wb in B_RADICES:
            total = NPOS[wa] + NPOS[wb]
            nper = (total + 3) // 4
            assert nper <= 12  # COMB_MAX_STEPS
            seen = [q * nper + jj for q in range(4) for jj in range(nper) if q * nper + jj < total]
            assert seen == list(range(total))
    # the default geometry: radix-2^13 keys + radix-2^22 B = 32 additions, 8 per lane
    assert (NPOS[13] + NPOS[22] + 3) // 4 == 8
