"""N > 1 BLS path on CPU: world-size-2 gloo runs of
cbft_multigpu.bls_verify_shares_sharded / bls_combine_sharded / bls_verify_multisig_sharded.
Each rank's GPU is stood in for by the Python oracle (oracle/bn254_ref.py) and the host build of
the BN-P254 code (tests/cpp/libbn254_shim.so); partial points travel as fixed-size byte strings
exactly like the library's opaque partials.  The sharded results must equal the single-process
ones: the planted bad shares, sk * H(m), and the multisig verdict."""
import multiprocessing as mp
import os
import socket

import pytest

import bn254_ref as B
import blsgen

G1_PART, G2_PART = 108, 220


def _pt_bytes(pt, size, coords):
    if pt is None:
        return bytes(size)
    flat = b""
    for c in pt:
        flat += b"".join(v.to_bytes(32, "big") for v in ([c] if isinstance(c, int) else [c.a, c.b]))
    return (b"\x01" + flat).ljust(size, b"\x00")


def _pt_from(b, g2):
    if b[0] == 0:
        return None
    vals = [int.from_bytes(b[1 + 32 * i:33 + 32 * i], "big") for i in range(4 if g2 else 2)]
    if g2:
        return (B.F2(vals[0], vals[1]), B.F2(vals[2], vals[3]))
    return (vals[0], vals[1])


class OracleBackend:
    """The library's BLS partial API restated over the oracle (test stand-in for one GPU)."""

    def __init__(self, vks):
        self.vks = [B.g2_from_bytes(v) for v in vks]

    def bls_verify_shares(self, kid, msg, shares):
        H = B.g1_map(msg)
        out = []
        for s in shares:
            i, p = B.parse_share(s)
            out.append(1 <= i <= len(self.vks) and B.verify_share(H, p, self.vks[i - 1]))
        return out

    def bls_combine_partial(self, shares, lo, hi, multisig=False):
        parsed = [B.parse_share(s) for s in shares]
        lam = B.lagrange_coeffs([i for i, _ in parsed])
        acc = None
        for i, p in parsed[lo:hi]:
            acc = B.ec_add(acc, p if multisig else B.ec_mul(lam[i], p), None)
        return _pt_bytes(acc, G1_PART, 2)

    def bls_combine_finish(self, parts):
        acc = None
        for b in parts:
            acc = B.ec_add(acc, _pt_from(b, False), None)
        return B.g1_to_bytes(acc)

    def bls_sum_keys_partial(self, kid, bm, lo_id, hi_id):
        acc = None
        for i in range(lo_id, hi_id):
            if bm[(i - 1) // 8] >> ((i - 1) % 8) & 1:
                acc = B.ec_add(acc, self.vks[i - 1], B.F2(0, 0))
        return _pt_bytes(acc, G2_PART, 4)

    def bls_verify_multisig_partials(self, msg, sig33, parts):
        acc = None
        for b in parts:
            acc = B.ec_add(acc, _pt_from(b, True), B.F2(0, 0))
        return acc is not None and B.verify(msg, sig33, acc)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    n, k = 12, 9
    sk, sks, pk, vks = blsgen.keyset(n, k, seed=41, threads=2)
    msg = bytes(range(32))
    ids = [1, 2, 3, 5, 6, 8, 9, 11, 12]
    shares = blsgen.shares(sks, ids, msg, threads=2)
    bad = list(shares)
    bad[4] = blsgen.doubled(bad[4])
    return n, sk, vks, msg, ids, shares, bad


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import cbft_multigpu as mg

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, sk, vks, msg, ids, shares, bad = _case()
    be = OracleBackend(vks)
    valid = mg.bls_verify_shares_sharded(be, 1, msg, bad, world, rank, dist, "cpu")
    sig = mg.bls_combine_sharded(be, shares, world, rank, dist, "cpu")
    msig = mg.bls_combine_sharded(be, shares, world, rank, dist, "cpu", multisig=True)
    ok = mg.bls_verify_multisig_sharded(be, 1, n, msg, msig, B.signers_bitmap(ids), world, rank, dist, "cpu")
    nok = mg.bls_verify_multisig_sharded(be, 1, n, msg, msig, B.signers_bitmap(ids[:-1]), world, rank, dist, "cpu")
    q.put((rank, [bool(v) for v in valid], sig, ok, nok))
    dist.destroy_process_group()


def test_slices_cover():
    import cbft_multigpu as mg

    for k in (1, 7, 8, 9, 683, 1024):
        for w in (1, 2, 3, 8):
            sl = [mg.share_slice(k, w, r) for r in range(w)]
            assert sl[0][0] == 0 and sl[-1][1] == k and all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert all(lo % 8 == 0 or lo == k for lo, _ in sl)
            il = [mg.id_slice(k, w, r) for r in range(w)]
            assert il[0][0] == 1 and il[-1][1] == k + 1 and all(a[1] == b[0] for a, b in zip(il, il[1:]))


@pytest.mark.timeout(600)
def test_gloo_world2_bls_sharded():
    n, sk, vks, msg, ids, shares, bad = _case()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=500) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_valid = [j != 4 for j in range(len(bad))]
    want_sig = blsgen.sign_point(sk, msg)
    for r in range(2):
        valid, sig, ok, nok = res[r]
        assert valid == want_valid
        assert sig == want_sig
        assert ok and not nok
