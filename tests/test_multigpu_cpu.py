"""N > 1 path on CPU: world-size-2 gloo run of the static shard + all-gather of verdict words
(concord-bft_amd/cbft_multigpu.py).  Each rank verifies its shard with the host OpenSSL path
standing in for its GPU; the gathered bitmap must equal the single-process bitmap."""
import os
import socket

import numpy as np
import pytest

import cbft_multigpu as mg


def test_shard_bounds_cover_and_align():
    for n in (1, 63, 64, 65, 1000, 65536, 1 << 20, 1048577):
        for w in (1, 2, 3, 4, 8):
            spans = [mg.shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            for lo, _ in spans:
                assert lo % 64 == 0 or lo == n


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, result_q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import workload

    ss = workload.make_sigset(n, nkeys=16, msg_len=(64, 300), seed=5, invalid_frac=0.2, threads=2,
                              compute_expected=False)

    def verify_range(lo, hi, out_words):
        sub = workload.SigSet(ss.pk, ss.key_idx[lo:hi], ss.sig[lo:hi], ss.blob, ss.off[lo:hi], ss.len[lo:hi],
                              None)
        v = workload.cpu_verify(sub, threads=2).astype(np.uint8)
        bits = np.packbits(v, bitorder="little")
        buf = np.zeros(out_words.numel() * 8, dtype=np.uint8)
        buf[: bits.size] = bits
        out_words.copy_(torch.from_numpy(buf.view(np.int64)))

    g = mg.verify_sharded(n, world, rank, verify_range, dist, "cpu")
    result_q.put((rank, g.numpy().view(np.uint8).tobytes()))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_gather_matches_single_process():
    import multiprocessing as mp

    import workload

    n = 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ss = workload.make_sigset(n, nkeys=16, msg_len=(64, 300), seed=5, invalid_frac=0.2, threads=2)
    want = np.packbits(ss.expected.astype(np.uint8), bitorder="little").tobytes()
    for r in range(2):
        got = res[r][: len(want)]
        assert got == want
    assert 0 < ss.expected.sum() < n
