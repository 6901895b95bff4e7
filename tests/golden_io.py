"""Reader for tests/golden/ed25519_vectors.bin (format: tests/golden/gen_ed25519_vectors.py)."""
import os
import struct
from dataclasses import dataclass

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ed25519_vectors.bin")


@dataclass
class Vec:
    cls: int
    verdict: int
    pk: bytes
    sig: bytes
    msg: bytes


def load_ed25519_vectors(path: str = GOLDEN):
    data = open(path, "rb").read()
    assert data[:16] == b"CBFTED25519V1\0\0\0", "bad golden header"
    (n,) = struct.unpack_from("<I", data, 16)
    off = 20
    out = []
    for _ in range(n):
        mlen, v, cls, _pad = struct.unpack_from("<IBBH", data, off)
        off += 8
        pk = data[off:off + 32]
        sig = data[off + 32:off + 96]
        msg = data[off + 96:off + 96 + mlen]
        off += 96 + mlen
        out.append(Vec(cls, v, pk, sig, msg))
    assert off == len(data)
    return out
