"""Writes tests/golden/bls_sets.txt: BLS BN-P254 key sets for the C++ threshsign host test
(tests/cpp/test_bls_host.cpp).  Everything comes from the Python oracle (oracle/bn254_ref.py):
Shamir keygen as BlsThresholdKeygen, vk_i = sk_i g2, and the expected combined signature
sk * g1_map(msg) (what a correct threshold combine must reproduce byte for byte).  RELIC is not
available here, so parity with RELIC's encodings is unpinned.

Format, one record per line:  set <n> <k> | sk <dec> | pk <hex65> | vk <i> <hex65> |
ski <i> <dec> | msg <hex> | sig <hex33> | end
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bn254_ref as B  # noqa: E402

SETS = [(7, 5, 11), (7, 6, 12), (4, 4, 13), (10, 7, 14)]  # (n, k, seed); (7, 6) = almost-multisig


def main():
    out = []
    for n, k, seed in SETS:
        sk, sks = B.keygen(n, k, seed)
        msg = bytes((seed * 7 + i) & 0xFF for i in range(32))
        out.append(f"set {n} {k}")
        out.append(f"sk {sk}")
        out.append(f"pk {B.g2_to_bytes(B.ec_mul(sk, B.G2_GEN)).hex()}")
        for i in range(1, n + 1):
            out.append(f"vk {i} {B.g2_to_bytes(B.ec_mul(sks[i], B.G2_GEN)).hex()}")
            out.append(f"ski {i} {sks[i]}")
        out.append(f"msg {msg.hex()}")
        out.append(f"sig {B.g1_to_bytes(B.ec_mul(sk, B.g1_map(msg))).hex()}")
        out.append("end")
    with open(os.path.join(HERE, "bls_sets.txt"), "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
