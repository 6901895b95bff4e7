"""Writes tests/golden/bls_sets.txt: BLS BN-P254 key sets for the C++ threshsign host test
(tests/cpp/test_bls_host.cpp).

* First the reference's own RELIC-generated cryptosystems (tests/golden/relic_bls_keys.json, from
  tests/simpleKVBC/scripts/set{A,B}_replica_*): pk, vk_i and the secret shares exactly as RELIC
  wrote them; the group secret is interpolated from the shares (threshold) or summed (multisig,
  also when threshold == n, as Cryptosystem forces, ThresholdSignaturesTypes.cpp:31,44-47).
* Then larger sets from the Python oracle (Shamir keygen as BlsThresholdKeygen).
The expected combined signature is group_sk * g1_map(msg) from the oracle (hash-to-G1 itself is
RELIC-unpinned; the point encodings are pinned by the reference's key files).

Format, one record per line:  set <n> <k> | scheme threshold|multisig | sk <dec> | pk <hex65> |
vk <i> <hex65> | ski <i> <dec> | msg <hex> | sig <hex33> | end
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bn254_ref as B  # noqa: E402

SETS = [(7, 5, 11), (7, 6, 12), (4, 4, 13), (10, 7, 14)]  # (n, k, seed); (7, 6) = almost-multisig


def reference_sets(out):
    sys.path.insert(0, os.path.join(HERE, ".."))
    import relic_keys
    for r, s in enumerate(relic_keys.load()):
        sk = s.group_secret()
        msg = bytes((r * 13 + i) & 0xFF for i in range(32))
        out.append(f"set {s.n} {s.threshold}")
        out.append(f"scheme {'multisig' if s.multisig else 'threshold'}")
        out.append(f"sk {sk}")
        out.append(f"pk {s.pk.hex()}")
        for i in range(1, s.n + 1):
            out.append(f"vk {i} {s.vks[i - 1].hex()}")
            out.append(f"ski {i} {s.sks[i]}")
        out.append(f"msg {msg.hex()}")
        out.append(f"sig {B.g1_to_bytes(B.ec_mul(sk, B.g1_map(msg))).hex()}")
        out.append("end")


def main():
    out = []
    reference_sets(out)
    for n, k, seed in SETS:
        sk, sks = B.keygen(n, k, seed)
        msg = bytes((seed * 7 + i) & 0xFF for i in range(32))
        out.append(f"set {n} {k}")
        out.append("scheme threshold")
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
