"""Writes tests/golden/relic_bls_vectors.json: expected BLS BN-P254 signing / combination bytes
under the reference's own RELIC key files (tests/golden/relic_bls_keys.json, extracted from
/root/reference/tests/simpleKVBC/scripts/set{A,B}_replica_* by gen_relic_key_fixture.py),
computed with the pure-Python restatement oracle/bn254_ref.py — not with the HIP code or its host
build — so the GPU's signing, Lagrange combination and encodings are checked against an
independent implementation.  Data only; bench.py's parity gate and __graft_entry__.smoke() read
it on the GPU box without importing the oracle.

Per cryptosystem (8): a 32-byte digest, every replica's 37-byte share of it
(BlsThresholdSigner::signData, BlsThresholdSigner.cpp:32-47), one "doubled" bad share
(TestBlsBatchVerifier.cpp:84-90), the expected combined signature (threshold: Lagrange over any
`threshold` shares, BlsThresholdAccumulator.cpp:42-55; multisig: the sum of all shares,
BlsMultisigAccumulator.cpp:57-65) and the signer subsets to combine.  g1_map (RELIC ep_map) is
parity unpinned; the G2 keys and the G1/G2 codecs are pinned by the key file.

    python3 tests/golden/gen_relic_sign_vectors.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import bn254_ref as B  # noqa: E402
import relic_keys  # noqa: E402


def main():
    out = {"source": "oracle/bn254_ref.py over tests/golden/relic_bls_keys.json", "systems": []}
    for s in relic_keys.load():
        msg = bytes((7 * len(s.name) + i) & 0xFF for i in range(32))
        shares = [B.sign_share(s.sks[i], i, msg) for i in range(1, s.n + 1)]
        bad = shares[0][:4] + B.g1_to_bytes(B.ec_mul(2, B.parse_share(shares[0])[1]))
        expected = B.g1_to_bytes(B.ec_mul(s.group_secret(), B.g1_map(msg)))
        if s.multisig:
            subsets = [list(range(1, s.n + 1))]
        else:
            subsets = [list(range(lo + 1, lo + 1 + s.threshold)) for lo in range(s.n - s.threshold + 1)]
        for ids in subsets:  # the oracle's own combination agrees with sk * H(m)
            sub = {i: B.parse_share(shares[i - 1])[1] for i in ids}
            comb = B.combine_threshold(sub) if not s.multisig else None
            if comb is not None:
                assert B.g1_to_bytes(comb) == expected, (s.name, ids)
        out["systems"].append({"name": s.name, "msg": msg.hex(), "h_g1": B.g1_to_bytes(B.g1_map(msg)).hex(),
                               "shares": [x.hex() for x in shares], "bad_share": bad.hex(),
                               "combined": expected.hex(), "subsets": subsets})
    path = os.path.join(HERE, "relic_bls_vectors.json")
    json.dump(out, open(path, "w"), indent=1)
    print(f"wrote {path}: {len(out['systems'])} systems")


if __name__ == "__main__":
    main()
