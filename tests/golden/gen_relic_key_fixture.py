"""Writes tests/golden/relic_bls_keys.json: the RELIC-generated BLS BN-P254 key material held in
the reference's own test key files, /root/reference/tests/simpleKVBC/scripts/set{A,B}_replica_*
(produced by the reference's tools/GenerateConcordKeys.cpp with RELIC @0998bfcb).  Data only:
for every cryptosystem of every key set — type, n, threshold, the group public key and the n
verification keys (65-byte compressed G2, hex as in the files) and each replica's decimal secret
key share (replica r's file holds share r + 1).  These pin the G2 codec (sk_i * g2 == vk_i byte
for byte) and the key algebra (Lagrange / sum of the vks == the group key) without RELIC.

Run in the build container (the reference tree is absent on the GPU box):
    python3 tests/golden/gen_relic_key_fixture.py
"""
import glob
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/tests/simpleKVBC/scripts"
SYSTEMS = ("execution", "slow_commit", "commit", "optimistic_commit")


def parse(path):
    txt = open(path).read()
    rid = int(re.search(r"^replica_id: (\d+)", txt, re.M).group(1))
    out = {}
    for s in SYSTEMS:
        def field(name, pat=r"(\S+)"):
            return re.search(rf"^{s}_cryptosystem_{name}: {pat}", txt, re.M).group(1)
        vks = re.search(rf"^{s}_cryptosystem_verification_keys:\n((?:  - \w+\n)+)", txt, re.M).group(1)
        out[s] = {"type": field("type"), "subtype": field("subtype_parameter"),
                  "n": int(field("num_signers")), "threshold": int(field("threshold")),
                  "public_key": field("public_key"), "verification_keys": re.findall(r"- (\w+)", vks),
                  "private_key": field("private_key", r"(\d+)")}
    return rid, out


def main():
    sets = {}
    for path in sorted(glob.glob(os.path.join(SRC, "set*_replica_*"))):
        name = os.path.basename(path).split("_replica_")[0]
        rid, systems = parse(path)
        st = sets.setdefault(name, {})
        for s, v in systems.items():
            rec = st.setdefault(s, {k: v[k] for k in ("type", "subtype", "n", "threshold", "public_key",
                                                      "verification_keys")})
            assert rec["public_key"] == v["public_key"] and rec["verification_keys"] == v["verification_keys"]
            rec.setdefault("secret_shares", {})[str(rid + 1)] = v["private_key"]
    doc = {"source": "reference tests/simpleKVBC/scripts/set{A,B}_replica_* (RELIC-generated)",
           "sets": sets}
    with open(os.path.join(HERE, "relic_bls_keys.json"), "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
