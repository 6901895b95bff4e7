"""Loader for tests/golden/relic_bls_keys.json: the RELIC-generated BLS BN-P254 key material of the
reference's own test key files (tests/simpleKVBC/scripts/set{A,B}_replica_*; extracted by
tests/golden/gen_relic_key_fixture.py).  One record per (key set, cryptosystem)."""
import json
import os
from dataclasses import dataclass
from typing import Dict, List

import bn254_ref as B

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "relic_bls_keys.json")


@dataclass
class RelicSystem:
    name: str            # e.g. "setA/slow_commit"
    type: str            # threshold-bls | multisig-bls
    n: int
    threshold: int
    pk: bytes            # 65-byte compressed G2 group key
    vks: List[bytes]     # vk_1..vk_n, 65 bytes each
    sks: Dict[int, int]  # share id -> secret share

    @property
    def multisig(self) -> bool:
        # Cryptosystem forces multisig when threshold == n (ThresholdSignaturesTypes.cpp:31,44-47)
        return self.type == "multisig-bls" or self.threshold == self.n

    def group_secret(self) -> int:
        if self.multisig:
            return sum(self.sks.values()) % B.R
        ids = sorted(self.sks)[: self.threshold]
        lam = B.lagrange_coeffs(ids)
        return sum(lam[i] * self.sks[i] for i in ids) % B.R


def load() -> List[RelicSystem]:
    doc = json.load(open(PATH))
    out = []
    for sname, systems in sorted(doc["sets"].items()):
        for cname, r in sorted(systems.items()):
            out.append(RelicSystem(f"{sname}/{cname}", r["type"], r["n"], r["threshold"],
                                   bytes.fromhex(r["public_key"]), [bytes.fromhex(h) for h in r["verification_keys"]],
                                   {int(i): int(v) for i, v in r["secret_shares"].items()}))
    return out
