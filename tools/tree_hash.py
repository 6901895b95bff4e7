"""Stamp of the device-code tree: sha256 over concord-bft_amd/csrc/* (name + bytes, sorted), 16 hex.

PMC records under profiles/ carry the stamp of the tree they were collected on; bench.py attaches
a record to its line only while the stamp still matches the tree it runs (a stale record is
dropped and the line says so)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "concord-bft_amd", "csrc")


def csrc_tree_hash() -> str:
    h = hashlib.sha256()
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".hip", ".h", ".cpp")):
            continue
        h.update(name.encode())
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(csrc_tree_hash() + "\n")
