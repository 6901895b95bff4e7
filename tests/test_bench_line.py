"""bench.py's line carries only current evidence: PMC records are attached
only while their csrc stamp matches the tree, and the fields the driver's stdout tail must keep
come last.  CPU-only: the helpers, not a GPU run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import tree_hash  # noqa: E402


def test_tree_hash_stable_and_sensitive(tmp_path, monkeypatch):
    h = tree_hash.csrc_tree_hash()
    assert h == tree_hash.csrc_tree_hash() and len(h) == 16
    fake = tmp_path / "csrc"
    fake.mkdir()
    (fake / "a.hip").write_text("x")
    monkeypatch.setattr(tree_hash, "CSRC", str(fake))
    h1 = tree_hash.csrc_tree_hash()
    (fake / "a.hip").write_text("y")
    assert tree_hash.csrc_tree_hash() != h1
    (fake / "notes.txt").write_text("ignored")
    (fake / "a.hip").write_text("x")
    assert tree_hash.csrc_tree_hash() == h1


def test_pmc_record_stamp(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    rec = {"csrc_tree": tree_hash.csrc_tree_hash(), "kernels": {"k": {"duration_ms": 1.5, "hbm_bytes": 10}}}
    (prof / "pmc_x.json").write_text(json.dumps(rec))
    k, why = bench._pmc_record("pmc_x.json", "k")
    assert k["duration_ms"] == 1.5 and "csrc tree" in why
    assert bench._pmc_record("pmc_x.json", "other")[0] is None
    rec["csrc_tree"] = "0" * 16
    (prof / "pmc_x.json").write_text(json.dumps(rec))
    k, why = bench._pmc_record("pmc_x.json", "k")
    assert k is None and "stale" in why
    assert bench._pmc_record("absent.json", "k")[0] is None
    brief = bench._pmc_brief({"duration_ms": 0.123456789, "hbm_bytes": 7, "junk": 1}, "src")
    assert brief == {"source": "src", "duration_ms": 0.1235, "hbm_bytes": 7}


def test_parity_counts():
    parity = {"ed25519_golden": {"vectors": 1145, "accept": 176, "mismatch": 0, "classes": {"a": {"n": 1}}},
              "relic_bls_fixture": {"vk_sk_g2": 40, "systems": 8},
              "config3_mixed": {"n": 65536, "invalid": 6488, "mismatch": 0, "pipelined_exact": True},
              "config4_bls": {"shares": 760, "planted_bad": 76, "share_verdict_mismatch": 0}}
    c = bench._parity_counts(parity)
    assert c["ed25519_golden"] == {"n": 1145, "mismatch": 0}
    assert c["relic_bls_fixture"] == {"checks": 48, "mismatch": 0}
    assert c["config3_mixed"] == {"n": 65536, "mismatch": 0}
    assert c["config4_bls"] == {"n": 760, "mismatch": 0}


def test_line_tail_order():
    """The last keys of the line are the ones VERDICT r3 asked the driver's tail to keep."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    block = src[src.index("        out = {\n            \"metric\""):src.index("        print(json.dumps(out)")]
    keys = [ln.strip().split('"')[1] for ln in block.splitlines() if ln.strip().startswith('"') and '":' in ln]
    assert keys[0] == "metric"
    assert keys[-1] == "p50_latency_ms_batch1k"
    tail = keys[-8:]
    for k in ("pcie_inclusive_value", "key_table_load_ms", "per_request_path", "bls_config4"):
        assert k in tail, (k, tail)
