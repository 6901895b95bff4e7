"""Runs the C++ host-side tests of the plugin layer (concord::hip verifiers, HipSigManager over the
reference-restating SigManager base, request-batch walkers, BLS::Hip) and the per-request bench."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_host")


@pytest.mark.gpu
def test_cpp_host_sigmanager():
    if not os.path.exists(BIN):
        pytest.fail("tests/cpp/test_host not built (make host)")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_cpp_host_binary_built():
    # the host library and test binary link against the C ABI (no GPU needed to link)
    assert os.path.exists(os.path.join(ROOT, "concord-bft_amd", "libcbft_host.so")) or not os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_threshsign_bls():
    """BLS::Hip threshold/multisig verifier, accumulator and signer (threshsign mirror)."""
    exe = os.path.join(ROOT, "tests", "cpp", "test_bls_host")
    if not os.path.exists(exe):
        pytest.fail("tests/cpp/test_bls_host not built (make host)")
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden", "bls_sets.txt")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


@pytest.mark.gpu
def test_host_bench_per_request_path_exact():
    """tools/host_bench (the per-request leg bench.py reports): threads calling verify() and
    SigManager::verifySig() concurrently, every verdict checked against the planted corruptions
    and against OpenSSL on the host."""
    import json

    exe = os.path.join(ROOT, "tools", "host_bench")
    if not os.path.exists(exe):
        pytest.fail("tools/host_bench not built (make host)")
    r = subprocess.run([exe, "16", "150", "64", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout)
    for leg in ("verify_mt", "verifysig_mt", "single", "openssl_mt"):
        assert res[leg]["mismatches"] == 0
    assert res["verify_mt"]["gpu_batches"] < res["verify_mt"]["calls"]  # concurrent calls coalesce
