"""Runs the C++ host-side test (IVerifier/ISigner/SigManager mirror over the C ABI)."""
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
