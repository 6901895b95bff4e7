"""The oracle is pinned before it is trusted: both CPU restatements (pure Python and plain C)
must reproduce every golden verdict (OpenSSL 3.0.2 ground truth) and the RFC 8032 vectors."""
import ctypes
import os

import pytest

import ed25519_ref as E
from golden_io import load_ed25519_vectors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "libcbft_oracle.so")

RFC = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


@pytest.fixture(scope="module")
def vectors():
    return load_ed25519_vectors()


@pytest.fixture(scope="module")
def coracle():
    if not os.path.exists(ORACLE_SO):
        pytest.skip("oracle/libcbft_oracle.so not built (make oracle)")
    return ctypes.CDLL(ORACLE_SO)


@pytest.mark.parametrize("sk,pk,msg,sig", RFC)
def test_python_oracle_rfc8032(sk, pk, msg, sig):
    sk, pk, msg, sig = map(bytes.fromhex, (sk, pk, msg, sig))
    assert E.public_key(sk) == pk
    assert E.sign(sk, msg) == sig
    assert E.verify(pk, msg, sig)


def test_python_oracle_matches_golden(vectors):
    bad = [i for i, v in enumerate(vectors) if int(E.verify(v.pk, v.msg, v.sig)) != v.verdict]
    assert not bad, f"python oracle disagrees with OpenSSL on vectors {bad[:10]}"


def test_c_oracle_matches_golden(vectors, coracle):
    f = coracle.cbft_oracle_ed25519_verify
    bad = [i for i, v in enumerate(vectors)
           if f(v.pk, v.msg, ctypes.c_size_t(len(v.msg)), v.sig) != v.verdict]
    assert not bad, f"C oracle disagrees with OpenSSL on vectors {bad[:10]}"


@pytest.mark.parametrize("sk,pk,msg,sig", RFC)
def test_c_oracle_sign_rfc8032(coracle, sk, pk, msg, sig):
    sk, pk, msg, sig = map(bytes.fromhex, (sk, pk, msg, sig))
    out = ctypes.create_string_buffer(64)
    coracle.cbft_oracle_ed25519_sign(sk, msg, ctypes.c_size_t(len(msg)), out)
    assert out.raw == sig


def test_golden_covers_edge_classes(vectors):
    classes = {v.cls for v in vectors}
    assert set(range(15)) <= classes
    # both verdicts occur among the adversarial small-order / mixed-order classes
    for c in (8, 12):
        assert {v.verdict for v in vectors if v.cls == c} == {0, 1}
