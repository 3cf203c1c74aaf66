"""CPU pin of the batched RSA-OAEP key unwrap arithmetic (jfsx_rsa.h):
Montgomery CRT exponentiation, SHA-256/MGF1 and EME-OAEP decoding, compiled
for the host (tests/harness/rsa_host.cpp) and checked against libcrypto's
RSA-OAEP(SHA-256, label "keys") -- the rsaEncryptor of
pkg/object/encrypt.go:124-134 -- on freshly generated 2048-bit keys."""
import ctypes
import hashlib
import os
import subprocess

import pytest

from juicefs_amd import encrypt as enc

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def rsa(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("rsa") / "rsa_host.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", out,
                           os.path.join(HERE, "harness", "rsa_host.cpp")])
    return ctypes.CDLL(out)


def crt_components(priv):
    """p, q, dp, dq, qinv of an EVP_PKEY as 128-byte big-endian strings."""
    return enc.rsa_crt_components(priv)


@pytest.fixture(scope="module")
def keypair():
    priv = enc.GenerateRsaKey(2048)
    return priv, enc.NewRSAEncryptor(priv), crt_components(priv)


def unwrap(rsa, comps, ct, label=b"keys"):
    msg = ctypes.create_string_buffer(256)
    ctb = bytes(ct).rjust(256, b"\0")
    n = rsa.rsa_unwrap(*comps, label, len(label), ctb, msg)
    return None if n < 0 else msg.raw[:n]


def test_sha256(rsa):
    out = ctypes.create_string_buffer(32)
    for m in (b"", b"abc", b"keys", bytes(range(256)) * 3, b"x" * 55, b"y" * 56, b"z" * 64):
        rsa.sha256(m, len(m), out)
        assert out.raw == hashlib.sha256(m).digest()


def test_unwrap_matches_libcrypto(rsa, keypair):
    _, rsae, comps = keypair
    for i in range(6):
        key = os.urandom(32) if i else bytes(32)
        ct = rsae.Encrypt(key)
        assert len(ct) == 256
        assert rsae.Decrypt(ct) == key
        assert unwrap(rsa, comps, ct) == key


def test_unwrap_other_lengths(rsa, keypair):
    _, rsae, comps = keypair
    for n in (0, 1, 31, 33, 190):  # OAEP-SHA256 capacity of RSA-2048 is 190 bytes
        m = os.urandom(n)
        assert unwrap(rsa, comps, rsae.Encrypt(m)) == m


def test_unwrap_errors(rsa, keypair):
    priv, rsae, comps = keypair
    ct = bytearray(rsae.Encrypt(os.urandom(32)))
    ct[100] ^= 1
    assert unwrap(rsa, comps, bytes(ct)) is None            # corrupted
    good = rsae.Encrypt(os.urandom(32))
    assert unwrap(rsa, comps, good, label=b"other") is None  # wrong label -> lHash mismatch
    assert unwrap(rsa, comps, b"\xff" * 256) is None         # c >= n
