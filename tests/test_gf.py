"""CPU pin of the integer-multiply GF(2^128) product (juicefs_amd/csrc/jfsx_gf.h)
that GHASH's per-lane lifts use: equal to the bit-serial product of SP 800-38D
Algorithm 1 and to a Python carry-less product with the GCM reduction."""
import ctypes
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gf(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("gf") / "gf_host.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC",
                           "-o", out, os.path.join(HERE, "harness", "gf_host.cpp")])
    L = ctypes.CDLL(out)
    L.gf_clmul32.restype = ctypes.c_uint64
    L.gf_clmul32.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.gf_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    return L


def _have(tool):
    from shutil import which
    return which(tool) is not None


def _clmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        b >>= 1
    return r


def _ghash_mul(x, y):
    """x, y: 128-bit integers in plain order (bit i = x^i)."""
    p = _clmul(x, y)
    for i in range(254, 127, -1):
        if (p >> i) & 1:
            p ^= (1 << i) | (0x87 << (i - 128))
    return p


def _words_to_plain(w):
    v = 0
    for k in range(4):
        for b in range(32):
            if (w[k] >> (31 - b)) & 1:
                v |= 1 << (32 * k + b)
    return v


def test_clmul32_matches_python(gf):
    rnd = random.Random(3)
    for _ in range(2000):
        a, b = rnd.getrandbits(32), rnd.getrandbits(32)
        assert gf.gf_clmul32(a, b) == _clmul(a, b)
    for a, b in ((0xffffffff, 0xffffffff), (0x80000001, 0xffffffff), (0, 0x1234)):
        assert gf.gf_clmul32(a, b) == _clmul(a, b)


def test_product_matches_bit_serial(gf):
    assert gf.gf_check(0x9E3779B97F4A7C15, 20000) == 0


def test_product_matches_python_reduction(gf):
    rnd = random.Random(7)
    W = ctypes.c_uint32 * 4
    for _ in range(300):
        x = [rnd.getrandbits(32) for _ in range(4)]
        y = [rnd.getrandbits(32) for _ in range(4)]
        z = W()
        gf.gf_mul(W(*x), W(*y), z)
        assert _words_to_plain(list(z)) == _ghash_mul(_words_to_plain(x), _words_to_plain(y))
