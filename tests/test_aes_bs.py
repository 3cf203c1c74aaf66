"""CPU pin of the bitsliced AES-256-CTR decomposition (jfsx_aes_bs.h) that
gcm_main runs on the VALU: S-box circuit, 32x32 bit transposes, round-key
folding and the per-lane counter layout (slot k = c0 + 64k), all checked
against the oracle's AES-256 (FIPS-197) on the same keys and counters.  The
header is compiled for the host by g++ with plain-C emulations of v_bitop3 /
v_perm (tests/harness/aes_bs_host.cpp); the GPU parity tests pin the kernel."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def bs(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("bs") / "aes_bs_host.so")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", out,
                           os.path.join(HERE, "harness", "aes_bs_host.cpp")])
    return ctypes.CDLL(out)


def test_sbox_circuit(bs):
    sb = orc.sbox()
    out = ctypes.c_uint32()
    for mask in (0x00, 0x63, 0xA5):
        for x in range(256):
            bs.bs_sbox_byte(x, mask, ctypes.byref(out))
            assert out.value == int(sb[x]) ^ mask


def test_transpose32(bs):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2**32, 32, dtype=np.uint64).astype(np.uint32)
    m = np.array([[(int(a[j]) >> k) & 1 for k in range(32)] for j in range(32)])
    b = a.copy()
    bs.bs_transpose32(b.ctypes.data_as(ctypes.c_void_p))
    mt = np.array([[(int(b[j]) >> k) & 1 for k in range(32)] for j in range(32)])
    assert (mt == m.T).all()


@pytest.mark.parametrize("seed,c0", [(1, 2), (2, 2 + 64 * 32 * 5 + 17), (3, 0xFFFFFFF0), (4, 0x12345678)])
def test_ctr32_matches_oracle(bs, seed, c0):
    key, nonce = orc.gen_key(seed, 0)
    rk = np.frombuffer(orc.aes256_expand(key), dtype="<u4").copy()
    nz = np.frombuffer(bytes(nonce), dtype="<u4").copy()
    out = np.zeros(128, np.uint32)
    bs.bs_ctr32(rk.ctypes.data_as(ctypes.c_void_p), nz.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(c0),
                out.ctypes.data_as(ctypes.c_void_p))
    for k in range(32):
        ctr = (c0 + 64 * k) & 0xFFFFFFFF
        ref = orc.aes256_encrypt_block(key, bytes(nonce) + ctr.to_bytes(4, "big"))
        assert out[4 * k:4 * k + 4].tobytes() == ref, "slot %d" % k

