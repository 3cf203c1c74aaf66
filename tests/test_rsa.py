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
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", out,
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


def test_exponentiation_schedule_is_independent_of_the_exponent(rsa, keypair):
    """Constant time in the private exponent (as Go's crypto/internal/bigmod
    Exp, which rsa.DecryptOAEP uses; encrypt.go:132-134): the sequence of
    Montgomery products and window-table reads is the same for the key's real
    CRT exponent, a tiny one, an all-ones one and zero -- 3-bit fixed window
    over the full 1024 bits, one multiply per digit, every table entry read
    for every digit -- and every result equals pow().  (The exponentiation is
    mod_exp28, the one the GPU kernel runs, in 28-bit limbs.)"""
    _, _, comps = keypair
    p = comps[0]
    pi = int.from_bytes(p, "big")
    x = int.from_bytes(os.urandom(127), "big") % pi
    traces = set()
    for e in (int.from_bytes(comps[2], "big"), 3, (1 << 1024) - 1, 0, 1 << 1023, 0x10001):
        out = ctypes.create_string_buffer(128)
        ops = ctypes.c_uint64()
        rsa.rsa_exp_trace.restype = ctypes.c_uint64
        h = rsa.rsa_exp_trace(p, e.to_bytes(128, "big"), x.to_bytes(128, "big"), out, ctypes.byref(ops))
        assert int.from_bytes(out.raw, "big") == pow(x, e, pi)
        traces.add((h, ops.value))
    # edge bases: 0, 1 and m - 1 (the largest reduced value)
    for xe in (0, 1, pi - 1):
        out = ctypes.create_string_buffer(128)
        ops = ctypes.c_uint64()
        e = int.from_bytes(comps[2], "big")
        h = rsa.rsa_exp_trace(p, e.to_bytes(128, "big"), xe.to_bytes(128, "big"), out, ctypes.byref(ops))
        assert int.from_bytes(out.raw, "big") == pow(xe, e, pi), xe
        traces.add((h, ops.value))
    assert len(traces) == 1, traces
    (_, nops), = traces
    # table (8), 342 digits x (3 sq + 1 mul), exit; 8 reads per digit
    assert nops == 8 + 342 * 4 + 1 + 342 * 8


def test_pair_exponentiation_matches_pow_with_one_trace(rsa, keypair):
    """mod_exp28_pair, the GPU kernel's form (each Montgomery product split by
    columns over two lanes that exchange words per row), run on the CPU as two
    threads in lock step: every result equals pow(), both lanes return it,
    and the operation trace is one and the same for every exponent and base,
    as for mod_exp28."""
    _, _, comps = keypair
    for m in (comps[0], comps[1]):
        mi = int.from_bytes(m, "big")
        traces = set()
        cases = [(int.from_bytes(os.urandom(127), "big") % mi, e)
                 for e in (int.from_bytes(comps[2], "big"), 3, (1 << 1024) - 1, 0, 0x10001)]
        cases += [(xe, int.from_bytes(comps[3], "big")) for xe in (0, 1, mi - 1)]
        for xv, e in cases:
            out = ctypes.create_string_buffer(128)
            ops, same = ctypes.c_uint64(), ctypes.c_int()
            rsa.rsa_exp_pair_trace.restype = ctypes.c_uint64
            h = rsa.rsa_exp_pair_trace(m, e.to_bytes(128, "big"), xv.to_bytes(128, "big"), out,
                                       ctypes.byref(ops), ctypes.byref(same))
            assert same.value == 1
            assert int.from_bytes(out.raw, "big") == pow(xv, e, mi), (xv, e)
            traces.add((h, ops.value))
        assert len(traces) == 1, traces
        (_, nops), = traces
        assert nops == 8 + 342 * 4 + 1 + 342 * 8


def _oaep_encode(msg, seed, label=b"keys", k=256, db_patch=None):
    import hashlib as h
    lh = h.sha256(label).digest()
    ps = b"\0" * (k - len(msg) - 2 * 32 - 2)
    db = bytearray(lh + ps + b"\x01" + msg)
    if db_patch:
        db_patch(db)

    def mgf(s, n):
        out = b""
        c = 0
        while len(out) < n:
            out += h.sha256(s + c.to_bytes(4, "big")).digest()
            c += 1
        return out[:n]
    mdb = bytes(a ^ b for a, b in zip(db, mgf(seed, len(db))))
    ms = bytes(a ^ b for a, b in zip(seed, mgf(mdb, 32)))
    return bytearray(b"\0" + ms + mdb)


def test_oaep_decode_checks_without_branching_on_the_data(rsa):
    """The decode's outcomes, each reached by the masked scan (RFC 8017
    7.1.2 step 3g, Go's decryptOAEP): good messages of every length decode;
    a nonzero first byte, a wrong label hash, a missing 0x01 separator, or a
    nonzero byte in the padding all give the one decryption error."""
    seed = os.urandom(32)
    for n in (0, 1, 32, 190):
        m = os.urandom(n)
        em = _oaep_encode(m, seed)
        buf = ctypes.create_string_buffer(bytes(em), 256)
        assert rsa.oaep(buf, b"keys", 4) == n and buf.raw[:n] == m
    bad = []
    em = _oaep_encode(b"k" * 32, seed)
    em[0] = 1
    bad.append(em)
    bad.append(_oaep_encode(b"k" * 32, seed, label=b"other"))
    bad.append(_oaep_encode(b"", seed, db_patch=lambda db: db.__setitem__(len(db) - 1, 0)))  # no 0x01 at all
    bad.append(_oaep_encode(b"k" * 32, seed, db_patch=lambda db: db.__setitem__(40, 7)))  # junk in the padding
    bad.append(_oaep_encode(b"k" * 32, seed, db_patch=lambda db: db.__setitem__(40, 2)))
    for em in bad:
        buf = ctypes.create_string_buffer(bytes(em), 256)
        assert rsa.oaep(buf, b"keys", 4) == -1
