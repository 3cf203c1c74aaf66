"""The LZ4 oracle (oracle/jfs_lz4.c) pinned: against the committed golden
fixtures (compressed length + SHA-256 written by the LZ4 C library, see
tests/golden/make_lz4_golden.py) and, where the system liblz4 is loadable,
against it directly on the same inputs and on malformed streams."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests import lz4_data

GOLD = os.path.join(os.path.dirname(__file__), "golden", "lz4_golden.json")


def _sys_lz4():
    try:
        return ctypes.CDLL("liblz4.so.1")
    except OSError:
        return None


def test_golden_fixtures():
    g = json.load(open(GOLD))
    assert len(g["cases"]) == len(lz4_data.KINDS) * len(lz4_data.GOLDEN_SIZES)
    for c in g["cases"]:
        src = lz4_data.sample(c["kind"], c["n"], c["seed"])
        assert hashlib.sha256(src).hexdigest() == c["in_sha256"]
        assert orc.lz4_bound(c["n"]) == c["bound"]
        out = orc.lz4_compress(src)
        assert len(out) == c["out_len"], (c["kind"], c["n"])
        assert hashlib.sha256(out).hexdigest() == c["out_sha256"], (c["kind"], c["n"])
        rc, back = orc.lz4_decompress(out, c["n"])
        assert rc == c["n"] and back == src


def test_reference_error_cases():
    # LZ4_decompress_safe: empty input, zero capacity (only the 1-byte "0" block decodes)
    assert orc.lz4_decompress(b"", 10)[0] < 0
    assert orc.lz4_decompress(b"\x00", 0)[0] == 0
    assert orc.lz4_decompress(b"\x10a", 0)[0] < 0
    # a block one byte too large for the destination
    c = orc.lz4_compress(bytes(1000))
    assert orc.lz4_decompress(c, 999)[0] < 0
    assert orc.lz4_decompress(c, 1000) == (1000, bytes(1000))


@pytest.mark.skipif(_sys_lz4() is None, reason="system liblz4 not loadable")
def test_against_system_liblz4_random_and_malformed():
    L = _sys_lz4()
    rng = np.random.default_rng(11)
    for trial in range(1500):
        kind = lz4_data.KINDS[trial % len(lz4_data.KINDS)]
        n = int(rng.choice([20, 77, 1000, 5000, 65547, 70000]))
        src = lz4_data.sample(kind, n, seed=trial)
        cap = L.LZ4_compressBound(n)
        dst = ctypes.create_string_buffer(cap)
        r = L.LZ4_compress_default(src, dst, n, cap)
        ref = dst.raw[:r]
        assert orc.lz4_compress(src) == ref
        # corrupt: truncate, flip bits or overwrite a byte; vary the capacity
        c = bytearray(ref)
        m = trial % 4
        if m == 0 and len(c) > 1:
            c = c[:int(rng.integers(0, len(c)))]
        elif m == 1:
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, len(c)))
                c[i] ^= 1 << int(rng.integers(0, 8))
        elif m == 2:
            c[int(rng.integers(0, len(c)))] = int(rng.integers(0, 256))
        ocap = n if rng.random() < 0.7 else int(rng.integers(0, n + 50))
        out = ctypes.create_string_buffer(max(ocap, 1))
        r2 = L.LZ4_decompress_safe(bytes(c), out, len(c), ocap)
        r1, d1 = orc.lz4_decompress(bytes(c), ocap)
        assert (r1 < 0) == (r2 < 0), (trial, kind, n, m, ocap, r1, r2)
        if r1 >= 0:
            assert r1 == r2 and d1 == out.raw[:r2]
