"""CPU build of the engine's Zstandard decoder (juicefs_amd/csrc/jfsx_zstd.h,
the source the GPU kernel runs; tests/harness/zstd_host.cpp) against the
system zstd library: frames at several levels, with and without checksums,
concatenated and skippable frames decode to the original bytes, and a
seeded corpus of truncated / bit-flipped / overwritten frames is accepted or
rejected exactly as ZSTD_decompress does."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from tests import lz4_data, zstd_lib

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "harness", "libzstd_host.so")


@pytest.fixture(scope="module")
def host():
    src = os.path.join(HERE, "harness", "zstd_host.cpp")
    hdr = os.path.join(HERE, "..", "juicefs_amd", "csrc", "jfsx_zstd.h")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC", "-o", SO, src])
    h = ctypes.CDLL(SO)
    h.zstd_host_decompress.restype = ctypes.c_int64
    h.zstd_host_decompress.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]

    def dec(frame, cap):
        out = ctypes.create_string_buffer(max(cap, 1))
        r = h.zstd_host_decompress(bytes(frame), len(frame), out, cap)
        return (r, out.raw[:r]) if r >= 0 else (-1, b"")
    return dec


@pytest.mark.parametrize("kind", lz4_data.KINDS)
def test_round_trip_levels(host, kind):
    for n in (0, 1, 5, 100, 4096, 65536, 100003, 1 << 20, 4 << 20):
        for level in (1, 3, -3, 9):
            for ck in (False, True):
                src = lz4_data.sample(kind, n, seed=n + level + 10)
                fr = zstd_lib.compress(src, level, ck)
                assert host(fr, n) == (n, src), (kind, n, level, ck)


def test_concatenated_and_skippable(host):
    a = lz4_data.sample("text", 70000, seed=1)
    b = lz4_data.sample("runs", 5000, seed=2)
    fr = zstd_lib.skippable(b"juicefs") + zstd_lib.compress(a) + zstd_lib.skippable(b"", 15) + \
        zstd_lib.compress(b, 3, True)
    assert host(fr, len(a) + len(b)) == (len(a) + len(b), a + b)
    assert zstd_lib.decompress(fr, len(a) + len(b))[0] == len(a) + len(b)
    # the edge cases ZSTD_decompress defines: empty input decodes to nothing;
    # a tail of 1..4 bytes, a short skippable header, a wrong magic are errors
    assert host(b"", 10) == (0, b"")
    for bad in (fr + b"\x28\xb5", zstd_lib.skippable(b"x")[:6], b"\x00\x01\x02\x03\x04\x05\x06\x07\x08\x09"):
        assert host(bad, 10**6)[0] < 0 and zstd_lib.decompress(bad, 10**6)[0] < 0
    # output one byte short
    assert host(zstd_lib.compress(a), len(a) - 1)[0] < 0


def test_malformed_agrees_with_library(host):
    rng = np.random.default_rng(1)
    rejects = 0
    for trial in range(3000):
        kind = lz4_data.KINDS[trial % 6]
        n = int(rng.choice([50, 700, 5000, 70000, 300000]))
        fr = bytearray(zstd_lib.compress(lz4_data.sample(kind, n, seed=trial), int(rng.choice([1, 3, -1, 5])),
                                         trial % 3 == 0))
        m = trial % 4
        if m == 0 and len(fr) > 1:
            fr = fr[:int(rng.integers(0, len(fr)))]
        elif m == 1:
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, len(fr)))
                fr[i] ^= 1 << int(rng.integers(0, 8))
        elif m == 2:
            fr[int(rng.integers(0, len(fr)))] = int(rng.integers(0, 256))
        else:
            i = int(rng.integers(0, len(fr)))
            fr[i:i + 2] = bytes(rng.integers(0, 256, 2, dtype=np.uint8))
        cap = n if rng.random() < 0.8 else int(rng.integers(0, n + 10))
        got, ref = host(bytes(fr), cap), zstd_lib.decompress(bytes(fr), cap)
        if ref[0] < 0:
            rejects += 1
            assert got[0] < 0, (trial, kind, n, m, cap)
        else:
            assert got == ref, (trial, kind, n, m, cap)
    assert rejects > 1000


def test_log12_huffman_table(host):
    """Literals under a log-12 Huffman table: the decoder keeps tables up to
    log 11 in LDS and reads log-12 ones from global scratch."""
    rng = np.random.default_rng(12)
    for four in (False, True):
        for n in (4, 37, 200, 255):
            syms = [int(x) for x in rng.integers(0, 14, n)]
            fr = zstd_lib.huf12_frame(syms, four)
            want = zstd_lib.decompress(fr, 1000)
            assert want == (n, bytes(syms)), (four, n, want[0])
            assert host(fr, 1000) == want
