"""CPU build of the engine's Zstandard level-1 encoder (juicefs_amd/csrc/
jfsx_zstdc.h, the source the GPU kernel runs; tests/harness/zstdc_host.cpp)
against the system zstd library: every frame must equal ZSTD_compress(src,
level 1) byte for byte -- the call zstd.CompressLevel makes for the "zstd"
Compressor (pkg/compress/compress.go:82-91).  The system library is 1.4.8;
the reference's DataDog/zstd v1.5.0 is not in the tree (parity with it is
unpinned).  Mixed inputs copy spans from up to 540 KB back, so
matches and repcodes meet the 512 KiB window limit across 128 KiB blocks."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from tests import lz4_data, zstd_lib

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "harness", "libzstdc_host.so")
SIZES = (0, 1, 5, 6, 7, 8, 13, 63, 64, 65, 100, 255, 256, 1000, 1023, 1024, 4096, 16383, 16384, 16385, 65536,
         100003, 131071, 131072, 131073, 262144, 262145, 300000, 1 << 20, 4 << 20)


@pytest.fixture(scope="module")
def enc():
    src = os.path.join(HERE, "harness", "zstdc_host.cpp")
    hdr = os.path.join(HERE, "..", "juicefs_amd", "csrc", "jfsx_zstdc.h")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC", "-o", SO, src])
    h = ctypes.CDLL(SO)
    h.zstdc_host_compress.restype = ctypes.c_int64
    h.zstdc_host_compress.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]
    h.zstdc_host_bound.restype = ctypes.c_uint64

    def f(src):
        cap = h.zstdc_host_bound(len(src))
        out = ctypes.create_string_buffer(max(cap, 1))
        r = h.zstdc_host_compress(bytes(src), len(src), out, cap)
        assert r > 0
        return out.raw[:r]
    return f


def mixed(seed, n):
    """Spans of every kind, and copies from near (< 2 KB) and far (300-540 KB)
    back: block-to-block Huffman reuse, raw / RLE blocks between compressed
    ones, matches and repcodes at the window edge."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < n:
        m = int(rng.integers(1, 60000))
        if rng.random() < 0.3 and len(out) > 1000:
            d = min(len(out), int(rng.choice([rng.integers(1, 2000), rng.integers(300000, 530000),
                                              rng.integers(500000, 540000)])))
            st = len(out) - d
            for k in range(m):
                out.append(out[st + k])
        else:
            out += lz4_data.sample(lz4_data.KINDS[int(rng.integers(0, 6))], m, seed=int(rng.integers(0, 1 << 30)))
    return bytes(out[:n])


def test_bound_matches_library(enc):
    z = zstd_lib.lib()
    h = ctypes.CDLL(SO)
    h.zstdc_host_bound.restype = ctypes.c_uint64
    for n in SIZES + (131071 * 3, 1 << 30):
        assert h.zstdc_host_bound(n) == z.ZSTD_compressBound(ctypes.c_size_t(n))


@pytest.mark.parametrize("kind", lz4_data.KINDS)
def test_frames_equal_libzstd_level1(enc, kind):
    for n in SIZES:
        src = lz4_data.sample(kind, n, seed=n + 1)
        assert enc(src) == zstd_lib.compress_simple(src, 1), (kind, n)


@pytest.mark.parametrize("seed", range(24))
def test_mixed_inputs_equal_libzstd_level1(enc, seed):
    rng = np.random.default_rng(seed + 1000)
    n = int(rng.choice([rng.integers(1, 5000), rng.integers(5000, 300000), rng.integers(300000, 4 << 20)]))
    src = mixed(seed, n)
    assert enc(src) == zstd_lib.compress_simple(src, 1), (seed, n)


def test_round_trip_through_library_decoder(enc):
    for kind in lz4_data.KINDS:
        src = lz4_data.sample(kind, 777777, seed=9)
        rc, back = zstd_lib.decompress(enc(src), len(src))
        assert rc == len(src) and back == src
