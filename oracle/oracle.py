"""ctypes wrapper over oracle/_build/libjfs_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product package (juicefs_amd/) never imports
this module.  See jfs_oracle.c for the reference file:line each function
restates.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libjfs_oracle.so")
_lib = None

AES256GCM = 0
CHACHA20P1305 = 1
CS_NONE, CS_FULL, CS_SHRINK, CS_EXTEND = 0, 1, 2, 3
LEVELS = {"none": CS_NONE, "full": CS_FULL, "shrink": CS_SHRINK, "extend": CS_EXTEND}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, U64, I64, U32, I = (ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
                               ctypes.c_uint32, ctypes.c_int)
        sig = {
            "orc_gen_block": (None, [U64, U64, P, U64]),
            "orc_gen_key": (None, [U64, U64, P, P]),
            "orc_crc32c_update": (U32, [U32, P, U64]),
            "orc_crc32c_update_hw": (U32, [U32, P, U64]),
            "orc_crc32c_update_hw3": (U32, [U32, P, U64]),
            "orc_evp_seal": (I, [I, P, P, P, U64, P, P]),
            "orc_bench_seal_crc_evp": (ctypes.c_double, [I, I, U64, U64, U64, P]),
            "orc_checksum_len": (I64, [I64]),
            "orc_checksum": (I64, [P, I64, P, I]),
            "orc_open_cache_file": (I, [I64, I64, I]),
            "orc_cache_readat": (I, [P, I64, I64, I, I64, I64, P, P, P, P, P]),
            "orc_aes256_expand": (None, [P, P]),
            "orc_aes256_encrypt_block": (None, [P, P, P]),
            "orc_sbox": (None, [P]),
            "orc_gf128_mul": (None, [P, P, P]),
            "orc_aes256gcm_seal": (None, [P, P, P, U64, P, U64, P, P]),
            "orc_aes256gcm_open": (I, [P, P, P, U64, P, U64, P, P]),
            "orc_aes256gcm_seal_ni": (None, [P, P, P, U64, P, P]),
            "orc_aes256gcm_open_ni": (I, [P, P, P, U64, P, P]),
            "orc_chacha20_block": (None, [P, U32, P, P]),
            "orc_poly1305": (None, [P, P, U64, P]),
            "orc_chacha20poly1305_seal": (None, [P, P, P, U64, P, U64, P, P]),
            "orc_chacha20poly1305_open": (I, [P, P, P, U64, P, U64, P, P]),
            "orc_data_encrypt": (I64, [I, P, P, P, I, P, U64, P]),
            "orc_data_decrypt": (I64, [I, P, P, I64, P]),
            "orc_bench_seal_crc": (ctypes.c_double, [I, I, U64, U64, U64, P]),
            "orc_bench_baseline": (ctypes.c_double, [I, I, I, U64, P, U64, U64, P]),
            "orc_bench_readat": (ctypes.c_double, [I, I, U64, P, U64, U64, P, P, P, U64, P]),
            "orc_cache_readat_hw": (I, [P, I64, I64, I, I64, I64, P, P, P, P, P]),
            "orc_expect_batch": (ctypes.c_double, [I, I, U64, P, U64, U64, U64, P, P, U64]),
            "orc_lz4_bound": (I, [I]),
            "orc_lz4_compress": (I, [P, I, P, I]),
            "orc_lz4_decompress": (I, [P, I, P, I]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _buf(b):
    """Read-only pointer to bytes-like data (kept alive by the caller)."""
    if isinstance(b, np.ndarray):
        return b.ctypes.data
    if isinstance(b, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(b)), ctypes.c_void_p).value if isinstance(b, bytes) \
            else ctypes.addressof((ctypes.c_char * len(b)).from_buffer(b))
    raise TypeError(type(b))


def _np(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy() if not isinstance(b, np.ndarray) else b


def gen_block(seed, b, length):
    out = np.empty(max(length, 1), dtype=np.uint8)
    lib().orc_gen_block(seed, b, out.ctypes.data, length)
    return out[:length]


def gen_key(seed, b):
    k = np.empty(32, np.uint8)
    n = np.empty(12, np.uint8)
    lib().orc_gen_key(seed, b, k.ctypes.data, n.ctypes.data)
    return k.tobytes(), n.tobytes()


def crc32c(data, crc=0, hw=False):
    d = _np(data)
    f = {False: lib().orc_crc32c_update, True: lib().orc_crc32c_update_hw, 3: lib().orc_crc32c_update_hw3}[hw]
    return f(crc, d.ctypes.data if d.size else None, d.size)


def checksum(data, hw=False):
    d = _np(data)
    n = d.size
    out = np.empty(lib().orc_checksum_len(n), np.uint8)
    lib().orc_checksum(d.ctypes.data if n else None, n, out.ctypes.data, 1 if hw else 0)
    return out.tobytes()


def object_checksum(obj, hw=False):
    """generateChecksum (pkg/object/checksum.go:31-53): crc32.Update(0,
    Castagnoli, whole stored object) as a decimal string."""
    return str(crc32c(obj, 0, hw))


def open_cache_file(file_size, length, level):
    return lib().orc_open_cache_file(file_size, length, LEVELS.get(level, level))


def cache_readat(file_img, length, level, off, size):
    """Returns (rc, data, n, got, expect, bad_seg); rc 0 ok, 1 checksum, 2 eof."""
    f = _np(file_img)
    eff = open_cache_file(f.size, length, level)
    if eff < 0:
        raise ValueError("invalid file size %d, data length %d" % (f.size, length))
    out = np.zeros(max(size, 1), np.uint8)
    n = ctypes.c_int64()
    got = ctypes.c_uint32()
    exp = ctypes.c_uint32()
    seg = ctypes.c_int64(-1)
    rc = lib().orc_cache_readat(f.ctypes.data, f.size, length, eff, off, size, out.ctypes.data,
                                ctypes.byref(n), ctypes.byref(got), ctypes.byref(exp), ctypes.byref(seg))
    return rc, out[:size].tobytes(), n.value, got.value, exp.value, seg.value


def _aead(algo, fast=False):
    L = lib()
    if algo == AES256GCM:
        return L.orc_aes256gcm_seal, L.orc_aes256gcm_open
    return L.orc_chacha20poly1305_seal, L.orc_chacha20poly1305_open


def seal(algo, key, nonce, plaintext, aad=b"", fast=False):
    p = _np(plaintext)
    c = np.empty(max(p.size, 1), np.uint8)
    tag = np.empty(16, np.uint8)
    if fast and algo == AES256GCM and not aad:
        lib().orc_aes256gcm_seal_ni(key, nonce, p.ctypes.data, p.size, c.ctypes.data, tag.ctypes.data)
    else:
        a = _np(aad)
        _aead(algo)[0](key, nonce, a.ctypes.data if a.size else None, a.size, p.ctypes.data, p.size,
                       c.ctypes.data, tag.ctypes.data)
    return c[:p.size].tobytes(), tag.tobytes()


def open_(algo, key, nonce, ciphertext, tag, aad=b"", fast=False):
    c = _np(ciphertext)
    p = np.empty(max(c.size, 1), np.uint8)
    if fast and algo == AES256GCM and not aad:
        rc = lib().orc_aes256gcm_open_ni(key, nonce, c.ctypes.data, c.size, tag, p.ctypes.data)
    else:
        a = _np(aad)
        rc = _aead(algo)[1](key, nonce, a.ctypes.data if a.size else None, a.size, c.ctypes.data, c.size,
                            tag, p.ctypes.data)
    return None if rc else p[:c.size].tobytes()


def aes256_encrypt_block(key, block):
    rk = np.empty(240, np.uint8)
    out = np.empty(16, np.uint8)
    lib().orc_aes256_expand(key, rk.ctypes.data)
    lib().orc_aes256_encrypt_block(rk.ctypes.data, block, out.ctypes.data)
    return out.tobytes()


def aes256_expand(key):
    rk = np.empty(240, np.uint8)
    lib().orc_aes256_expand(key, rk.ctypes.data)
    return rk.tobytes()


def sbox():
    out = np.empty(256, np.uint8)
    lib().orc_sbox(out.ctypes.data)
    return out


def gf128_mul(x, y):
    out = np.empty(16, np.uint8)
    lib().orc_gf128_mul(x, y, out.ctypes.data)
    return out.tobytes()


def chacha20_block(key, counter, nonce):
    out = np.empty(64, np.uint8)
    lib().orc_chacha20_block(key, counter, nonce, out.ctypes.data)
    return out.tobytes()


def poly1305(key, msg):
    m = _np(msg)
    out = np.empty(16, np.uint8)
    lib().orc_poly1305(key, m.ctypes.data if m.size else None, m.size, out.ctypes.data)
    return out.tobytes()


def data_encrypt(algo, key, nonce, wrapped, plaintext):
    p = _np(plaintext)
    out = np.empty(3 + len(wrapped) + 12 + p.size + 16, np.uint8)
    n = lib().orc_data_encrypt(algo, key, nonce, wrapped, len(wrapped), p.ctypes.data if p.size else None,
                               p.size, out.ctypes.data)
    return out[:n].tobytes()


def data_decrypt(algo, key, obj):
    o = _np(obj)
    out = np.empty(max(o.size, 1), np.uint8)
    n = lib().orc_data_decrypt(algo, key, o.ctypes.data, o.size, out.ctypes.data)
    if n == -1:
        raise ValueError("misformed ciphertext")
    if n < 0:
        raise ValueError("open failed")
    return out[:n].tobytes()


def bench_seal_crc(algo, nthreads, nblocks, blen, seed):
    dg = ctypes.c_uint32()
    secs = lib().orc_bench_seal_crc(algo, nthreads, nblocks, blen, seed, ctypes.byref(dg))
    return secs, dg.value


def evp_seal(algo, key, nonce, plaintext):
    """OpenSSL EVP Seal (the CPU baseline's AEAD); None if libcrypto is absent."""
    p = _np(plaintext)
    c = np.empty(max(p.size, 1), np.uint8)
    tag = np.empty(16, np.uint8)
    if lib().orc_evp_seal(algo, key, nonce, p.ctypes.data, p.size, c.ctypes.data, tag.ctypes.data):
        return None
    return c[:p.size].tobytes(), tag.tobytes()


def bench_seal_crc_evp(algo, nthreads, nblocks, blen, seed):
    """(seconds, digest), seconds < 0 if libcrypto is absent."""
    dg = ctypes.c_uint32()
    secs = lib().orc_bench_seal_crc_evp(algo, nthreads, nblocks, blen, seed, ctypes.byref(dg))
    return secs, dg.value


BASE_SEAL, BASE_OPEN, BASE_CRC, BASE_ENCRYPT, BASE_DECRYPT = 0, 1, 2, 3, 4


def bench_baseline(algo, mode, nthreads, nblocks, blen, seed, lens=None):
    """(seconds, digest) of the CPU baseline for mode BASE_SEAL (checksum +
    EVP Seal), BASE_OPEN (EVP Open + CRC verify against the stored CRCs) or
    BASE_CRC (CRC verify only) over nblocks synthetic blocks of blen bytes
    (or lens[b]); seconds -1 without libcrypto, -2 if a block failed."""
    dg = ctypes.c_uint32()
    ln = np.asarray(lens, np.uint64) if lens is not None else None
    secs = lib().orc_bench_baseline(algo, mode, nthreads, nblocks, ln.ctypes.data if ln is not None else None, blen,
                                    seed, ctypes.byref(dg))
    return secs, dg.value


def bench_readat(nthreads, level, lens, seed, reads, reps):
    """(seconds, bytes returned) of cacheFile.ReadAt (3-stream SSE4.2 CRC) on
    nthreads threads: cache-file images of the synthetic blocks 0..n-1 of
    lens[b] bytes, reads = [(block, off, size)], each run reps times."""
    ln = np.asarray(lens, np.uint64)
    blk = np.asarray([r[0] for r in reads], np.uint32)
    off = np.asarray([r[1] for r in reads], np.uint64)
    size = np.asarray([r[2] for r in reads], np.uint64)
    nbytes = ctypes.c_uint64()
    secs = lib().orc_bench_readat(nthreads, level, ln.size, ln.ctypes.data, seed, len(reads), blk.ctypes.data,
                                  off.ctypes.data, size.ctypes.data, reps, ctypes.byref(nbytes))
    return secs, nbytes.value


def expect_batch(algo, nthreads, lens, seed, block0, crcstride):
    """The oracle's Seal tags (n x 16 B) and checksum() arrays (n x crcstride
    B, big-endian CRCs, zero-padded) of the synthetic blocks block0 + i of
    lens[i] bytes: the full check of a bench batch.  (tags, crcs, seconds)."""
    ln = np.asarray(lens, np.uint64)
    n = ln.size
    tags = np.zeros((n, 16), np.uint8)
    crcs = np.zeros((n, crcstride), np.uint8)
    secs = lib().orc_expect_batch(algo, nthreads, n, ln.ctypes.data, int(ln.max()) if n else 0, seed, block0,
                                  tags.ctypes.data, crcs.ctypes.data, crcstride)
    if secs < 0:
        raise ValueError("expect_batch: crcstride %d too small" % crcstride)
    return tags, crcs, secs


# -- LZ4 block codec (oracle/jfs_lz4.c; compress.go:107-125) ------------------
def lz4_bound(n):
    return lib().orc_lz4_bound(n)


def lz4_compress(data):
    """LZ4_compress_default(data) as bytes."""
    src = _np(data)
    cap = lz4_bound(src.size)
    dst = np.empty(max(cap, 1), np.uint8)
    r = lib().orc_lz4_compress(src.ctypes.data, src.size, dst.ctypes.data, cap)
    assert r > 0
    return dst[:r].tobytes()


def lz4_decompress(data, cap):
    """LZ4_decompress_safe(data, cap): (rc, bytes); rc < 0 for a malformed block."""
    src = _np(data)
    dst = np.empty(max(cap, 1), np.uint8)
    r = lib().orc_lz4_decompress(src.ctypes.data if src.size else None, src.size, dst.ctypes.data, cap)
    return r, (dst[:r].tobytes() if r > 0 else b"")
