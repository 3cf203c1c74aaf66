"""The system zstd C library (libzstd.so.1, 1.4.8 here) through ctypes: the
checker for the engine's Zstandard decoder (test data and reference results
only; the reference binds github.com/DataDog/zstd v1.5.0, go.mod:10, whose
vendored C sources are not in /root/reference).  Decoding is defined by the
format (RFC 8878), so frames from this library decode to the same bytes under
any conforming decoder; accept/reject of malformed frames is compared with
this library's ZSTD_decompress."""
import ctypes
import ctypes.util

_z = None


def lib():
    global _z
    if _z is None:
        z = ctypes.CDLL(ctypes.util.find_library("zstd") or "libzstd.so.1")
        z.ZSTD_compressBound.restype = ctypes.c_size_t
        z.ZSTD_decompress.restype = ctypes.c_size_t
        z.ZSTD_isError.restype = ctypes.c_uint
        z.ZSTD_createCCtx.restype = ctypes.c_void_p
        z.ZSTD_compress2.restype = ctypes.c_size_t
        z.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
        z.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
        _z = z
    return _z


def version():
    return lib().ZSTD_versionNumber()


def compress(src, level=1, checksum=False):
    """ZSTD_compress2 at level (ZSTD_c_compressionLevel = 100) with
    ZSTD_c_checksumFlag (201); level 1 without checksum is what
    zstd.CompressLevel(dst, src, 1) of the "zstd" Compressor writes."""
    z = lib()
    cap = z.ZSTD_compressBound(len(src))
    out = ctypes.create_string_buffer(max(cap, 1))
    cc = ctypes.c_void_p(z.ZSTD_createCCtx())
    try:
        z.ZSTD_CCtx_setParameter(cc, 100, int(level))
        z.ZSTD_CCtx_setParameter(cc, 201, 1 if checksum else 0)
        r = z.ZSTD_compress2(cc, out, cap, bytes(src), len(src))
        if z.ZSTD_isError(r):
            raise RuntimeError("ZSTD_compress2 failed")
    finally:
        z.ZSTD_freeCCtx(cc)
    return out.raw[:r]


def compress_simple(src, level=1):
    """ZSTD_compress(dst, bound, src, n, level): the one-shot call
    zstd.CompressLevel (DataDog/zstd, compress.go:82-91) makes -- the bytes
    the engine's level-1 encoder must reproduce."""
    z = lib()
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    cap = z.ZSTD_compressBound(len(src))
    out = ctypes.create_string_buffer(max(cap, 1))
    r = z.ZSTD_compress(out, cap, bytes(src), len(src), int(level))
    if z.ZSTD_isError(r):
        raise RuntimeError("ZSTD_compress failed")
    return out.raw[:r]


def decompress(frame, cap):
    """ZSTD_decompress into cap bytes: (rc, bytes) with rc < 0 on error."""
    z = lib()
    out = ctypes.create_string_buffer(max(cap, 1))
    r = z.ZSTD_decompress(out, cap, bytes(frame), len(frame))
    if z.ZSTD_isError(r):
        return -1, b""
    return r, out.raw[:r]


def skippable(payload, nibble=0):
    """A skippable frame (magic 0x184D2A50 + nibble) carrying payload."""
    return (0x184D2A50 + nibble).to_bytes(4, "little") + len(payload).to_bytes(4, "little") + bytes(payload)


def huf12_frame(syms, four):
    """A frame whose only block holds Huffman-coded literals (no sequences)
    under a log-12 table: weights 11, 11, 11, 10, ..., 1 for symbols 0..12
    and an implied 1 for symbol 13 (codes of 2 to 12 bits).  libzstd's
    encoder never writes log 12; its decoder takes it (HUF_TABLELOG_MAX 12).
    syms: values 0..13, 4..255 of them; four: four streams (else one)."""
    w = [11, 11, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 1]
    code, start = {}, 0
    for wv in range(1, 12):  # X1 layout: by weight, then symbol
        for s, ws in enumerate(w):
            if ws == wv:
                nb = 13 - wv
                code[s] = format(start >> (12 - nb), "0%db" % nb)
                start += 1 << (wv - 1)
    assert start == 4096

    def stream(part):
        bits = "".join(code[s] for s in part)
        v = (1 << len(bits)) | (int(bits, 2) if bits else 0)
        return v.to_bytes((len(bits) + 8) // 8, "little")

    n = len(syms)
    ew = w[:-1] + [0]
    tree = bytes([127 + 13]) + bytes((ew[k] << 4) | ew[k + 1] for k in range(0, 14, 2))
    if four:
        seg = (n + 3) // 4
        parts = [stream(syms[k * seg:(k + 1) * seg]) for k in range(3)] + [stream(syms[3 * seg:])]
        body = b"".join(len(p).to_bytes(2, "little") for p in parts[:3]) + b"".join(parts)
    else:
        body = stream(syms)
    litc = len(tree) + len(body)
    lh = 2 | ((1 if four else 0) << 2) | (n << 4) | (litc << 14)
    block = lh.to_bytes(3, "little") + tree + body + b"\x00"
    bh = (len(block) << 3) | (2 << 1) | 1
    return b"\x28\xb5\x2f\xfd" + bytes([0x20, n]) + bh.to_bytes(3, "little") + block
