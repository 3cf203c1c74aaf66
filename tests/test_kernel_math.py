"""CPU emulation of the kernels' decompositions, using the product's own
host-built tables (jfsx_debug_tables), checked against the oracle.

This pins the arithmetic the HIP kernels implement (lane-strided CRC32C with
shift-combine, lane-strided GHASH Horner with H^64 and exponent lifting,
AES T0/T2 tables) before any GPU run; the GPU parity tests then pin the
kernels themselves."""
import numpy as np
import pytest

from juicefs_amd import engine
from oracle import oracle as orc

POLY = 0x82F63B78


@pytest.fixture(scope="module")
def tables():
    return engine.debug_tables()


def mulmod(a, b):
    p = 0
    for _ in range(32):
        if a & 0x80000000:
            p ^= b
        a = (a << 1) & 0xFFFFFFFF
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def xpow8(n, x8):
    r = 0x80000000
    k = 0
    while n:
        if n & 1:
            r = mulmod(int(x8[k]), r)
        n >>= 1
        k += 1
    return r


def test_aes_tables_match_sbox(tables):
    aes = tables[0]
    sb = orc.sbox()
    for x in range(256):
        t0 = int(aes[x * 64])
        assert (t0 >> 8) & 0xFF == sb[x]
        assert all(int(v) == t0 for v in aes[x * 64:x * 64 + 32])
        assert int(aes[x * 64 + 32]) == ((t0 << 16) | (t0 >> 16)) & 0xFFFFFFFF


def emulate_segment_crc(seg, tables):
    _, crc, crcx = tables
    T = lambda t, v: int(crc[t * 256 + v])
    L = len(seg)
    A = [0] * 64
    lend = [0] * 64

    def piece(a, p):
        s = T(16, a & 255) ^ T(17, (a >> 8) & 255) ^ T(18, (a >> 16) & 255) ^ T(19, a >> 24)
        q = bytearray(p)
        q[0] ^= s & 255
        q[1] ^= (s >> 8) & 255
        q[2] ^= (s >> 16) & 255
        q[3] ^= s >> 24
        r = 0
        for j in range(16):
            r ^= T(j, q[j])
        return r

    def partial(a, p):
        c = T(16, a & 255) ^ T(17, (a >> 8) & 255) ^ T(18, (a >> 16) & 255) ^ T(19, a >> 24)
        for byte in p:
            c = T(15, (c ^ byte) & 255) ^ (c >> 8)
        return c

    for r in range((L + 1023) // 1024):
        for lane in range(64):
            o = 1024 * r + 16 * lane
            if o + 16 <= L:
                A[lane] = piece(A[lane], seg[o:o + 16])
                lend[lane] = o + 16
            elif o < L:
                A[lane] = partial(A[lane], seg[o:L])
                lend[lane] = L
    raw = 0
    for lane in range(64):
        x = int(crcx[lane]) if L == 32768 else xpow8(L - lend[lane], crcx[64:96])
        raw ^= mulmod(x, A[lane])
    K = int(crcx[96]) if L == 32768 else mulmod(xpow8(L, crcx[64:96]), 0xFFFFFFFF)
    return (~(K ^ raw)) & 0xFFFFFFFF


def emulate_full_segment_nibble(seg, tables):
    """crc_segments_k's full-segment path: A' = S1024(A) ^ U(piece), every
    byte lookup split into its low- and high-nibble halves (the tables are
    linear, so T[b] = T[b & 15] ^ T[b & 240])."""
    _, crc, crcx = tables
    T = lambda t, v: int(crc[t * 256 + (v & 15)]) ^ int(crc[t * 256 + (v & 240)])
    A = [0] * 64
    for r in range(32):
        for lane in range(64):
            o = 1024 * r + 16 * lane
            a = A[lane]
            v = 0
            for k in range(4):
                v ^= T(24 + k, (a >> (8 * k)) & 255)
            for j in range(16):
                v ^= T(j, seg[o + j])
            A[lane] = v
    raw = 0
    for lane in range(64):
        raw ^= mulmod(int(crcx[lane]), A[lane])
    return (~(int(crcx[96]) ^ raw)) & 0xFFFFFFFF


def test_nibble_row_shift_crc_matches_crc32c(tables):
    seg = orc.gen_block(7, 32768, 32768).tobytes()
    assert emulate_full_segment_nibble(seg, tables) == orc.crc32c(seg)


@pytest.mark.parametrize("L", [1, 15, 16, 17, 1000, 1024, 1025, 4111, 31999, 32767, 32768])
def test_lane_strided_crc_matches_crc32c(L, tables):
    seg = orc.gen_block(99, L, L).tobytes()
    assert emulate_segment_crc(seg, tables) == orc.crc32c(seg)


def _gmul(x, y):
    return orc.gf128_mul(x, y)


def _xor(a, b):
    return bytes(p ^ q for p, q in zip(a, b))


def _hpow(H, e):
    r = bytes([0x80]) + bytes(15)  # 1
    for _ in range(e):
        r = _gmul(r, H)
    return r


@pytest.mark.parametrize("nbytes,wave_bytes", [(5000, 32768), (70000, 32768), (100000, 65536), (16, 32768),
                                               (1, 32768), (131072, 32768)])
def test_lane_strided_ghash_matches_gcm(nbytes, wave_bytes):
    key, nonce = orc.gen_key(5, nbytes)
    p = orc.gen_block(5, nbytes, nbytes).tobytes()
    c, tag = orc.seal(orc.AES256GCM, key, nonce, p)
    H = orc.aes256_encrypt_block(key, bytes(16))
    EJ0 = orc.aes256_encrypt_block(key, nonce + b"\x00\x00\x00\x01")
    Y = _hpow(H, 64)
    n = (nbytes + 15) // 16
    cpad = c + bytes(16 * n - nbytes)
    S = bytes(16)
    for w0 in range(0, nbytes, wave_bytes):  # one "wave" per sub-chunk
        w1 = min(w0 + wave_bytes, nbytes)
        wend = (w1 + 15) // 16
        zsum = bytes(16)
        for lane in range(64):
            acc = bytes(16)
            jlast = None
            for row in range(w0, w1, 1024):
                o = row + 16 * lane
                if o >= w1:
                    continue
                j = o // 16
                acc = _xor(_gmul(acc, Y), cpad[16 * j:16 * j + 16])
                jlast = j
            if jlast is None:
                continue
            e = wend + 1 - jlast
            assert 2 <= e <= 65
            zsum = _xor(zsum, _gmul(acc, _hpow(H, e)))
        S = _xor(S, _gmul(zsum, _hpow(H, n - wend)))
    L = bytes(8) + (8 * nbytes).to_bytes(8, "big")
    init = _xor(EJ0, _gmul(L, H))
    assert _xor(init, S) == tag


def xpow8_fast(n, crcx):
    """crc_xpow8_fast (jfsx_internal.h): whole rows, 16-byte steps, then squares."""
    k, j, r = n >> 10, (n >> 4) & 63, n & 15
    v = int(crcx[96 + k]) if k else 0x80000000
    if j:
        v = mulmod(v, int(crcx[63 - j])) if k else int(crcx[63 - j])
    for b in range(4):
        if (r >> b) & 1:
            v = mulmod(v, int(crcx[64 + b]))
    return v


def test_fast_shift_powers_match_squares(tables):
    """The row-shift table crcx[97..127] and the three-step x^(8n) agree with
    the square-and-multiply powers for every distance a segment can need."""
    _, _, crcx = tables
    x8 = crcx[64:96]
    for k in range(1, 32):
        assert int(crcx[96 + k]) == xpow8(1024 * k, x8), k
    rng = np.random.default_rng(3)
    for n in [0, 1, 15, 16, 17, 1008, 1023, 1024, 1025, 32767, 31 * 1024, 31 * 1024 + 1008] + \
            [int(x) for x in rng.integers(0, 32768, 300)]:
        assert xpow8_fast(n, crcx) == xpow8(n, x8), n
