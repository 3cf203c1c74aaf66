"""Generate tests/golden/*.json -- independent golden vectors for the hot path.

Run here (in the build container), never on the GPU box:
    python tests/golden/make_golden.py

Sources of truth (none of them is this repo's oracle or kernels):
  * AEAD outputs come from OpenSSL 3 libcrypto (EVP aes-256-gcm and
    chacha20-poly1305), driven through ctypes.  OpenSSL implements the same
    NIST SP 800-38D / RFC 8439 constructions Go's crypto/cipher and
    golang.org/x/crypto v0.19.0 implement; the reference itself cannot run
    here (no Go toolchain, see DESIGN.md "Oracle").
  * CRC32C arrays come from a pure-Python bitwise CRC32C (reflected
    0x82F63B78), packed big-endian per 32 KiB segment exactly as
    checksum() does (pkg/chunk/disk_cache.go:1218-1231).
  * Plaintexts are the repo's synthetic SplitMix64 stream, restated here in
    pure Python so the fixture also pins the generator (sha256 of P kept).

Lengths follow SURVEY.md §8c.  Full byte strings are stored only for short
inputs; long ones are stored as sha256 digests.
"""
import ctypes
import ctypes.util
import hashlib
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def gen_block(seed, b, length):
    nw = (length + 7) // 8
    out = bytearray()
    for k in range(nw):
        out += struct.pack("<Q", mix64(seed + GOLDEN * ((b << 40) + k + 1)))
    return bytes(out[:length])


def gen_key(seed, b):
    key = b"".join(struct.pack("<Q", mix64((seed ^ 0x4B4559) + GOLDEN * ((b << 8) + i + 1))) for i in range(4))
    w0 = mix64((seed ^ 0x4E4F4E4345) + GOLDEN * ((b << 8) + 1))
    w1 = mix64((seed ^ 0x4E4F4E4345) + GOLDEN * ((b << 8) + 2))
    return key, struct.pack("<Q", w0) + struct.pack("<Q", w1)[:4]


_CRC_T = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_T.append(_c)


def crc32c(data, crc=0):
    crc ^= 0xFFFFFFFF
    t = _CRC_T
    for x in data:
        crc = t[(crc ^ x) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def checksum(data):
    n = len(data)
    out = bytearray(((n - 1) // 32768 + 1) * 4 if n else 4)
    off = 0
    for s in range(0, n, 32768):
        out[off:off + 4] = struct.pack(">I", crc32c(data[s:s + 32768]))
        off += 4
    return bytes(out)


class OpenSSL:
    def __init__(self):
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.EVP_CIPHER_CTX_new.restype = P
        L.EVP_aes_256_gcm.restype = P
        L.EVP_chacha20_poly1305.restype = P
        L.EVP_EncryptInit_ex.argtypes = [P, P, P, P, P]
        L.EVP_DecryptInit_ex.argtypes = [P, P, P, P, P]
        L.EVP_EncryptUpdate.argtypes = [P, P, P, P, ctypes.c_int]
        L.EVP_DecryptUpdate.argtypes = [P, P, P, P, ctypes.c_int]
        L.EVP_EncryptFinal_ex.argtypes = [P, P, P]
        L.EVP_DecryptFinal_ex.argtypes = [P, P, P]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        L.EVP_CIPHER_CTX_free.argtypes = [P]
        self.L = L

    def seal(self, algo, key, nonce, pt, aad=b""):
        L = self.L
        ctx = L.EVP_CIPHER_CTX_new()
        cipher = L.EVP_aes_256_gcm() if algo == "aes256gcm" else L.EVP_chacha20_poly1305()
        assert L.EVP_EncryptInit_ex(ctx, cipher, None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, 0x9, len(nonce), None) == 1
        assert L.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
        outl = ctypes.c_int()
        if aad:
            assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(outl), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 32)
        total = 0
        if pt:
            assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), pt, len(pt)) == 1
            total = outl.value
        assert L.EVP_EncryptFinal_ex(ctx, ctypes.byref(out, total), ctypes.byref(outl)) == 1
        total += outl.value
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag) == 1
        L.EVP_CIPHER_CTX_free(ctx)
        return out.raw[:total], tag.raw


LENGTHS = [0, 1, 15, 16, 17, 63, 64, 65, 1000, 1024, 1025, 4095, 16384, 32767, 32768, 32769, 65536,
           98304 + 5, 102400, 1 << 20, (4 << 20) - 1, 4 << 20]
SEED = 0x4A465321


def main():
    ssl = OpenSSL()
    vectors = []
    for algo in ("aes256gcm", "chacha20poly1305"):
        for i, n in enumerate(LENGTHS):
            b = i + (0 if algo == "aes256gcm" else 100)
            key, nonce = gen_key(SEED, b)
            p = gen_block(SEED, b, n)
            c, tag = ssl.seal(algo, key, nonce, p)
            v = {"algo": algo, "seed": SEED, "block": b, "len": n, "key": key.hex(), "nonce": nonce.hex(),
                 "p_sha256": hashlib.sha256(p).hexdigest(), "c_sha256": hashlib.sha256(c).hexdigest(),
                 "tag": tag.hex(), "crc": checksum(p).hex()}
            if n <= 4096:
                v["c"] = c.hex()
            vectors.append(v)
            print(algo, n, tag.hex())
    with open(os.path.join(HERE, "aead_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (OpenSSL EVP + pure-Python CRC32C)",
                   "vectors": vectors}, f, indent=1)

    # published KATs, re-checked against OpenSSL here before they are committed
    kats = []
    z32 = bytes(32)
    for name, key, iv, pt, aad in [
        ("gcm_tc13", z32, bytes(12), b"", b""),
        ("gcm_tc14", z32, bytes(12), bytes(16), b""),
        ("gcm_tc15", bytes.fromhex("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308"),
         bytes.fromhex("cafebabefacedbaddecaf888"),
         bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e24"
                       "49a6b525b16aedf5aa0de657ba637b391aafd255"), b""),
        ("gcm_tc16", bytes.fromhex("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308"),
         bytes.fromhex("cafebabefacedbaddecaf888"),
         bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e24"
                       "49a6b525b16aedf5aa0de657ba637b39"),
         bytes.fromhex("feedfacedeadbeeffeedfacedeadbeefabaddad2")),
    ]:
        c, t = ssl.seal("aes256gcm", key, iv, pt, aad)
        kats.append({"name": name, "algo": "aes256gcm", "key": key.hex(), "nonce": iv.hex(), "p": pt.hex(),
                     "aad": aad.hex(), "c": c.hex(), "tag": t.hex()})
    rfc_key = bytes(range(0x80, 0xa0))
    rfc_nonce = bytes.fromhex("070000004041424344454647")
    rfc_aad = bytes.fromhex("50515253c0c1c2c3c4c5c6c7")
    rfc_pt = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, "
              b"sunscreen would be it.")
    c, t = ssl.seal("chacha20poly1305", rfc_key, rfc_nonce, rfc_pt, rfc_aad)
    kats.append({"name": "rfc8439_2_8_2", "algo": "chacha20poly1305", "key": rfc_key.hex(),
                 "nonce": rfc_nonce.hex(), "p": rfc_pt.hex(), "aad": rfc_aad.hex(), "c": c.hex(), "tag": t.hex()})
    crc_kats = [
        {"name": "check_123456789", "data": b"123456789".hex(), "crc": crc32c(b"123456789")},
        {"name": "rfc3720_zeros32", "data": bytes(32).hex(), "crc": crc32c(bytes(32))},
        {"name": "rfc3720_ones32", "data": (b"\xff" * 32).hex(), "crc": crc32c(b"\xff" * 32)},
        {"name": "rfc3720_inc32", "data": bytes(range(32)).hex(), "crc": crc32c(bytes(range(32)))},
        {"name": "rfc3720_dec32", "data": bytes(range(31, -1, -1)).hex(), "crc": crc32c(bytes(range(31, -1, -1)))},
        {"name": "hello", "data": b"hello".hex(), "crc": crc32c(b"hello")},
    ]
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump({"aead": kats, "crc32c": crc_kats}, f, indent=1)
    for k in kats:
        print(k["name"], k["c"][:32], k["tag"])
    for k in crc_kats:
        print(k["name"], hex(k["crc"]))


if __name__ == "__main__":
    main()
