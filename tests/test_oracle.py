"""The CPU restatement (oracle/) pinned against published KATs and the
OpenSSL-generated golden vectors (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ALGO = {"aes256gcm": orc.AES256GCM, "chacha20poly1305": orc.CHACHA20P1305}


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


# Published values (McGrew-Viega GCM spec test cases 13-16, RFC 8439 §2.8.2,
# RFC 3720 B.4), written out here independently of the fixture file.
PUBLISHED = {
    "gcm_tc13": ("", "530f8afbc74536b9a963b4f1c4cb738b"),
    "gcm_tc14": ("cea7403d4d606b6e074ec5d3baf39d18", "d0d1c8a799996bf0265b98b5d48ab919"),
    "gcm_tc15": ("522dc1f099567d07f47f37a32a84427d", "b094dac5d93471bdec1a502270e3cc6c"),
    "gcm_tc16": ("522dc1f099567d07f47f37a32a84427d", "76fc6ece0f4e1768cddf8853bb2d551b"),
    "rfc8439_2_8_2": ("d31a8d34648e60db7b86afbc53ef7ec2", "1ae10b594f09e26a7e902ecbd0600691"),
}
CRC_PUBLISHED = {"check_123456789": 0xE3069283, "rfc3720_zeros32": 0x8A9136AA, "rfc3720_ones32": 0x62A8AB43,
                 "rfc3720_inc32": 0x46DD794E, "rfc3720_dec32": 0x113FDB5C, "hello": 0x9A71BB4C}


@pytest.mark.parametrize("kat", _load("kats.json")["aead"], ids=lambda k: k["name"])
def test_aead_kat(kat):
    algo = ALGO[kat["algo"]]
    key, nonce = bytes.fromhex(kat["key"]), bytes.fromhex(kat["nonce"])
    p, aad = bytes.fromhex(kat["p"]), bytes.fromhex(kat["aad"])
    c, tag = orc.seal(algo, key, nonce, p, aad)
    assert c.hex() == kat["c"] and tag.hex() == kat["tag"]
    c16, t = PUBLISHED[kat["name"]]
    assert c.hex()[:32] == c16 and tag.hex() == t
    assert orc.open_(algo, key, nonce, c, tag, aad) == p
    bad = bytearray(tag)
    bad[0] ^= 1
    assert orc.open_(algo, key, nonce, c, bytes(bad), aad) is None


@pytest.mark.parametrize("kat", _load("kats.json")["crc32c"], ids=lambda k: k["name"])
def test_crc_kat(kat):
    d = bytes.fromhex(kat["data"])
    assert orc.crc32c(d) == kat["crc"] == CRC_PUBLISHED[kat["name"]]
    assert orc.crc32c(d, hw=True) == kat["crc"]


def test_poly1305_rfc8439_2_5_2():
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    assert orc.poly1305(key, b"Cryptographic Forum Research Group").hex() == "a8061dc1305136c6c22b8baf0c0127a9"


def test_chacha20_block_rfc8439_2_3_2():
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    out = orc.chacha20_block(key, 1, nonce)
    assert out.hex()[:32] == "10f1e7e4d13b5915500fdd1fa32071c4"


def test_aes_fips197_c3():
    key = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert orc.aes256_encrypt_block(key, pt).hex() == "8ea2b7ca516745bfeafc49904b496089"


@pytest.mark.parametrize("v", _load("aead_vectors.json")["vectors"],
                         ids=lambda v: "%s-%d" % (v["algo"], v["len"]))
def test_golden_vectors(v):
    algo = ALGO[v["algo"]]
    p = orc.gen_block(v["seed"], v["block"], v["len"])
    assert hashlib.sha256(p.tobytes()).hexdigest() == v["p_sha256"]
    key, nonce = orc.gen_key(v["seed"], v["block"])
    assert key.hex() == v["key"] and nonce.hex() == v["nonce"]
    fast = v["len"] > 70000
    c, tag = orc.seal(algo, key, nonce, p, fast=fast)
    assert tag.hex() == v["tag"]
    assert hashlib.sha256(c).hexdigest() == v["c_sha256"]
    if "c" in v:
        assert c.hex() == v["c"]
    assert orc.checksum(p).hex() == v["crc"]
    assert orc.checksum(p, hw=True).hex() == v["crc"]
    if algo == orc.AES256GCM:
        c2, t2 = orc.seal(algo, key, nonce, p, fast=True)
        assert (c2, t2) == (c, tag)
        assert orc.open_(algo, key, nonce, c, tag, fast=True) == p.tobytes()


def test_checksum_len_quirks():
    # disk_cache.go:1221 -- Go's truncating division gives 4 bytes for n=0
    assert orc.checksum(b"") == b"\x00\x00\x00\x00"
    assert len(orc.checksum(bytes(32768))) == 4
    assert len(orc.checksum(bytes(32769))) == 8


def test_object_format_roundtrip():
    key, nonce = orc.gen_key(7, 3)
    wrapped = bytes(range(256))
    for algo in (orc.AES256GCM, orc.CHACHA20P1305):
        obj = orc.data_encrypt(algo, key, nonce, wrapped, b"hello")
        assert obj[:3] == b"\x01\x00\x0c" and obj[3:259] == wrapped and obj[259:271] == nonce
        assert len(obj) == 3 + 256 + 12 + 5 + 16
        assert orc.data_decrypt(algo, key, obj) == b"hello"
        with pytest.raises(ValueError, match="misformed"):
            orc.data_decrypt(algo, key, obj[:271])
        bad = bytearray(obj)
        bad[-1] ^= 0x80
        with pytest.raises(ValueError, match="open failed"):
            orc.data_decrypt(algo, key, bytes(bad))


def test_crc32c_three_stream_matches_serial():
    """orc_crc32c_update_hw3 (three interleaved crc32 streams + GF(2)
    combine, the CPU baseline's checksum()) equals the serial CRC32C."""
    from oracle import oracle as orc
    for n in (0, 1, 7, 767, 768, 769, 5000, 32767, 32768, 32769, 100000, 1 << 20):
        d = orc.gen_block(1, n, n)
        assert orc.crc32c(d, hw=3) == orc.crc32c(d) == orc.crc32c(d, hw=True), n
        assert orc.crc32c(d, 0xDEADBEEF, hw=3) == orc.crc32c(d, 0xDEADBEEF), n


def test_evp_baseline_matches_oracle():
    """The CPU baseline's AEAD (OpenSSL EVP) gives the oracle's bytes, and its
    timed loop the same tag/CRC digest as the port's."""
    import pytest
    from oracle import oracle as orc
    if orc.evp_seal(0, bytes(32), bytes(12), b"x") is None:
        pytest.skip("libcrypto.so.3 not loadable")
    for algo in (orc.AES256GCM, orc.CHACHA20P1305):
        k, nc = orc.gen_key(5, algo)
        for n in (0, 1, 16, 1000, 65537, 1 << 20):
            p = orc.gen_block(5, n, n)
            assert orc.evp_seal(algo, k, nc, p) == orc.seal(algo, k, nc, p), (algo, n)
        s1, d1 = orc.bench_seal_crc(algo, 2, 4, 1 << 20, 9)
        s2, d2 = orc.bench_seal_crc_evp(algo, 2, 4, 1 << 20, 9)
        assert s2 > 0 and d1 == d2
