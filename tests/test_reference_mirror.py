"""Reference-interface behaviour that needs no GPU: the TestChecksum level
matrix on the oracle's restatement of cacheFile.ReadAt, RSA-OAEP key wrapping
(encrypt_test.go:96-139 analogue), algorithm dispatch errors."""
import pytest

from oracle import oracle as orc
from tests import checksum_matrix as M


def test_checksum_level_matrix_on_oracle():
    def read(img, length, level, off, size):
        rc = orc.cache_readat(img, length, level, off, size)[0]
        assert rc in (0, 1)
        return rc == 0
    assert M.run(read, orc.checksum) == []


def test_open_cache_file_size_rule():
    assert orc.open_cache_file(10, 10, orc.CS_FULL) == orc.CS_NONE
    assert orc.open_cache_file(14, 10, orc.CS_EXTEND) == orc.CS_EXTEND
    assert orc.open_cache_file(15, 10, orc.CS_FULL) == -1
    assert orc.open_cache_file(4, 0, orc.CS_FULL) == orc.CS_FULL  # empty block keeps one CRC


def test_rsa_oaep_roundtrip_and_wrong_key():
    from juicefs_amd import encrypt as enc
    k1 = enc.GenerateRsaKey(2048)
    k2 = enc.GenerateRsaKey(2048)
    e1, e2 = enc.NewRSAEncryptor(k1), enc.NewRSAEncryptor(k2)
    secret = bytes(range(32))
    c = e1.Encrypt(secret)
    assert len(c) == 256 and c != e1.Encrypt(secret)  # OAEP is randomised
    assert e1.Decrypt(c) == secret
    with pytest.raises(enc.EncryptError):
        e2.Decrypt(c)
    # PEM round trip (ParseRsaPrivateKeyFromPem)
    k3 = enc.ParseRsaPrivateKeyFromPem(k1.to_pem())
    assert enc.NewRSAEncryptor(k3).Decrypt(c) == secret
    with pytest.raises(enc.EncryptError, match="failed to parse PEM"):
        enc.ParseRsaPrivateKeyFromPem(b"not a key")


def test_new_data_encryptor_dispatch():
    from juicefs_amd import encrypt as enc
    class Null:
        def Encrypt(self, b): return b
        def Decrypt(self, b): return b
    assert enc.NewDataEncryptor(Null(), "").algo == 0
    assert enc.NewDataEncryptor(Null(), "aes256gcm-rsa").algo == 0
    assert enc.NewDataEncryptor(Null(), "chacha20-rsa").algo == 1
    with pytest.raises(enc.EncryptError, match="unsupport cipher: sm4"):
        enc.NewDataEncryptor(Null(), "sm4")


def _pem_fixtures():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "pem_fixtures.json")) as f:
        return json.load(f)


def test_parse_pkcs8_fixture():
    """TestParsePKCS8 (encrypt_test.go:69-78) on the reference's own key
    fixture: the right passphrase parses, a wrong one fails."""
    from juicefs_amd import encrypt as enc
    fx = _pem_fixtures()
    k = enc.ParseRsaPrivateKeyFromPem(fx["keyInPKCS8"].encode(), b"12345678")
    with pytest.raises(enc.EncryptError):
        enc.ParseRsaPrivateKeyFromPem(fx["keyInPKCS8"].encode(), b"1234567")
    # the parsed key wraps and unwraps a data key (rsaEncryptor, encrypt.go:124-134)
    e = enc.NewRSAEncryptor(k)
    secret = bytes(range(100, 132))
    assert e.Decrypt(e.Encrypt(secret)) == secret


def test_parse_pem_without_password_fixture():
    """TestParsePemWithoutPassword (encrypt_test.go:80-89): a PKCS#1 key parses
    with no passphrase, and a passphrase given for an unencrypted key is
    ignored."""
    from juicefs_amd import encrypt as enc
    fx = _pem_fixtures()
    k1 = enc.ParseRsaPrivateKeyFromPem(fx["pemWithoutPass"].encode(), None)
    k2 = enc.ParseRsaPrivateKeyFromPem(fx["pemWithoutPass"].encode(), b"123")
    assert k1.size == k2.size == 128  # 1024-bit fixture key
    e1, e2 = enc.NewRSAEncryptor(k1), enc.NewRSAEncryptor(k2)
    secret = bytes(32)
    assert e2.Decrypt(e1.Encrypt(secret)) == secret


# ---- pkg/compress/compress.go mirror (host logic; no GPU calls) ----------
def test_new_compressor_names():
    from juicefs_amd import compress as C
    assert isinstance(C.NewCompressor("LZ4"), C.LZ4)
    assert isinstance(C.NewCompressor("zstd"), C.ZStandard)
    assert isinstance(C.NewCompressor(""), C.noOp) and isinstance(C.NewCompressor("none"), C.noOp)
    assert C.NewCompressor("gzip") is None
    assert [C.NewCompressor(a).Name() for a in ("lz4", "zstd", "none")] == ["LZ4", "Zstd", "Noop"]


def test_compress_bounds_and_noop_errors():
    import pytest
    from juicefs_amd import compress as C
    lz = C.NewCompressor("lz4")
    for n in (0, 1, 254, 255, 4 << 20):
        assert lz.CompressBound(n) == n + n // 255 + 16  # LZ4_COMPRESSBOUND
    assert C.ZStandard().CompressBound(4 << 20) == (4 << 20) + (4 << 12)
    assert C.ZStandard().CompressBound(1000) == 1000 + 3 + ((128 << 10) - 1000) // 2048
    nop = C.noOp()
    assert nop.CompressBound(77) == 77
    buf = bytearray(3)
    with pytest.raises(C.CompressError, match="buffer too short: 3 < 4"):
        nop.Compress(buf, b"abcd")
    assert nop.Decompress(bytearray(4), b"abcd") == 4
    with pytest.raises(C.CompressError, match="decompress an empty input"):
        lz.Decompress(bytearray(10), b"")
    # zstd.CompressLevel allocates its own buffer below CompressBound, which
    # compress.go:87-89 reports; an empty frame input is DataDog's empty-slice
    # error (both decided before any engine call)
    z = C.ZStandard()
    with pytest.raises(C.CompressError, match="buffer too short: 10 < %d" % z.CompressBound(1)):
        z.Compress(bytearray(10), b"x")
    with pytest.raises(C.CompressError, match="Bytes slice is empty"):
        z.Decompress(bytearray(10), b"")
