"""The reference's encrypt_test.go / disk_cache_test.go behaviours, run on the
GPU engine through the mirrored interfaces (juicefs_amd.encrypt / .chunk)."""
import os

import numpy as np
import pytest

from juicefs_amd import chunk
from juicefs_amd import encrypt as enc
from oracle import oracle as orc
from tests import checksum_matrix as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rsa():
    return enc.NewRSAEncryptor(enc.GenerateRsaKey(2048))


@pytest.mark.parametrize("algo", [enc.CHACHA20_RSA, enc.AES256GCM_RSA])
def test_hello_roundtrip(rsa, algo):
    # TestChaCha20 / TestAESGCM (encrypt_test.go:182-204)
    dc = enc.NewDataEncryptor(rsa, algo)
    ct = dc.Encrypt(b"hello")
    assert len(ct) == 3 + 256 + 12 + 5 + 16
    assert dc.Decrypt(ct) == b"hello"


def test_encrypted_store_range_get(rsa):
    # TestEncryptedStore (encrypt_test.go:206-227)
    es = enc.NewEncrypted(enc.MemStorage(), enc.NewDataEncryptor(rsa, enc.AES256GCM_RSA))
    es.Put("a", b"hello")
    assert es.Get("a", 1, 2) == b"el"
    assert es.Get("a", 0, -1) == b"hello"
    assert es.Get("a", 9, 3) == b""
    assert es.String() == "mem://(encrypted)"


@pytest.mark.parametrize("algo", [enc.CHACHA20_RSA, enc.AES256GCM_RSA])
def test_object_matches_oracle_after_unwrap(rsa, algo):
    dc = enc.NewDataEncryptor(rsa, algo)
    p = orc.gen_block(3, 1, 100003).tobytes()
    obj = dc.Encrypt(p)
    klen = (obj[0] << 8) + obj[1]
    key = rsa.Decrypt(obj[3:3 + klen])
    o_algo = orc.AES256GCM if algo == enc.AES256GCM_RSA else orc.CHACHA20P1305
    assert orc.data_decrypt(o_algo, key, obj) == p


@pytest.mark.parametrize("algo", [enc.CHACHA20_RSA, enc.AES256GCM_RSA])
def test_decrypt_errors(rsa, algo):
    dc = enc.NewDataEncryptor(rsa, algo)
    obj = dc.Encrypt(b"hello world")
    with pytest.raises(enc.EncryptError, match="misformed ciphertext: 256 12"):
        dc.Decrypt(obj[:271])
    bad = bytearray(obj)
    bad[-1] ^= 1
    msg = "cipher: message authentication failed" if algo == enc.AES256GCM_RSA else \
        "chacha20poly1305: message authentication failed"
    with pytest.raises(enc.EncryptError, match=msg):
        dc.Decrypt(bytes(bad))
    other = enc.NewDataEncryptor(enc.NewRSAEncryptor(enc.GenerateRsaKey(2048)), algo)
    with pytest.raises(enc.EncryptError, match="decryt key: "):
        other.Decrypt(obj)


def test_batch_encrypt_decrypt(rsa):
    dc = enc.NewDataEncryptor(rsa, enc.AES256GCM_RSA)
    rng = np.random.default_rng(5)
    ps = [orc.gen_block(5, i, int(n)).tobytes() for i, n in enumerate(rng.integers(0, 300000, 24))]
    objs = dc.EncryptBatch(ps)
    objs[7] = objs[7][:-1] + bytes([objs[7][-1] ^ 0x40])
    out = dc.DecryptBatch(objs)
    for i, (p, o) in enumerate(zip(ps, out)):
        if i == 7:
            assert isinstance(o, enc.EncryptError)
        else:
            assert o == p


def test_checksum_matrix_on_files(tmp_path):
    # TestChecksum (disk_cache_test.go:134-221) through openCacheFile/ReadAt on real files
    def read(img, length, level, off, size):
        path = os.path.join(str(tmp_path), "blk")
        with open(path, "wb") as f:
            f.write(img)
        cf = chunk.openCacheFile(path, length, level)
        try:
            data, n = cf.ReadAt(size, off)
        except chunk.ChecksumError as e:
            assert str(e).startswith("data checksum ")
            return False
        assert data == img[off:off + size] and n == size
        return True
    assert M.run(read, chunk.checksum) == []


def test_write_cache_file_layout(tmp_path):
    d = orc.gen_block(6, 0, 70000).tobytes()
    p = os.path.join(str(tmp_path), "c")
    chunk.write_cache_file(p, d, chunk.CsFull)
    raw = open(p, "rb").read()
    assert raw == d + orc.checksum(d)
    chunk.write_cache_file(p, d, chunk.CsNone)
    assert open(p, "rb").read() == d


# ---- compress stage around the block store (cached_store.go:371-392, 673-745) ----
def test_upload_load_blocks_lz4_through_encrypted_store():
    from juicefs_amd import compress as C
    from juicefs_amd import encrypt as EN
    from tests import lz4_data
    priv = EN.GenerateRsaKey(2048)
    enc = EN.NewDataEncryptor(EN.NewRSAEncryptor(priv), EN.CHACHA20_RSA)
    store = EN.NewEncrypted(EN.MemStorage(), enc)
    lz = C.NewCompressor("lz4")
    blocks = [lz4_data.sample(k, n, seed=i) for i, (k, n) in
              enumerate([("text", 4 << 20), ("random", 1 << 20), ("zeros", 70000), ("runs", 12345), ("text", 5)])]
    keys = ["chunks/0/0/%d_0_%d" % (i, len(b)) for i, b in enumerate(blocks)]
    outs = C.upload_blocks(store, keys, blocks, lz)
    from oracle import oracle as orc
    assert outs == [orc.lz4_compress(b) for b in blocks]
    assert len(outs[0]) < len(blocks[0]) // 2 and len(outs[2]) < 1000
    assert C.load_blocks(store, keys, [len(b) for b in blocks], lz) == blocks
    # a block whose object decodes short of its length: "read %s fully"
    store.Put(keys[3], orc.lz4_compress(blocks[3][:-1]))
    import pytest
    with pytest.raises(C.CompressError, match="read chunks/0/0/3_0_12345 fully"):
        C.load_blocks(store, keys[3:4], [len(blocks[3])], lz)


def test_lz4_compressor_single_calls():
    from juicefs_amd import compress as C
    lz = C.NewCompressor("lz4")
    src = b"abcabcabcabc" * 1000
    dst = bytearray(lz.CompressBound(len(src)))
    n = lz.Compress(dst, src)
    page = bytearray(len(src))
    assert lz.Decompress(page, bytes(dst[:n])) == len(src) and bytes(page) == src
    import pytest
    with pytest.raises(C.CompressError, match="lz4: malformed block"):
        lz.Decompress(bytearray(len(src)), bytes(dst[:n - 3]))
