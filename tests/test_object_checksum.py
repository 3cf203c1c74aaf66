"""Object-store CRC32C (pkg/object/checksum.go) -- §8(f)-1.

CPU: the host combine helpers of the C-ABI against the oracle and against the
values the reference's own test computes (object/checksum_test.go:30-44 hashes
"hello" with crc32.Update; CRC32C("123456789") is the standard check value).
GPU: the ciphertext-side segment CRCs (JFSX_CRC_CT) fused into Seal/Open, the
whole-object checksum of data_encrypt/data_decrypt, and the checksum.py mirror
(ChecksumStorage under Encrypted) -- all against oracle.object_checksum.
"""
import numpy as np
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc

SEG = 32 << 10


def test_update_known_values():
    assert E.crc32c_update(0, b"hello") == 2591144780
    assert E.crc32c_update(0, b"123456789") == 0xE3069283
    assert E.crc32c_update(0, b"") == 0
    # streaming: Update(Update(0, a), b) == Update(0, a||b)
    assert E.crc32c_update(E.crc32c_update(0, b"hel"), b"lo") == 2591144780


@pytest.mark.parametrize("na,nb", [(0, 5), (5, 0), (1, 1), (271, 32768), (32768, 32767), (100000, 4097)])
def test_combine_vs_oracle(na, nb):
    rng = np.random.default_rng(na * 7 + nb)
    a = rng.integers(0, 256, na, dtype=np.uint8).tobytes()
    b = rng.integers(0, 256, nb, dtype=np.uint8).tobytes()
    assert E.crc32c_combine(orc.crc32c(a), orc.crc32c(b), nb) == orc.crc32c(a + b)


@pytest.mark.parametrize("clen", [0, 1, 15, 16, 32767, 32768, 32769, 98309, (1 << 20) + 3])
def test_object_crc_from_segments_vs_oracle(clen):
    # segments as the engine returns them for C: checksum(C), big-endian
    rng = np.random.default_rng(clen)
    hdr = bytes([1, 0, 12]) + rng.integers(0, 256, 268, dtype=np.uint8).tobytes()
    c = rng.integers(0, 256, clen, dtype=np.uint8).tobytes()
    tag = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    segs = orc.checksum(c, hw=True)
    got = E.object_crc32c(hdr, segs, clen, tag)
    assert str(got) == orc.object_checksum(hdr + c + tag)


def test_verify_checksum_passthrough_rules():
    from juicefs_amd import checksum as cs
    body = b"abc"
    assert cs.verifyChecksum(body, "", 3) is body       # no metadata: unchecked
    assert cs.verifyChecksum(body, "xyz", 3) is body    # unparsable: logged and ignored
    # strconv.Atoi's grammar: sign and digits only, int64 range; uint32() wraps
    assert cs.parse_checksum("2591144780") == 2591144780
    assert cs.parse_checksum("+7") == 7 and cs.parse_checksum("-1") == 0xFFFFFFFF
    assert cs.parse_checksum(str((1 << 32) + 5)) == 5
    for bad in ("", " 7", "7 ", "1_0", "0x10", "9223372036854775808", None):
        assert cs.parse_checksum(bad) is None, bad
        assert cs.verifyChecksum(body, bad, 3) is body


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


ALGOS = [E.AES256GCM, E.CHACHA20P1305]
ORC = {E.AES256GCM: orc.AES256GCM, E.CHACHA20P1305: orc.CHACHA20P1305}
LENS = [0, 1, 17, 1024, 32767, 32768, 32769, 65536 + 5, 300001, (1 << 20) + 16, (4 << 20) - 1, 4 << 20]


def _batch(eng, algo, items, open_, crc_mode):
    bufs, specs = [], []
    for key, nonce, data, tag in items:
        src = eng.alloc(max(data.size, 16))
        dst = eng.alloc(max(data.size, 16))
        src.upload(data)
        nseg = max(1, -(-data.size // SEG))
        cb = eng.alloc(4 * nseg)
        bufs.append((src, dst, cb, nseg, data.size))
        sp = {"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": data.size, "crc": cb.ptr}
        if tag is not None:
            sp["tag"] = tag
        specs.append(sp)
    arr, n = eng.make_blocks(specs)
    (eng.open_batch if open_ else eng.seal_batch)(algo, arr, n, crc_mode, E.MEM_DEVICE)
    return [(b[1].download(b[4]).tobytes(), bytes(arr[i].tag), b[2].download(4 * b[3]).tobytes(), arr[i].status)
            for i, b in enumerate(bufs)]


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ALGOS)
def test_seal_open_ct_segments_vs_oracle(eng, algo):
    items = []
    for i, n in enumerate(LENS):
        key, nonce = orc.gen_key(21, i)
        items.append((key, nonce, orc.gen_block(21, i, n), None))
    sealed = _batch(eng, algo, items, False, E.CRC_GEN | E.CRC_CT)
    opened_in = []
    for (key, nonce, p, _), (c, tag, crc, st) in zip(items, sealed):
        c2, t2 = orc.seal(ORC[algo], key, nonce, p, fast=True)
        assert st == E.OK and c == c2 and tag == t2
        assert crc == orc.checksum(np.frombuffer(c, np.uint8), hw=True), "seal CT len %d" % p.size
        opened_in.append((key, nonce, np.frombuffer(c, np.uint8).copy(), tag))
    opened = _batch(eng, algo, opened_in, True, E.CRC_GEN | E.CRC_CT)
    for (key, nonce, c, tag), (p, _, crc, st), (_, _, p0, _) in zip(opened_in, opened, items):
        assert st == E.OK and p == p0.tobytes()
        assert crc == orc.checksum(c, hw=True), "open CT len %d" % c.size


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ALGOS)
def test_open_ct_verify_detects_corruption(eng, algo):
    key, nonce = orc.gen_key(22, 0)
    n = 3 * SEG + 100
    p = orc.gen_block(22, 0, n)
    c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
    good = orc.checksum(np.frombuffer(c, np.uint8), hw=True)
    for flip in (None, 5, SEG + 7, n - 1):
        cc = np.frombuffer(c, np.uint8).copy()
        if flip is not None:
            cc[flip] ^= 0x40
        src, dst, cb = eng.alloc(n), eng.alloc(n), eng.alloc(len(good))
        src.upload(cc)
        cb.upload(np.frombuffer(good, np.uint8))
        arr, cnt = eng.make_blocks([{"key": key, "nonce": nonce, "src": src.ptr, "dst": dst.ptr, "len": n,
                                     "crc": cb.ptr, "tag": tag}])
        eng.open_batch(algo, arr, cnt, E.CRC_VERIFY | E.CRC_CT, E.MEM_DEVICE)
        if flip is None:
            assert arr[0].status == E.OK and arr[0].crc_bad_seg == -1
        else:
            # the failing segment is located; the tag fails too (status ETAG
            # takes precedence in the per-block status, as Open's error would)
            assert arr[0].crc_bad_seg == flip // SEG
            assert arr[0].status == E.ETAG


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", [0, 5, 32768, 100003, 4 << 20])
def test_data_encrypt_object_checksum(eng, algo, n):
    key, nonce = orc.gen_key(23, n)
    p = orc.gen_block(23, 1, n).tobytes()
    wrapped = bytes(range(256))
    obj, crc = eng.data_encrypt(algo, key, nonce, wrapped, p, obj_crc=True)
    assert obj == orc.data_encrypt(ORC[algo], key, nonce, wrapped, p)
    assert str(crc) == orc.object_checksum(obj)
    rc, back = eng.data_decrypt(algo, key, obj, expect_crc=crc)
    assert rc == 0 and back == p
    rc, back = eng.data_decrypt(algo, key, obj, expect_crc=crc ^ 1)
    assert rc == E.ECRC and back == b"" and eng.last_got_crc == crc
    if n:
        bad = bytearray(obj)
        bad[len(obj) // 2] ^= 1
        rc, _ = eng.data_decrypt(algo, key, bytes(bad), expect_crc=crc)
        assert rc == E.ECRC and str(eng.last_got_crc) == orc.object_checksum(bytes(bad))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["aes256gcm-rsa", "chacha20-rsa"])
def test_encrypted_store_with_checksum_metadata(eng, algo):
    from juicefs_amd import checksum as cs
    from juicefs_amd import encrypt as enc
    priv = enc.GenerateRsaKey(2048)
    de = enc.NewDataEncryptor(enc.NewRSAEncryptor(priv), algo, eng)
    store = cs.ChecksumStorage(enc.MemStorage(), eng=eng)
    es = enc.NewEncrypted(store, de)
    data = orc.gen_block(24, 0, 200001).tobytes()
    es.Put("k", data)
    raw = store.inner.Get("k")
    assert store.GetChecksum("k") == orc.object_checksum(raw)
    assert cs.generateChecksum(raw, eng) == orc.object_checksum(raw)
    assert es.Get("k") == data and es.Get("k", 10, 20) == data[10:30]
    # corrupt the stored object: the store's checksum read fails first
    bad = bytearray(raw)
    bad[1000] ^= 0xFF
    store.inner.Put("k", bytes(bad))
    with pytest.raises(cs.ChecksumVerifyError, match="verify checksum failed"):
        es.Get("k")
    # the plain (unfused) reader path reports the same values
    with pytest.raises(cs.ChecksumVerifyError) as ei:
        store.Get("k")
    assert str(ei.value.got) == orc.object_checksum(bytes(bad))


@pytest.mark.gpu
def test_checksum_error_precedes_header_and_key_errors(eng):
    """An object that fails before the AEAD pass (misformed header, wrapped
    key that does not unwrap) still reports the store's checksum mismatch
    first, as the reference's checksumReader runs before Decrypt sees the
    bytes (checksum.go:55-70, encrypt.go:232-255); an unparsable expected
    checksum is ignored (checksum.go:76-80)."""
    from juicefs_amd import checksum as cs
    from juicefs_amd import encrypt as enc
    de = enc.NewDataEncryptor(enc.NewRSAEncryptor(enc.GenerateRsaKey(2048)), "aes256gcm-rsa", eng)
    good = de.Encrypt(b"hello world" * 100)
    misformed = good[:200]
    badkey = bytearray(good)
    badkey[10] ^= 1  # inside the wrapped key
    for obj in (misformed, bytes(badkey)):
        wrong = str((E.crc32c_update(0, obj) + 1) & 0xFFFFFFFF)
        r = de.DecryptBatch([obj], [wrong])[0]
        assert isinstance(r, cs.ChecksumVerifyError), r
        assert r.got == E.crc32c_update(0, obj)
        right = str(E.crc32c_update(0, obj))
        r = de.DecryptBatch([obj], [right])[0]
        assert isinstance(r, enc.EncryptError) and not isinstance(r, cs.ChecksumVerifyError), r
        r = de.DecryptBatch([obj], ["not-a-number"])[0]
        assert isinstance(r, enc.EncryptError), r
    assert de.DecryptBatch([good], ["x1"])[0] == b"hello world" * 100
