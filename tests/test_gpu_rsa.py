"""GPU parity of the batched RSA-OAEP key unwrap (jfsx_rsa.hip) against
libcrypto's RSA-OAEP(SHA-256, label "keys") -- the rsaEncryptor of
pkg/object/encrypt.go:124-134 -- and the batched DataEncryptor.DecryptBatch
that uses it (encrypt.go:196-216)."""
import os

import pytest

from juicefs_amd import encrypt as enc
from juicefs_amd import engine as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def rsae():
    return enc.NewRSAEncryptor(enc.GenerateRsaKey(2048))


def test_batch_unwrap_matches_libcrypto(eng, rsae):
    keys = [os.urandom(32) for _ in range(300)] + [bytes(32), b"\xff" * 32]
    wrapped = [rsae.Encrypt(k) for k in keys]
    got = rsae.DecryptBatch(wrapped, eng)
    assert got == keys
    assert [rsae.Decrypt(w) for w in wrapped[:8]] == keys[:8]


def test_batch_unwrap_errors_and_lengths(eng, rsae):
    good = rsae.Encrypt(b"k" * 32)
    bad = bytearray(good)
    bad[7] ^= 0x40
    msgs = [b"", b"x", os.urandom(190)]
    items = [bytes(bad), b"\xff" * 256, b"\x01" * 257, good[1:] if good[0] == 0 else good] + \
            [rsae.Encrypt(m) for m in msgs]
    got = rsae.DecryptBatch(items, eng)
    for r in got[:3]:
        assert isinstance(r, enc.EncryptError) and str(r) == "crypto/rsa: decryption error"
    assert got[3] == b"k" * 32
    assert got[4:] == msgs


def test_data_decrypt_batch_end_to_end(eng, rsae):
    for algo in ("aes256gcm-rsa", "chacha20-rsa"):
        de = enc.NewDataEncryptor(rsae, algo, eng)
        plains = [os.urandom(n) for n in (0, 1, 4096, 100003, 1 << 20)]
        objs = de.EncryptBatch(plains)
        assert de.DecryptBatch(objs) == plains
        broken = bytearray(objs[2])
        broken[5] ^= 1  # inside the wrapped key
        r = de.DecryptBatch([bytes(broken)])[0]
        assert isinstance(r, enc.EncryptError) and str(r).startswith("decryt key: ")
