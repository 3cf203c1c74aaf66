"""Mirror of pkg/object/encrypt.go on the GPU engine.

Same names, argument meaning and error behaviour as the reference:

  Encryptor                  interface {Encrypt, Decrypt}            encrypt.go:38-41
  ParseRsaPrivateKeyFromPem  PEM (PKCS#1/PKCS#8, optional passphrase) encrypt.go:66-107
  NewRSAEncryptor            RSA-OAEP(SHA-256, label "keys")          encrypt.go:124-134
  NewDataEncryptor           "" / "aes256gcm-rsa" / "chacha20-rsa"    encrypt.go:142-162
  DataEncryptor.Encrypt      random key+nonce, wrap, header, Seal    encrypt.go:164-194
  DataEncryptor.Decrypt      header parse, unwrap, Open              encrypt.go:196-216
  NewEncrypted / Encrypted   object-store wrapper (Get/Put)          encrypt.go:218-267

The AEAD work (Seal/Open) runs on the HIP engine (libjfsx.so); RSA-OAEP key
wrapping stays on the host, as it does in the reference, through OpenSSL's
libcrypto.  DataEncryptor.EncryptBatch / DecryptBatch are the batched entry
points an upload/download worker pool uses (one engine call per batch).
"""
import ctypes
import ctypes.util
import os
import threading

from . import engine as E

AES256GCM_RSA = "aes256gcm-rsa"
CHACHA20_RSA = "chacha20-rsa"

_ALGO = {"": E.AES256GCM, AES256GCM_RSA: E.AES256GCM, CHACHA20_RSA: E.CHACHA20P1305}
# Go error texts: crypto/cipher gcm.go errOpen, x/crypto chacha20poly1305 errOpen
_ERR_OPEN = {E.AES256GCM: "cipher: message authentication failed",
             E.CHACHA20P1305: "chacha20poly1305: message authentication failed"}


class EncryptError(Exception):
    pass


# ---------------------------------------------------------------------------
# shared engine (one context per process, device from JFSX_DEVICE)
# ---------------------------------------------------------------------------
_eng = None
_eng_lock = threading.Lock()


def default_engine():
    global _eng
    with _eng_lock:
        if _eng is None:
            _eng = E.Engine(int(os.environ.get("JFSX_DEVICE", "0")))
        return _eng


# ---------------------------------------------------------------------------
# RSA-OAEP key wrapping through libcrypto (host side, as in the reference)
# ---------------------------------------------------------------------------
class _Crypto:
    _inst = None

    def __init__(self):
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(path)
        P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        for name, res, args in [
            ("BIO_new_mem_buf", P, [P, I]), ("BIO_free", I, [P]),
            ("PEM_read_bio_PrivateKey", P, [P, P, P, P]), ("EVP_PKEY_free", None, [P]),
            ("EVP_PKEY_CTX_new", P, [P, P]), ("EVP_PKEY_CTX_free", None, [P]),
            ("EVP_PKEY_encrypt_init", I, [P]), ("EVP_PKEY_decrypt_init", I, [P]),
            ("EVP_PKEY_encrypt", I, [P, P, ctypes.POINTER(SZ), P, SZ]),
            ("EVP_PKEY_decrypt", I, [P, P, ctypes.POINTER(SZ), P, SZ]),
            ("EVP_PKEY_CTX_set_rsa_padding", I, [P, I]), ("EVP_PKEY_CTX_set_rsa_oaep_md", I, [P, P]),
            ("EVP_PKEY_CTX_set_rsa_mgf1_md", I, [P, P]), ("EVP_PKEY_CTX_set0_rsa_oaep_label", I, [P, P, I]),
            ("EVP_sha256", P, []), ("CRYPTO_malloc", P, [SZ, ctypes.c_char_p, I]),
            ("EVP_PKEY_get_size", I, [P]),
            ("PEM_write_bio_PrivateKey", I, [P, P, P, P, I, P, P]), ("BIO_new", P, [P]),
            ("BIO_s_mem", P, []), ("BIO_ctrl", ctypes.c_long, [P, I, ctypes.c_long, P]),
            ("ERR_clear_error", None, []),
            ("EVP_PKEY_get_bn_param", I, [P, ctypes.c_char_p, ctypes.POINTER(P)]),
            ("BN_bn2binpad", I, [P, P, I]), ("BN_free", None, [P]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        L.EVP_PKEY_Q_keygen.restype = P  # variadic: (libctx, propq, "RSA", size_t bits)
        self.L = L

    @classmethod
    def get(cls):
        if cls._inst is None:
            cls._inst = _Crypto()
        return cls._inst


class RSAPrivateKey:
    """An RSA private key held by libcrypto (EVP_PKEY)."""

    def __init__(self, pkey):
        self._pkey = pkey

    def __del__(self):
        try:
            _Crypto.get().L.EVP_PKEY_free(self._pkey)
        except Exception:
            pass

    @property
    def size(self):
        return _Crypto.get().L.EVP_PKEY_get_size(self._pkey)

    def to_pem(self):
        L = _Crypto.get().L
        bio = L.BIO_new(L.BIO_s_mem())
        try:
            if L.PEM_write_bio_PrivateKey(bio, self._pkey, None, None, 0, None, None) != 1:
                raise EncryptError("cannot export key")
            ptr = ctypes.c_void_p()
            n = L.BIO_ctrl(bio, 3, 0, ctypes.byref(ptr))  # BIO_CTRL_INFO = 3 (BIO_get_mem_data)
            return ctypes.string_at(ptr, n)
        finally:
            L.BIO_free(bio)


def GenerateRsaKey(bits=2048):
    """The `openssl genrsa 2048` the reference's docs use (docs/en/security/encryption.md)."""
    pkey = _Crypto.get().L.EVP_PKEY_Q_keygen(None, None, b"RSA", ctypes.c_size_t(bits))
    if not pkey:
        raise EncryptError("RSA key generation failed")
    return RSAPrivateKey(pkey)


def ParseRsaPrivateKeyFromPem(enc, passphrase=b""):
    """encrypt.go:66-107: PKCS#1 or PKCS#8 PEM, optionally passphrase-protected."""
    L = _Crypto.get().L
    data = bytes(enc)
    buf = ctypes.create_string_buffer(data, len(data))
    bio = L.BIO_new_mem_buf(buf, len(data))
    try:
        pw = ctypes.c_char_p(bytes(passphrase)) if passphrase else None
        pkey = L.PEM_read_bio_PrivateKey(bio, None, None, pw)
    finally:
        L.BIO_free(bio)
    if not pkey:
        L.ERR_clear_error()
        if b"-----BEGIN" not in data:
            raise EncryptError("failed to parse PEM block containing the key")
        raise EncryptError("cannot decode private key (wrong passphrase or not an RSA key)")
    return RSAPrivateKey(pkey)


def ParseRsaPrivateKeyFromPath(path, passphrase=""):
    """encrypt.go:109-122 (JFS_RSA_PASSPHRASE is the caller's business)."""
    with open(path, "rb") as f:
        b = f.read()
    if not passphrase and b"ENCRYPTED" in b:
        raise EncryptError("passphrase is required to private key, please try again after setting the "
                           "'JFS_RSA_PASSPHRASE' environment variable")
    return ParseRsaPrivateKeyFromPem(b, passphrase.encode() if isinstance(passphrase, str) else passphrase)


def rsa_crt_components(priv, nbytes=128):
    """(p, q, dp, dq, qinv) of an RSA private key, big-endian, nbytes each --
    the precomputed CRT values Go's rsa.PrivateKey carries (Primes, Dp, Dq,
    Qinv), which the engine's batched unwrap consumes."""
    L = _Crypto.get().L
    out = []
    for name in (b"rsa-factor1", b"rsa-factor2", b"rsa-exponent1", b"rsa-exponent2", b"rsa-coefficient1"):
        bn = ctypes.c_void_p()
        if L.EVP_PKEY_get_bn_param(priv._pkey, name, ctypes.byref(bn)) != 1:
            L.ERR_clear_error()
            raise EncryptError("not an RSA private key with CRT parameters")
        try:
            buf = ctypes.create_string_buffer(nbytes)
            if L.BN_bn2binpad(bn, buf, nbytes) != nbytes:
                raise EncryptError("RSA CRT parameter %s does not fit %d bytes" % (name.decode(), nbytes))
            out.append(buf.raw)
        finally:
            L.BN_free(bn)
    return tuple(out)


class RsaEncryptor:
    """rsaEncryptor: RSA-OAEP with SHA-256 (OAEP and MGF1) and label "keys"."""

    def __init__(self, priv, label=b"keys"):
        self.privKey = priv
        self.label = label

    def _ctx(self, decrypt):
        C = _Crypto.get()
        L = C.L
        ctx = L.EVP_PKEY_CTX_new(self.privKey._pkey, None)
        ok = (L.EVP_PKEY_decrypt_init(ctx) if decrypt else L.EVP_PKEY_encrypt_init(ctx)) == 1
        ok = ok and L.EVP_PKEY_CTX_set_rsa_padding(ctx, 4) == 1  # RSA_PKCS1_OAEP_PADDING
        ok = ok and L.EVP_PKEY_CTX_set_rsa_oaep_md(ctx, L.EVP_sha256()) == 1
        ok = ok and L.EVP_PKEY_CTX_set_rsa_mgf1_md(ctx, L.EVP_sha256()) == 1
        if ok and self.label:
            lab = L.CRYPTO_malloc(len(self.label), b"encrypt.py", 0)  # ownership passes to the ctx
            ctypes.memmove(lab, self.label, len(self.label))
            ok = L.EVP_PKEY_CTX_set0_rsa_oaep_label(ctx, lab, len(self.label)) == 1
        if not ok:
            L.EVP_PKEY_CTX_free(ctx)
            raise EncryptError("rsa oaep setup failed")
        return ctx

    def _run(self, data, decrypt):
        L = _Crypto.get().L
        ctx = self._ctx(decrypt)
        try:
            n = ctypes.c_size_t(self.privKey.size)
            out = ctypes.create_string_buffer(n.value)
            f = L.EVP_PKEY_decrypt if decrypt else L.EVP_PKEY_encrypt
            if f(ctx, out, ctypes.byref(n), data, len(data)) != 1:
                L.ERR_clear_error()
                raise EncryptError("crypto/rsa: decryption error" if decrypt else "crypto/rsa: message too long")
            return out.raw[:n.value]
        finally:
            L.EVP_PKEY_CTX_free(ctx)

    def Encrypt(self, plaintext):
        return self._run(bytes(plaintext), False)

    def Decrypt(self, ciphertext):
        return self._run(bytes(ciphertext), True)

    def DecryptBatch(self, ciphertexts, eng=None):
        """Decrypt for a whole read window at once: the engine's batched
        RSA-OAEP unwrap on the GPU, bit-exact to
        rsa.DecryptOAEP.  Returns, per item, the plaintext or the EncryptError
        Decrypt would raise.  Keys the engine does not take (not RSA-2048)
        unwrap on the host as the reference does (encrypt.go:132-134)."""
        eng = eng or default_engine()
        dk = self._device_key(eng)
        if dk is None:
            out = []
            for c in ciphertexts:
                try:
                    out.append(self.Decrypt(c))
                except EncryptError as e:
                    out.append(e)
            return out
        res = eng.oaep_decrypt_batch(dk, ciphertexts)
        return [EncryptError("crypto/rsa: decryption error") if r is None else r for r in res]

    def _device_key(self, eng):
        keys = self.__dict__.setdefault("_dev_keys", {})
        if eng.ctx not in keys:
            try:
                keys[eng.ctx] = eng.rsa_key(*rsa_crt_components(self.privKey), label=self.label)
            except Exception:  # not RSA-2048 with CRT parameters
                keys[eng.ctx] = None
        return keys[eng.ctx]


def NewRSAEncryptor(privKey):
    return RsaEncryptor(privKey, b"keys")


# ---------------------------------------------------------------------------
# dataEncryptor
# ---------------------------------------------------------------------------
class DataEncryptor:
    """dataEncryptor: per-object random 32-byte key + 12-byte nonce, the key
    wrapped by keyEncryptor, AEAD on the GPU engine."""

    keyLen = 32

    def __init__(self, keyEncryptor, algo, eng=None, rand=os.urandom, agg=None):
        """agg: an engine.Aggregator; one-object Encrypt/Decrypt calls made
        concurrently from many threads (the reference's per-goroutine calls)
        are then coalesced into engine batches."""
        self.keyEncryptor = keyEncryptor
        self.algo = algo
        self._eng = eng
        self._rand = rand
        self._agg = agg

    @property
    def eng(self):
        return self._eng or default_engine()

    def Encrypt(self, plaintext):
        return self.EncryptBatch([plaintext])[0]

    def Decrypt(self, ciphertext):
        r = self.DecryptBatch([ciphertext])[0]
        if isinstance(r, Exception):
            raise r
        return r

    def EncryptBatch(self, plaintexts, checksums=False):
        """Encrypt many objects with one engine call (the shim's aggregation
        window).  checksums=True also returns each stored object's CRC32C
        (checksum.go:31-53), computed in the same pass (JFSX_CRC_CT): then the
        result is a list of (object, checksum string)."""
        import numpy as np
        specs, outs, hdrs, segs = [], [], [], []
        for p in plaintexts:
            p = bytes(p)
            key = self._rand(self.keyLen)
            cipherkey = self.keyEncryptor.Encrypt(key)
            nonce = self._rand(12)
            hdr = bytes([len(cipherkey) >> 8, len(cipherkey) & 0xFF, len(nonce)]) + cipherkey + nonce
            src = np.frombuffer(p, np.uint8).copy() if p else np.zeros(1, np.uint8)
            dst = np.empty(max(len(p), 1), np.uint8)
            outs.append((src, dst, len(p)))
            hdrs.append(hdr)
            spec = {"key": key, "nonce": nonce, "src": src.ctypes.data if p else None, "dst": dst.ctypes.data,
                    "len": len(p)}
            if checksums:
                sb = np.zeros(4 * max(1, -(-len(p) // (32 << 10))), np.uint8)
                segs.append(sb)
                spec["crc"] = sb.ctypes.data
            specs.append(spec)
        if not specs:
            return []
        arr, n = self.eng.make_blocks(specs)
        mode = E.CRC_GEN | E.CRC_CT if checksums else E.CRC_NONE
        if self._agg is not None and n == 1:
            self._agg.seal(self.algo, arr[0], mode, E.MEM_HOST)
        else:
            self.eng.seal_batch(self.algo, arr, n, mode, E.MEM_HOST)
        objs = [hdrs[i] + outs[i][1][:outs[i][2]].tobytes() + bytes(arr[i].tag) for i in range(n)]
        if not checksums:
            return objs
        return [(objs[i], str(self.eng.object_crc32c(hdrs[i], segs[i], outs[i][2], bytes(arr[i].tag))))
                for i in range(n)]

    def DecryptBatch(self, ciphertexts, checksums=None):
        """Returns, per object, the plaintext or the exception Decrypt would
        raise.  checksums (optional, one decimal string or None per object) are
        the object-store CRC32Cs to verify in the same pass; a mismatch yields
        the store's "verify checksum failed" error (checksum.go:65)."""
        import numpy as np
        from .checksum import ChecksumVerifyError, parse_checksum
        res = [None] * len(ciphertexts)
        want = [parse_checksum(checksums[i]) if checksums is not None else None for i in range(len(ciphertexts))]
        specs, idx, bufs, segs = [], [], [], []
        parsed = []
        for i, c in enumerate(ciphertexts):
            c = bytes(c)
            if len(c) < 3:
                res[i] = EncryptError("misformed ciphertext: 0 0")
                continue
            keyLen = (c[0] << 8) + c[1]
            nonceLen = c[2]
            if 3 + keyLen + nonceLen >= len(c):
                res[i] = EncryptError("misformed ciphertext: %d %d" % (keyLen, nonceLen))
                continue
            parsed.append((i, c, keyLen, nonceLen))
        # unwrap every object key of the window at once when the key encryptor
        # batches (the GPU RSA-OAEP unwrap), else one by one (encrypt.go:207)
        wrapped = [c[3:3 + kl] for _, c, kl, _ in parsed]
        if hasattr(self.keyEncryptor, "DecryptBatch"):
            keys = self.keyEncryptor.DecryptBatch(wrapped, self.eng)
        else:
            keys = []
            for w in wrapped:
                try:
                    keys.append(self.keyEncryptor.Decrypt(w))
                except Exception as e:
                    keys.append(e)
        for (i, c, keyLen, nonceLen), key in zip(parsed, keys):
            body = c[3:]
            nonce = body[keyLen:keyLen + nonceLen]
            ct = body[keyLen + nonceLen:]
            if isinstance(key, Exception):  # encrypt.go:207-210
                res[i] = EncryptError("decryt key: " + str(key))
                continue
            if len(key) != self.keyLen:
                res[i] = EncryptError("crypto/aes: invalid key size %d" % len(key))
                continue
            if nonceLen != 12 or len(ct) < 16:
                res[i] = EncryptError(_ERR_OPEN[self.algo])
                continue
            n = len(ct) - 16
            src = np.frombuffer(ct[:n], np.uint8).copy() if n else np.zeros(1, np.uint8)
            dst = np.zeros(max(n, 1), np.uint8)
            bufs.append((src, dst, n))
            idx.append(i)
            spec = {"key": key, "nonce": nonce, "src": src.ctypes.data if n else None, "dst": dst.ctypes.data,
                    "len": n, "tag": ct[n:]}
            if checksums is not None:
                sb = np.zeros(4 * max(1, -(-n // (32 << 10))), np.uint8)
                segs.append((sb, c[:3 + keyLen + nonceLen], checksums[i]))
                spec["crc"] = sb.ctypes.data
            specs.append(spec)
        if specs:
            arr, cnt = self.eng.make_blocks(specs)
            mode = E.CRC_GEN | E.CRC_CT if checksums is not None else E.CRC_NONE
            if self._agg is not None and cnt == 1:
                self._agg.open(self.algo, arr[0], mode, E.MEM_HOST)
            else:
                self.eng.open_batch(self.algo, arr, cnt, mode, E.MEM_HOST)
            for k, i in enumerate(idx):
                if want[i] is not None:
                    sb, hdr, _ = segs[k]
                    got = self.eng.object_crc32c(hdr, sb, bufs[k][2], bytes(arr[k].tag))
                    if got != want[i]:  # the store's read fails before Decrypt
                        res[i] = ChecksumVerifyError(got, want[i])
                        continue
                if arr[k].status == E.ETAG:
                    res[i] = EncryptError(_ERR_OPEN[self.algo])
                else:
                    res[i] = bufs[k][1][:bufs[k][2]].tobytes()
        # objects that failed before the AEAD pass (header, key unwrap, nonce):
        # the store's checksumReader still runs first (checksum.go:55-70), so a
        # checksum mismatch is the error they report
        opened = set(idx)
        for i, c in enumerate(ciphertexts):
            if want[i] is not None and i not in opened:
                got = E.crc32c_update(0, bytes(c))
                if got != want[i]:
                    res[i] = ChecksumVerifyError(got, want[i])
        return res


def NewDataEncryptor(keyEncryptor, algo, eng=None, agg=None):
    """encrypt.go:147-162."""
    if algo not in _ALGO:
        raise EncryptError("unsupport cipher: %s" % algo)
    return DataEncryptor(keyEncryptor, _ALGO[algo], eng, agg=agg)


# ---------------------------------------------------------------------------
# object storage wrapper (encrypted)
# ---------------------------------------------------------------------------
class MemStorage:
    """Minimal in-memory object store (the reference's "mem" backend,
    pkg/object/mem.go) for tests and examples."""

    def __init__(self):
        self._d = {}

    def String(self):
        return "mem://"

    def Put(self, key, data):
        self._d[key] = bytes(data)

    def Get(self, key, off=0, limit=-1):
        if key not in self._d:
            raise KeyError(key)
        d = self._d[key]
        if limit < 0:
            return d[off:]
        return d[off:off + limit]

    def Delete(self, key):
        self._d.pop(key, None)

    def Head(self, key):
        return len(self._d[key])

    def List(self, prefix=""):
        return sorted(k for k in self._d if k.startswith(prefix))


class Encrypted:
    """encrypted ObjectStorage: Put seals the whole object, Get opens the whole
    object then slices [off, off+limit) (encrypt.go:232-267)."""

    def __init__(self, store, enc):
        self.store = store
        self.enc = enc

    def String(self):
        return "%s(encrypted)" % self.store.String()

    def _fused(self):
        # a store that keeps the object CRC32C as metadata (checksum.ChecksumStorage,
        # the S3/OSS/COS path): hash the stored bytes inside the Seal/Open pass
        return getattr(self.store, "GetChecksum", None) is not None and not self.store.disableChecksum \
            and hasattr(self.enc, "EncryptBatch")

    def Get(self, key, off=0, limit=-1):
        if self._fused() and self.store.GetChecksum(key) is not None:
            ciphertext = self.store.inner.Get(key, 0, -1)
            r = self.enc.DecryptBatch([ciphertext], [self.store.GetChecksum(key)])[0]
            from .checksum import ChecksumVerifyError
            if isinstance(r, ChecksumVerifyError):
                raise r  # a read error of the store (io.ReadAll), not wrapped
            if isinstance(r, Exception):
                raise EncryptError("Decrypt: %s" % r)
            plain = r
        else:
            ciphertext = self.store.Get(key, 0, -1)
            try:
                plain = self.enc.Decrypt(ciphertext)
            except Exception as e:
                raise EncryptError("Decrypt: %s" % e)
        n = len(plain)
        if off > n:
            off = n
        if limit == -1 or off + limit > n:
            limit = n - off
        return plain[off:off + limit]

    def Put(self, key, data):
        if self._fused():
            obj, cs = self.enc.EncryptBatch([bytes(data)], checksums=True)[0]
            self.store.Put(key, obj, checksum=cs)
        else:
            self.store.Put(key, self.enc.Encrypt(bytes(data)))

    def Delete(self, key):
        self.store.Delete(key)

    def List(self, prefix=""):
        return self.store.List(prefix)


def NewEncrypted(store, enc):
    return Encrypted(store, enc)
