"""Mirror of pkg/object/checksum.go -- the object-store CRC32C of a stored
object -- on the GPU engine.

  checksumAlgr = "Crc32c"                        checksum.go:29
  generateChecksum(in) -> decimal string         checksum.go:31-53
  checksumReader / verifyChecksum                checksum.go:55-82
  ChecksumStorage: Put stores the checksum as    s3.go:173-176 (Put),
  metadata, Get verifies it while reading        s3.go:140-146 (Get)

The bytes are hashed on the GPU as 32 KiB segment CRCs (jfsx_crc32c_segments)
and folded into the whole-object value on the host (jfsx_crc32c_combine);
Encrypted stores get it fused into the Seal/Open pass instead (JFSX_CRC_CT,
encrypt.DataEncryptor.EncryptBatch(checksums=True)).
"""
import re

import numpy as np

from . import engine as E
from .encrypt import default_engine

checksumAlgr = "Crc32c"
_SEG = 32 << 10


class ChecksumVerifyError(IOError):
    """"verify checksum failed: %d != %d" (checksum.go:65)."""

    def __init__(self, got, expected):
        super().__init__("verify checksum failed: %d != %d" % (got, expected))
        self.got, self.expected = got, expected


def crc32c(data, eng=None):
    """crc32.Update(0, crc32c, data) with the segment CRCs computed on the GPU."""
    eng = eng or default_engine()
    d = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data.view(np.uint8).ravel()
    if d.size == 0:
        return 0
    segs = eng.checksum(d)
    crc = 0
    for j in range(len(segs) // 4):
        lj = min(_SEG, d.size - j * _SEG)
        crc = eng.crc32c_combine(crc, int.from_bytes(segs[4 * j:4 * j + 4], "big"), lj)
    return crc


def generateChecksum(data, eng=None):
    """checksum.go:31-53: the decimal string of the CRC32C of the whole body."""
    return str(crc32c(data, eng))


class checksumReader:
    """checksum.go:55-70: hashes what is read; at EOF (or once contentLength
    bytes were read) a mismatch turns the read into an error."""

    def __init__(self, body, expected, contentLength, eng=None):
        self._b = bytes(body)
        self._pos = 0
        self.expected = expected
        self.remainingLength = contentLength
        self.checksum = 0
        self._eng = eng or default_engine()

    def Read(self, n):
        chunk = self._b[self._pos:self._pos + n]
        self._pos += len(chunk)
        eof = self._pos >= len(self._b)
        self.checksum = self._eng.crc32c_update(self.checksum, chunk)
        self.remainingLength -= len(chunk)
        if (eof or self.remainingLength == 0) and self.checksum != self.expected:
            raise ChecksumVerifyError(self.checksum, self.expected)
        return chunk

    def ReadAll(self):
        out = []
        while True:
            c = self.Read(1 << 20)
            out.append(c)
            if not c or self._pos >= len(self._b):
                break
        return b"".join(out)


def parse_checksum(checksum):
    """strconv.Atoi(checksum) then uint32(...) (checksum.go:76-81): an optional
    sign and decimal digits that fit an int64; None for "" or anything Atoi
    rejects (the reference logs "invalid crc32c" and skips verification)."""
    if checksum is None or not re.fullmatch(r"[+-]?[0-9]+", checksum):
        return None
    v = int(checksum)
    if not -(1 << 63) <= v < (1 << 63):
        return None
    return v & 0xFFFFFFFF


def verifyChecksum(body, checksum, contentLength, eng=None):
    """checksum.go:72-82: no checksum -> body unchanged; an unparsable one is
    logged and ignored; otherwise a checksumReader."""
    expected = parse_checksum(checksum)
    if expected is None:
        return body
    return checksumReader(body, expected, contentLength, eng)


class ChecksumStorage:
    """An object store that keeps the CRC32C as object metadata, as the S3 /
    OSS / COS backends do (s3.go:140-146,173-176; disable-checksum turns it
    off, s3.go:550-553).  Put(key, data, checksum=None) takes a checksum
    already computed (the fused Seal path) or computes it."""

    def __init__(self, inner, disableChecksum=False, eng=None):
        self.inner = inner
        self.disableChecksum = disableChecksum
        self._eng = eng
        self.meta = {}

    def String(self):
        return self.inner.String()

    def Put(self, key, data, checksum=None):
        if not self.disableChecksum:
            self.meta[key] = checksum if checksum is not None else generateChecksum(data, self._eng)
        self.inner.Put(key, data)

    def Get(self, key, off=0, limit=-1):
        body = self.inner.Get(key, off, limit)
        cs = self.meta.get(key)
        if off == 0 and limit == -1 and cs is not None:  # s3.go:140-146: whole-object reads only
            r = verifyChecksum(body, cs, len(body), self._eng)
            return r.ReadAll() if isinstance(r, checksumReader) else r
        return body

    def GetChecksum(self, key):
        return self.meta.get(key)

    def Delete(self, key):
        self.meta.pop(key, None)
        self.inner.Delete(key)

    def List(self, prefix=""):
        return self.inner.List(prefix)
