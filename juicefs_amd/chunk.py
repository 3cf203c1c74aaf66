"""Mirror of the disk-cache checksum surface of pkg/chunk/disk_cache.go on
the GPU engine.

  CsNone/CsFull/CsShrink/CsExtend, csBlock    disk_cache.go:1201-1208
  checksum(data) -> bytes                     disk_cache.go:1218-1231
  write_cache_file (flushPage's data||crc)    disk_cache.go:463-474
  openCacheFile(name, length, level)          disk_cache.go:1233-1253
  CacheFile.ReadAt(b, off)                    disk_cache.go:1255-1329

The CRC32C work runs on the HIP engine (jfsx_checksum / jfsx_cache_verify).
A mismatch raises ChecksumError("data checksum %d != expect %d").
"""
import os

from . import engine as E
from .encrypt import default_engine

CsNone = "none"
CsFull = "full"
CsShrink = "shrink"
CsExtend = "extend"
csBlock = 32 << 10
_LEVEL = {CsNone: 0, CsFull: 1, CsShrink: 2, CsExtend: 3}

ChecksumError = E.ChecksumError


def checksum(data, eng=None):
    """One big-endian CRC32C per 32 KiB segment (4 zero bytes for empty data)."""
    return (eng or default_engine()).checksum(data)


def write_cache_file(path, data, level, eng=None):
    """flushPage: data, then checksum(data) unless the level is none; tmp + rename."""
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(bytes(data))
        if level != CsNone:
            f.write(checksum(data, eng))
    os.replace(tmp, path)


class CacheFile:
    def __init__(self, path, length, csLevel, eng=None):
        self.path = path
        self.length = length
        self.csLevel = csLevel
        self._eng = eng

    def ReadAt(self, size, off):
        """Returns (data, n).  Raises ChecksumError on a CRC mismatch and
        EOFError on a short read, as the reference's ReadAt returns them."""
        with open(self.path, "rb") as f:
            img = f.read()
        eng = self._eng or default_engine()
        rc, data, n, got, exp, seg = eng.cache_verify(img, self.length, _LEVEL[self.csLevel], off, size)
        if rc == E.ECRC:
            raise ChecksumError(got, exp, seg)
        if rc == E.EOF:
            raise EOFError("EOF")
        return data, n


def openCacheFile(name, length, level, eng=None):
    """disk_cache.go:1233-1253: the file size decides whether CRCs are present."""
    size = os.stat(name).st_size
    clen = ((length - 1) // csBlock + 1) * 4 if length > 0 else 4
    if size - length == 0:
        return CacheFile(name, length, CsNone, eng)
    if size - length == clen:
        return CacheFile(name, length, level, eng)
    raise ValueError("invalid file size %d, data length %d" % (size, length))
