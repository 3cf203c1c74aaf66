"""The reference's own compressor contract, testCompress
(pkg/compress/compress_test.go:25-76), for "none", "lz4" and "zstd" through
the compress.go mirror (juicefs_amd/compress.py) on the engine:

  * Compress into a 1-byte dst fails when len(src) > 1  (:29-33)
  * a CompressBound-sized dst compresses                 (:35-39)
  * Decompress into a 1-byte dst fails when len(src) > 1 (:40-44)
  * the decompressed bytes equal src                     (:46-53)
  * all of the above for src = Name() and src = nil      (:56-57)
  * Decompress of an empty input fails when CompressBound(0) > 0 (:59-64)

"none" runs on the host (noOp is a copy); "lz4" and "zstd" need the GPU."""
import pytest

from juicefs_amd import compress as C


def check_compressor(c):
    def test_it(src):
        if len(src) > 1:
            with pytest.raises(C.CompressError):
                c.Compress(bytearray(1), src)
        dst = bytearray(c.CompressBound(len(src)))
        n = c.Compress(dst, src)
        if len(src) > 1:
            with pytest.raises(C.CompressError):
                c.Decompress(bytearray(1), bytes(dst[:n]))
        src2 = bytearray(len(src))
        m = c.Decompress(src2, bytes(dst[:n]))
        assert bytes(src2[:m]) == bytes(src), (c.Name(), src)

    test_it(c.Name().encode())
    test_it(b"")
    if c.CompressBound(0) > 0:
        with pytest.raises(C.CompressError):
            c.Decompress(bytearray(100), b"")


def test_uncompressed():
    check_compressor(C.NewCompressor("none"))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["lz4", "zstd"])
def test_engine_compressors(algo):
    from juicefs_amd import engine as E
    eng = E.Engine(0)
    try:
        check_compressor(C.NewCompressor(algo, eng))
    finally:
        eng.close()


@pytest.mark.gpu
def test_error_texts():
    """The errors the reference's callers see: LZ4's "decompress an empty
    input" (compress.go:121-123), zstd's empty-slice error, and
    "buffer too short: %d < %d" (compress.go:87-89, :98-100)."""
    from juicefs_amd import engine as E
    eng = E.Engine(0)
    try:
        lz, zs = C.NewCompressor("lz4", eng), C.NewCompressor("zstd", eng)
        with pytest.raises(C.CompressError, match="decompress an empty input"):
            lz.Decompress(bytearray(10), b"")
        with pytest.raises(C.CompressError, match="Bytes slice is empty"):
            zs.Decompress(bytearray(10), b"")
        with pytest.raises(C.CompressError, match=r"buffer too short: 1 < %d" % zs.CompressBound(4)):
            zs.Compress(bytearray(1), b"Zstd")
        dst = bytearray(zs.CompressBound(4))
        n = zs.Compress(dst, b"Zstd")
        with pytest.raises(C.CompressError, match=r"buffer too short: 1 < 4"):
            zs.Decompress(bytearray(1), bytes(dst[:n]))
    finally:
        eng.close()
