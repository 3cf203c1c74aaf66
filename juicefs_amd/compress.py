"""Mirror of pkg/compress/compress.go on the GPU engine, and the compress /
decompress steps of the chunk store's block upload and load.

  Compressor interface {Name, CompressBound, Compress, Decompress}  compress.go:30-36
  NewCompressor("lz4" | "zstd" | "none" | "")                       compress.go:38-50
  noOp (copy; "buffer too short: %d < %d")                         compress.go:52-70
  LZ4 (lz4.CompressDefault / lz4.DecompressSafe;
       "decompress an empty input")                                compress.go:104-125
  ZStandard.Decompress (zstd.Decompress; "buffer too short")       compress.go:93-102
  upload_block: CompressBound buffer, Compress, then Put           cached_store.go:371-392
  load_block: Get, Decompress into the block, "read %s fully"      cached_store.go:673-745

The LZ4 block codec runs on the HIP engine (jfsx_lz4_compress_batch /
jfsx_lz4_decompress_batch, jfsx_lz4.hip), bit-exact to the LZ4 C library the
reference binds; CompressBatch / DecompressBatch are the batched entry points
(one engine call per batch).  Zstandard decompression runs on the engine
too (jfsx_zstd_decompress_batch, jfsx_zstd.hip); Zstandard compression
(zstd.CompressLevel at level 1) stays with the Go host's libzstd, so
ZStandard.Compress raises NotImplementedError rather than run anywhere else.
"""
from . import engine as E
from .encrypt import default_engine


class CompressError(Exception):
    pass


class noOp:
    def Name(self):
        return "Noop"

    def CompressBound(self, n):
        return n

    def Compress(self, dst, src):
        if len(dst) < len(src):
            raise CompressError("buffer too short: %d < %d" % (len(dst), len(src)))
        dst[:len(src)] = src
        return len(src)

    def Decompress(self, dst, src):
        if len(dst) < len(src):
            raise CompressError("buffer too short: %d < %d" % (len(dst), len(src)))
        dst[:len(src)] = src
        return len(src)


class LZ4:
    """The "lz4" compressor.  Compress/Decompress follow Go's (dst, src) ->
    (n, error) shape: they return n and raise CompressError for the error."""

    def __init__(self, eng=None):
        self._eng = eng

    @property
    def eng(self):
        return self._eng or default_engine()

    def Name(self):
        return "LZ4"

    def CompressBound(self, n):
        return int(E.lz4_bound(n))

    def Compress(self, dst, src):
        out = self.CompressBatch([src])[0]
        if len(dst) < len(out):
            raise CompressError("buffer too short: %d < %d" % (len(dst), len(out)))
        dst[:len(out)] = out
        return len(out)

    def Decompress(self, dst, src):
        if len(src) == 0:
            raise CompressError("decompress an empty input")
        (st, out), = self.eng.lz4_decompress([src], [len(dst)])
        if st != E.OK:
            raise CompressError("lz4: malformed block")
        dst[:len(out)] = out
        return len(out)

    # -- batched: one GPU call for many blocks -----------------------------
    def CompressBatch(self, blocks):
        """blocks -> compressed bytes per block (LZ4_compress_default)."""
        return self.eng.lz4_compress(blocks)

    def DecompressBatch(self, blobs, sizes):
        """(compressed blob, destination size) per block -> decoded bytes,
        or a CompressError instance for a block that does not decode."""
        out = []
        todo = [i for i, b in enumerate(blobs) if len(b)]
        res = dict(zip(todo, self.eng.lz4_decompress([blobs[i] for i in todo], [sizes[i] for i in todo])))
        for i in range(len(blobs)):
            if i not in res:
                out.append(CompressError("decompress an empty input"))
            else:
                st, d = res[i]
                out.append(d if st == E.OK else CompressError("lz4: malformed block"))
        return out


class ZStandard:
    """The "zstd" compressor (DataDog/zstd v1.5.0, level 1).  Decompress runs on
    the engine; Compress is the Go host's libzstd call."""

    def __init__(self, level=1, eng=None):
        self.level = level
        self._eng = eng

    @property
    def eng(self):
        return self._eng or default_engine()

    def Name(self):
        return "Zstd"

    def CompressBound(self, n):
        # ZSTD_COMPRESSBOUND(n)
        return n + (n >> 8) + (((128 << 10) - n) >> 11 if n < (128 << 10) else 0)

    def Compress(self, dst, src):
        raise NotImplementedError("zstd compression runs in the Go host's libzstd, not in the jfsx engine")

    def Decompress(self, dst, src):
        d = self.DecompressBatch([src], [len(dst)])[0]
        if isinstance(d, Exception):
            raise d
        dst[:len(d)] = d
        return len(d)

    def DecompressBatch(self, blobs, sizes):
        """(frames, destination size) per block -> decoded bytes, or a
        CompressError: "buffer too short: %d < %d" where the frames decode but
        not into the destination (zstd.Decompress then returns a larger
        buffer, compress.go:98-100), else the decoder's error."""
        res = self.eng.zstd_decompress(blobs, sizes)
        out, retry = [], []
        for i, (st, d) in enumerate(res):
            out.append(d if st == E.OK else None)
            if st != E.OK:
                retry.append(i)
        if retry:
            big = self.eng.zstd_decompress([blobs[i] for i in retry],
                                           [max(4 * sizes[i], 1 << 20) for i in retry])
            for i, (st, d) in zip(retry, big):
                out[i] = CompressError("buffer too short: %d < %d" % (sizes[i], len(d)) if st == E.OK
                                       else "zstd: corrupted frame")
        return out


def NewCompressor(algr, eng=None):
    """compress.go:38-50: None for an unknown name."""
    algr = algr.lower()
    if algr == "zstd":
        return ZStandard(1, eng)
    if algr == "lz4":
        return LZ4(eng)
    if algr in ("none", ""):
        return noOp()
    return None


# ---------------------------------------------------------------------------
# chunk-store steps around the codec (cached_store.go)
# ---------------------------------------------------------------------------
def upload_blocks(store, keys, blocks, compressor):
    """cachedStore.upload for a batch of blocks: compress each (into a
    CompressBound-sized buffer when the bound exceeds the block), then Put."""
    if isinstance(compressor, LZ4):
        outs = compressor.CompressBatch(blocks)
    else:
        outs = []
        for b in blocks:
            buf = bytearray(max(compressor.CompressBound(len(b)), len(b)))
            n = compressor.Compress(buf, bytes(b))
            outs.append(bytes(buf[:n]))
    for k, o in zip(keys, outs):
        store.Put(k, o)
    return outs


def load_blocks(store, keys, lengths, compressor):
    """cachedStore.load for a batch: Get each object, decompress into a page of
    the block's length; a short result is "read %s fully: %s (%d < %d)"."""
    objs = [store.Get(k, 0, -1) for k in keys]
    compressed = [compressor.CompressBound(n) > n for n in lengths]
    if isinstance(compressor, (LZ4, ZStandard)):
        dec = compressor.DecompressBatch(objs, lengths)
    else:
        dec = []
        for o, n in zip(objs, lengths):
            page = bytearray(n)
            try:
                m = compressor.Decompress(page, o)
                dec.append(bytes(page[:m]))
            except CompressError as e:
                dec.append(e)
    out = []
    for k, o, n, c, d in zip(keys, objs, lengths, compressed, dec):
        if not c:
            d = o[:n]
        if isinstance(d, Exception):
            raise CompressError("read %s fully: %s (%d < %d)" % (k, d, 0, n))
        if len(d) < n:
            raise CompressError("read %s fully: %s (%d < %d)" % (k, None, len(d), n))
        out.append(d)
    return out
