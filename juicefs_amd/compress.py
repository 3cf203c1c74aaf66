"""Mirror of pkg/compress/compress.go on the GPU engine, and the compress /
decompress steps of the chunk store's block upload and load.

  Compressor interface {Name, CompressBound, Compress, Decompress}  compress.go:30-36
  NewCompressor("lz4" | "zstd" | "none" | "")                       compress.go:38-50
  noOp (copy; "buffer too short: %d < %d")                         compress.go:52-70
  LZ4 (lz4.CompressDefault / lz4.DecompressSafe;
       "decompress an empty input")                                compress.go:104-125
  ZStandard.Compress (zstd.CompressLevel(dst, src, 1))             compress.go:82-91
  ZStandard.Decompress (zstd.Decompress; "buffer too short")       compress.go:93-102
  upload_block: CompressBound buffer, Compress, then Put           cached_store.go:371-392
  load_block: Get, Decompress into the block, "read %s fully"      cached_store.go:673-745

The LZ4 block codec runs on the HIP engine (jfsx_lz4_compress_batch /
jfsx_lz4_decompress_batch, jfsx_lz4.hip), bit-exact to the LZ4 C library the
reference binds; CompressBatch / DecompressBatch are the batched entry points
(one engine call per batch).  Zstandard runs on the engine both ways:
jfsx_zstd_compress_batch (jfsx_zstdc.hip) writes the zstd library's level-1
frames byte for byte, jfsx_zstd_decompress_batch (jfsx_zstd.hip) decodes as
ZSTD_decompress.
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
    """The "zstd" compressor (DataDog/zstd v1.5.0, level 1): Compress and
    Decompress both run on the engine.  jfsx_zstd_compress_batch is bit-exact
    to the system libzstd 1.4.8's ZSTD_compress(level 1); byte parity with the
    v1.5.0 library the reference links is unpinned (its vendored C is not in
    the reference tree), but every frame is valid zstd and reads back through
    this Decompress and through libzstd's ZSTD_decompress alike.
    jfsx_zstd_decompress_batch decodes as ZSTD_decompress."""

    def __init__(self, level=1, eng=None):
        if level != 1:
            raise ValueError("the engine implements zstd level 1 (compress.go:28 ZSTD_LEVEL)")
        self.level = level
        self._eng = eng

    @property
    def eng(self):
        return self._eng or default_engine()

    def Name(self):
        return "Zstd"

    def CompressBound(self, n):
        return int(E.zstd_bound(n))  # ZSTD_COMPRESSBOUND(n)

    def Compress(self, dst, src):
        """compress.go:82-91: zstd.CompressLevel allocates a new buffer when
        cap(dst) < CompressBound(len(src)), and Compress reports that as
        "buffer too short: %d < %d" (cap(dst), cap(d))."""
        bound = self.CompressBound(len(src))
        if len(dst) < bound:
            raise CompressError("buffer too short: %d < %d" % (len(dst), bound))
        out = self.CompressBatch([src])[0]
        dst[:len(out)] = out
        return len(out)

    def Decompress(self, dst, src):
        d = self.DecompressBatch([src], [len(dst)])[0]
        if isinstance(d, Exception):
            raise d
        dst[:len(d)] = d
        return len(d)

    # -- batched: one GPU call for many blocks -----------------------------
    def CompressBatch(self, blocks):
        """blocks -> one level-1 frame per block (ZSTD_compress(level 1))."""
        return self.eng.zstd_compress(blocks)

    def DecompressBatch(self, blobs, sizes):
        """(frames, destination size) per block -> decoded bytes, or a
        CompressError:
          * an empty input: DataDog's ErrEmptySlice ("Bytes slice is empty");
          * frames that decode, but not into the destination: zstd.Decompress
            returns a larger buffer, which compress.go:98-100 reports as
            "buffer too short: %d < %d" (len(dst), decoded size);
          * anything else the decoder rejects: "zstd: corrupted frame"."""
        out = [None] * len(blobs)
        todo = []
        for i, b in enumerate(blobs):
            if len(b) == 0:
                out[i] = CompressError("Bytes slice is empty")
            else:
                todo.append(i)
        res = self.eng.zstd_decompress([blobs[i] for i in todo], [sizes[i] for i in todo]) if todo else []
        short = []
        for i, (st, d) in zip(todo, res):
            if st == E.OK:
                out[i] = d
            elif st == E.EDSTSIZE:
                short.append(i)
            else:
                out[i] = CompressError("zstd: corrupted frame")
        # the decoded size of a frame that does not fit: its content size
        # field when it has one, else doubling capacities (up to 2^31 - 1)
        caps = {i: max(_frame_content_size(blobs[i]) or 0, 2 * sizes[i], 1 << 16) for i in short}
        while short:
            res = self.eng.zstd_decompress([blobs[i] for i in short], [min(caps[i], (1 << 31) - 1) for i in short])
            again = []
            for i, (st, d) in zip(short, res):
                if st == E.OK:
                    out[i] = CompressError("buffer too short: %d < %d" % (sizes[i], len(d)))
                elif st == E.EDSTSIZE and caps[i] < (1 << 31) - 1:
                    caps[i] *= 2
                    again.append(i)
                else:
                    out[i] = CompressError("zstd: corrupted frame")
            short = again
        return out


def _frame_content_size(b):
    """Frame_Content_Size of the first frame's header (RFC 8878 3.1.1.1), or
    None when absent or unreadable."""
    b = bytes(b[:18])
    if len(b) < 6 or b[:4] != b"\x28\xb5\x2f\xfd":
        return None
    fhd = b[4]
    single, fcs_id, did = (fhd >> 5) & 1, fhd >> 6, fhd & 3
    pos = 5 + (0 if single else 1) + (0, 1, 2, 4)[did]
    size = (1 if single else 0, 2, 4, 8)[fcs_id]
    if size == 0 or len(b) < pos + size:
        return None
    v = int.from_bytes(b[pos:pos + size], "little")
    return v + 256 if size == 2 else v


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
    if isinstance(compressor, (LZ4, ZStandard)):
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
