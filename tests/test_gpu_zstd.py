"""GPU Zstandard decompression (jfsx_zstd_decompress_batch, jfsx_zstd.hip)
against the system zstd library: decoded bytes of frames at several levels,
with checksums, concatenated / skippable frames, device-resident unaligned
buffers, and accept/reject of malformed frames as ZSTD_decompress."""
import numpy as np
import pytest

from juicefs_amd import engine as E
from tests import lz4_data, zstd_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def test_levels_and_checksums(eng):
    srcs, frames = [], []
    for kind in lz4_data.KINDS:
        for n in (0, 1, 100, 4096, 100003, 1 << 20):
            for level, ck in ((1, False), (3, True), (-3, False), (9, True)):
                src = lz4_data.sample(kind, n, seed=n + level + 10)
                srcs.append(src)
                frames.append(zstd_lib.compress(src, level, ck))
    got = eng.zstd_decompress(frames, [len(s) for s in srcs])
    for i, (src, (st, d)) in enumerate(zip(srcs, got)):
        assert st == E.OK and d == src, i


@pytest.mark.parametrize("kind", ["text", "random", "runs"])
def test_4mib_blocks(eng, kind):
    srcs = [lz4_data.sample(kind, 4 << 20, seed=s) for s in range(3)]
    got = eng.zstd_decompress([zstd_lib.compress(s, 1) for s in srcs], [4 << 20] * 3)
    assert all(st == E.OK and d == s for s, (st, d) in zip(srcs, got))


def test_concatenated_skippable_and_edges(eng):
    a = lz4_data.sample("text", 70000, seed=1)
    b = lz4_data.sample("runs", 5000, seed=2)
    fr = zstd_lib.skippable(b"juicefs") + zstd_lib.compress(a) + zstd_lib.skippable(b"", 15) + \
        zstd_lib.compress(b, 3, True)
    got = eng.zstd_decompress([fr, b"", fr + b"\x28\xb5", zstd_lib.compress(a)], [len(a) + len(b), 10, 10**6,
                                                                                  len(a) - 1])
    assert got[0] == (E.OK, a + b)
    assert got[1] == (E.OK, b"")
    assert got[2][0] == E.EFORMAT and got[3][0] == E.EDSTSIZE


def test_device_batch_unaligned(eng):
    rng = np.random.default_rng(5)
    n = 24
    lens = [int(x) for x in rng.integers(0, 300000, n)]
    srcs = [lz4_data.sample(lz4_data.KINDS[i % 6], lens[i], seed=50 + i) for i in range(n)]
    frames = [zstd_lib.compress(s, 1 + (i % 3)) for i, s in enumerate(srcs)]
    inb = eng.alloc(sum(len(f) + 8 for f in frames))
    outb = eng.alloc(sum(L + 8 for L in lens))
    specs, io, oo = [], 0, 0
    for i, f in enumerate(frames):
        a, c = io + (i % 4), oo + (i % 3)
        inb.upload(np.frombuffer(f, np.uint8), a)
        specs.append((inb.ptr + a, len(f), outb.ptr + c, lens[i]))
        io += len(f) + 8
        oo += lens[i] + 8
    arr, m = eng.make_zblocks(specs)
    eng.zstd_decompress_batch(arr, m, E.MEM_DEVICE)
    for i in range(n):
        assert arr[i].status == E.OK and arr[i].out_len == lens[i]
        assert outb.download(lens[i], specs[i][2] - outb.ptr).tobytes() == srcs[i]


def test_malformed_agrees_with_library(eng):
    rng = np.random.default_rng(3)
    frames, caps, ref = [], [], []
    for trial in range(600):
        kind = lz4_data.KINDS[trial % 6]
        n = int(rng.choice([50, 700, 5000, 70000]))
        fr = bytearray(zstd_lib.compress(lz4_data.sample(kind, n, seed=trial), int(rng.choice([1, 3, -1])),
                                         trial % 3 == 0))
        m = trial % 3
        if m == 0 and len(fr) > 1:
            fr = fr[:int(rng.integers(0, len(fr)))]
        elif m == 1:
            i = int(rng.integers(0, len(fr)))
            fr[i] ^= 1 << int(rng.integers(0, 8))
        else:
            fr[int(rng.integers(0, len(fr)))] = int(rng.integers(0, 256))
        cap = n if rng.random() < 0.8 else int(rng.integers(0, n + 10))
        frames.append(bytes(fr))
        caps.append(cap)
        ref.append(zstd_lib.decompress(bytes(fr), cap))
    got = eng.zstd_decompress(frames, caps)
    rejects = 0
    for (st, d), (rc, r) in zip(got, ref):
        if rc < 0:
            rejects += 1
            assert st in (E.EFORMAT, E.EDSTSIZE)
        else:
            assert st == E.OK and d == r
    assert rejects > 200


def test_mirror_decompress_and_load_blocks(eng):
    """compress.go:93-102 (ZStandard.Decompress) and cachedStore.load's
    decompress step (cached_store.go:680-745) through the engine."""
    from juicefs_amd import compress as C
    z = C.NewCompressor("zstd", eng)
    src = lz4_data.sample("text", 300000, seed=9)
    fr = zstd_lib.compress(src)
    dst = bytearray(len(src))
    assert z.Decompress(dst, fr) == len(src) and bytes(dst) == src
    with pytest.raises(C.CompressError, match="buffer too short: %d < %d" % (len(src) - 1, len(src))):
        z.Decompress(bytearray(len(src) - 1), fr)
    with pytest.raises(C.CompressError, match="zstd: corrupted frame"):
        z.Decompress(bytearray(len(src)), fr[:len(fr) // 2])

    class Store:
        def __init__(self):
            self.d = {}

        def Put(self, k, v):
            self.d[k] = bytes(v)

        def Get(self, k, off, lim):
            return self.d[k]
    st = Store()
    blocks = [lz4_data.sample(k, 4 << 20, seed=i) for i, k in enumerate(("text", "runs", "random"))]
    keys = ["chunks/0/0/%d_0_%d" % (i, len(b)) for i, b in enumerate(blocks)]
    for k, b in zip(keys, blocks):
        st.Put(k, zstd_lib.compress(b))
    assert C.load_blocks(st, keys, [len(b) for b in blocks], z) == blocks


def test_per_block_calls_through_the_aggregator_and_mctx():
    """cachedStore.load calls Decompress once per block from many goroutines:
    through jfsx_agg they become batches; a multi-device context splits a
    host batch over its devices (one here)."""
    import threading
    eng = E.Engine(0)
    try:
        T = 24
        srcs = [lz4_data.sample(lz4_data.KINDS[i % 6], 50000 + 997 * i, seed=i) for i in range(T)]
        frames = [np.frombuffer(zstd_lib.compress(s, 1 + i % 3), np.uint8) for i, s in enumerate(srcs)]
        backs = [np.zeros(len(s), np.uint8) for s in srcs]
        zd = [E.jfsx_zblk() for _ in range(T)]
        with E.Aggregator(eng, window_us=3000) as agg:
            def worker(i):
                d = zd[i]
                d.src, d.src_len, d.dst, d.dst_cap = frames[i].ctypes.data, frames[i].size, backs[i].ctypes.data, \
                    backs[i].size
                agg.zstd_decompress(d)
            th = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            calls, batches, blocks = agg.stats()
        for i in range(T):
            assert zd[i].status == E.OK and zd[i].out_len == len(srcs[i]) and backs[i].tobytes() == srcs[i]
        assert calls == T and batches < calls
    finally:
        eng.close()
    m = E.MultiEngine(0)
    try:
        outs = [np.zeros(len(s), np.uint8) for s in srcs]
        arr, n = E.Engine.make_zblocks((f.ctypes.data, f.size, o.ctypes.data, o.size) for f, o in zip(frames, outs))
        m.zstd_decompress_batch(arr, n)
        assert all(arr[i].status == E.OK and outs[i].tobytes() == srcs[i] for i in range(T))
    finally:
        m.close()


def test_log12_huffman_table(eng):
    """Log-12 Huffman tables (read from global scratch, not LDS), one and
    four streams, beside log-11 frames in the same batch."""
    rng = np.random.default_rng(12)
    frames, want = [], []
    for four in (False, True):
        for n in (4, 37, 200, 255):
            syms = bytes(int(x) for x in rng.integers(0, 14, n))
            frames.append(zstd_lib.huf12_frame(list(syms), four))
            want.append(syms)
            src = lz4_data.sample("text", 5000 + n, seed=n)
            frames.append(zstd_lib.compress(src, 1))
            want.append(src)
    got = eng.zstd_decompress(frames, [1000 if len(w) < 256 else len(w) for w in want])
    for i, (w, (st, d)) in enumerate(zip(want, got)):
        assert st == E.OK and d == w, i


def test_checksum_tail_reads_inside_output(eng):
    # the XXH64 tail read 8 bytes per step past the decoded end.
    # Checksummed frames whose lengths are not multiples of 8, each decoded
    # into its own device buffer of exactly the decoded size.
    for n in (1, 3, 7, 9, 13, 31, 33, 1001, 4099, 65537, 131075):
        src = lz4_data.sample("text", n, seed=n)
        fr = zstd_lib.compress(src, 1, True)
        inb = eng.alloc(len(fr))
        inb.upload(np.frombuffer(fr, np.uint8))
        outb = eng.alloc(n)
        arr, k = eng.make_zblocks([(inb.ptr, len(fr), outb.ptr, n)])
        eng.zstd_decompress_batch(arr, k, E.MEM_DEVICE)
        assert arr[0].status == E.OK and arr[0].out_len == n, n
        assert outb.download(n).tobytes() == src, n
        inb.free()
        outb.free()


def test_block_parallel_decoder_takes_level1_frames(eng):
    """The block-parallel decoder (jfsx_zstd2.h) takes every one-frame object
    of up to 64 blocks without handing it to the serial decoder, across data
    kinds, sizes, levels and content checksums; the bytes equal the input."""
    srcs, frames, what = [], [], []
    for kind in lz4_data.KINDS:
        for n in (9, 4096, 131071, 131072, 131073, 1 << 20, (4 << 20) + 17):
            for level, ck in ((1, False), (1, True), (3, False), (9, False)):
                src = lz4_data.sample(kind, n, seed=7 * n + level)
                srcs.append(src)
                frames.append(zstd_lib.compress(src, level, ck))
                what.append((kind, n, level, ck))
    eng.metrics(reset=True)
    got = eng.zstd_decompress(frames, [len(s) for s in srcs])
    m = eng.metrics()
    for i, (src, (st, d)) in enumerate(zip(srcs, got)):
        assert st == E.OK and d == src, i
    serial = [(w, r) for w, r in zip(what, eng.zstd_serial_reasons) if r]
    assert m["zstdd_blocks"] == len(frames) and m["zstd_serial"] == 0, serial
    assert m["zstdd_out"] == sum(len(s) for s in srcs)


def test_block_parallel_decoder_hands_off_other_shapes(eng):
    """Concatenated frames, skippable frames and frames of more than 64 blocks
    go to the serial decoder (counted in zstd_serial) and still decode."""
    a = lz4_data.sample("text", 300000, seed=3)
    big = lz4_data.sample("text", 9 << 20, seed=4)
    fr = [zstd_lib.compress(a) + zstd_lib.compress(a), zstd_lib.skippable(b"x") + zstd_lib.compress(a),
          zstd_lib.compress(big)]
    eng.metrics(reset=True)
    got = eng.zstd_decompress(fr, [2 * len(a), len(a), len(big)])
    assert got[0] == (E.OK, a + a) and got[1] == (E.OK, a) and got[2] == (E.OK, big)
    assert eng.metrics()["zstd_serial"] == 3


def test_block_parallel_matches_across_blocks(eng):
    """Matches and repeat offsets that cross 128 KiB block boundaries: a
    period longer than a block, short periods (overlapping copies), and runs
    of one byte; level 1 and 19-style long matches (level 9)."""
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, 200000, dtype=np.uint8).tobytes()
    srcs = [(base * 6)[:1100000], (b"abcdefg" * 300000)[:2000000], bytes(1500000),
            (rng.integers(0, 4, 3 << 20, dtype=np.uint8) + 65).astype(np.uint8).tobytes(),
            b"".join(base[i:i + 5000] for i in range(0, 190000, 3700)) * 4]
    frames = [zstd_lib.compress(s, lvl) for s in srcs for lvl in (1, 9)]
    exp = [s for s in srcs for _ in (1, 9)]
    eng.metrics(reset=True)
    got = eng.zstd_decompress(frames, [len(s) for s in exp])
    for i, (s, (st, d)) in enumerate(zip(exp, got)):
        assert st == E.OK and d == s, i
    assert eng.metrics()["zstd_serial"] == 0


def test_arena_budget_caps_the_decoder_waves(monkeypatch):
    """The block-parallel decoder's arenas (13.8 MiB per wave) are capped by
    the context's budget (JFSX_ZSTD_ARENA_MB, read at context open): with room
    for 2 arenas, or for less than one (one wave then), a 20-frame batch still
    decodes to the same bytes on the block-parallel kernel."""
    srcs = [lz4_data.sample(lz4_data.KINDS[i % 6], 200000 + 977 * i, seed=300 + i) for i in range(20)]
    frames = [zstd_lib.compress(s, 1) for s in srcs]
    for mb in ("30", "1"):
        monkeypatch.setenv("JFSX_ZSTD_ARENA_MB", mb)
        e = E.Engine(0)
        try:
            got = e.zstd_decompress(frames, [len(s) for s in srcs])
            assert all(st == E.OK and d == s for s, (st, d) in zip(srcs, got)), mb
        finally:
            e.close()
