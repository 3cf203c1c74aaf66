"""GPU parity of the fused modes the reference's call stacks need, and the
edges around them, against the oracle:

  CS-2  uploadStagingFile: cacheFile.ReadAt verify + Seal of the same bytes
        (pkg/chunk/cached_store.go:944-999)            -> seal + CRC_VERIFY
  CS-3  store.load -> cacheStore.cache: Open, then checksum() of the
        plaintext for the cache file (cached_store.go:673-748,
        disk_cache.go:389-422, :612-629)               -> open + CRC_GEN
  blocks above 4 MiB (--block-size up to 16 MiB, cmd/format.go:200-216)
  device-mode Open with a failed tag: nothing released (encrypt.go:215; Go's
        Open clears its in-place output)
  cacheFile.ReadAt (disk_cache.go:1255-1329): a seeded sweep of ranges,
        levels and corruptions, every output field equal to the oracle's
  the ciphers' length limits at the boundary (EINVAL, no launch)

Bit-exact everywhere: ciphertext, tags, CRC arrays, statuses, the first
failing segment and its got/expect values."""
import numpy as np
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ORC = {E.AES256GCM: orc.AES256GCM, E.CHACHA20P1305: orc.CHACHA20P1305}
ALGOS = [E.AES256GCM, E.CHACHA20P1305]


@pytest.fixture(scope="module", params=["ttable", "bitslice"])
def eng(request):
    e = E.Engine(0, E.CTX_BITSLICE if request.param == "bitslice" else 0)
    yield e
    e.close()


def _nseg(n):
    return max(1, -(-n // E.SEG))


class Batch:
    """Device buffers for a batch of blocks: src, dst and a CRC array each."""

    def __init__(self, eng, srcs, crcs=None):
        self.eng = eng
        self.lens = [len(s) for s in srcs]
        self.src, self.dst, self.crc = [], [], []
        for i, s in enumerate(srcs):
            n = len(s)
            a, b, c = eng.alloc(max(n, 16)), eng.alloc(max(n, 16)), eng.alloc(4 * _nseg(n))
            if n:
                a.upload(np.frombuffer(bytes(s), np.uint8))
            b.upload(np.full(max(n, 16), 0xA5, np.uint8))
            if crcs is not None:
                c.upload(np.frombuffer(bytes(crcs[i]), np.uint8))
            self.src.append(a), self.dst.append(b), self.crc.append(c)

    def specs(self, keys, tags=None):
        return [{"key": k, "nonce": nc, "src": self.src[i].ptr, "dst": self.dst[i].ptr, "len": self.lens[i],
                 "crc": self.crc[i].ptr, "tag": tags[i] if tags else None} for i, (k, nc) in enumerate(keys)]

    def out(self, i):
        return self.dst[i].download(self.lens[i]).tobytes()

    def crcs(self, i):
        return self.crc[i].download(4 * _nseg(self.lens[i])).tobytes()


def _items(seed, lens):
    keys = [orc.gen_key(seed, i) for i in range(len(lens))]
    ps = [orc.gen_block(seed, i, n) for i, n in enumerate(lens)]
    return keys, ps


# ---------------------------------------------------------------------------
# CS-2: seal + CRC_VERIFY (staging file re-read, then upload)


@pytest.mark.parametrize("algo", ALGOS)
def test_cs2_seal_with_crc_verify(eng, algo):
    lens = [0, 100, 32768, 32769, 5 * 32768 + 1000, (1 << 20) + 16, 4 << 20, (2 << 20) + 77]
    keys, ps = _items(41 + algo, lens)
    crcs = [bytearray(orc.checksum(p, hw=True)) for p in ps]
    srcs = [p.tobytes() for p in ps]
    # block 4: the stored CRC of segment 3 is corrupted; block 6: the staged
    # data of segment 100 is corrupted after its CRCs were written
    crcs[4][4 * 3 + 1] ^= 0x40
    bad6 = bytearray(srcs[6])
    bad6[100 * E.SEG + 12345] ^= 0x08
    srcs[6] = bytes(bad6)
    bt = Batch(eng, srcs, crcs)
    arr, n = eng.make_blocks(bt.specs(keys))
    eng.seal_batch(algo, arr, n, E.CRC_VERIFY, E.MEM_DEVICE)
    for i in range(n):
        b = arr[i]
        c, tag = orc.seal(ORC[algo], keys[i][0], keys[i][1], np.frombuffer(srcs[i], np.uint8), fast=True)
        # the transform itself always runs: C and tag are those of the bytes given
        assert bt.out(i) == c and bytes(b.tag) == tag, i
        assert bt.crcs(i) == bytes(crcs[i]), i  # VERIFY never writes the expected array
        if i == 4:
            assert (b.status, b.crc_bad_seg) == (E.ECRC, 3)
            assert b.crc_got == orc.crc32c(ps[4][3 * E.SEG:4 * E.SEG].tobytes())
            assert b.crc_expect == int.from_bytes(crcs[4][12:16], "big")
        elif i == 6:
            assert (b.status, b.crc_bad_seg) == (E.ECRC, 100)
            assert b.crc_got == orc.crc32c(srcs[6][100 * E.SEG:101 * E.SEG])
            assert b.crc_expect == int.from_bytes(crcs[6][400:404], "big")
        else:
            assert (b.status, b.crc_bad_seg) == (E.OK, -1), i


# ---------------------------------------------------------------------------
# CS-3: open + CRC_GEN of the plaintext (download -> cache write)


@pytest.mark.parametrize("algo", ALGOS)
def test_cs3_open_with_plaintext_crc_gen(eng, algo):
    lens = [0, 1, 4095, 32768, 65537, 1 << 20, (4 << 20) - 3, 3 << 20]
    keys, ps = _items(51 + algo, lens)
    sealed = [orc.seal(ORC[algo], k, nc, p, fast=True) for (k, nc), p in zip(keys, ps)]
    bt = Batch(eng, [c for c, _ in sealed])
    arr, n = eng.make_blocks(bt.specs(keys, [t for _, t in sealed]))
    eng.open_batch(algo, arr, n, E.CRC_GEN, E.MEM_DEVICE)
    for i in range(n):
        assert arr[i].status == E.OK, i
        assert bt.out(i) == ps[i].tobytes(), i
        assert bt.crcs(i) == orc.checksum(ps[i], hw=True), i  # the cache file's checksum() bytes


# ---------------------------------------------------------------------------
# blocks above 4 MiB


@pytest.mark.parametrize("algo", ALGOS)
def test_blocks_8_and_16_mib(eng, algo):
    lens = [8 << 20, 16 << 20, (16 << 20) - 3, (8 << 20) + 13]
    keys, ps = _items(61 + algo, lens)
    bt = Batch(eng, [p.tobytes() for p in ps])
    arr, n = eng.make_blocks(bt.specs(keys))
    eng.seal_batch(algo, arr, n, E.CRC_GEN, E.MEM_DEVICE)
    tags = []
    for i in range(n):
        c, tag = orc.seal(ORC[algo], keys[i][0], keys[i][1], ps[i], fast=True)
        assert arr[i].status == E.OK
        assert bytes(arr[i].tag) == tag, lens[i]
        assert bt.out(i) == c, lens[i]
        assert bt.crcs(i) == orc.checksum(ps[i], hw=True), lens[i]
        tags.append(tag)
    # and back: open + verify of the sealed bytes in place (dst == src)
    specs = [dict(s, src=bt.dst[i].ptr, dst=bt.dst[i].ptr, tag=tags[i]) for i, s in enumerate(bt.specs(keys))]
    oarr, n = eng.make_blocks(specs)
    eng.open_batch(algo, oarr, n, E.CRC_VERIFY, E.MEM_DEVICE)
    for i in range(n):
        assert (oarr[i].status, oarr[i].crc_bad_seg) == (E.OK, -1), lens[i]
        assert bt.out(i) == ps[i].tobytes(), lens[i]


# ---------------------------------------------------------------------------
# device-mode Open with a failed tag releases nothing


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("mode", [E.CRC_GEN, E.CRC_VERIFY, E.CRC_NONE])
def test_device_open_tag_failure_zeroes_output(eng, algo, mode):
    lens = [1000, 70000, 1 << 20, 5, 3 << 20]
    keys, ps = _items(71 + algo, lens)
    sealed = [orc.seal(ORC[algo], k, nc, p, fast=True) for (k, nc), p in zip(keys, ps)]
    tags = [t for _, t in sealed]
    bad = {1, 3, 4}
    for i in bad:
        tags[i] = bytes([tags[i][0] ^ 1]) + tags[i][1:]
    crcs = [orc.checksum(p, hw=True) for p in ps]
    bt = Batch(eng, [c for c, _ in sealed], crcs if mode == E.CRC_VERIFY else [b"\xee" * len(c) for c in crcs])
    arr, n = eng.make_blocks(bt.specs(keys, tags))
    eng.open_batch(algo, arr, n, mode, E.MEM_DEVICE)
    for i in range(n):
        if i in bad:
            assert arr[i].status == E.ETAG, i
            assert not any(bt.out(i)), i  # Go: the in-place output is cleared
            if mode == E.CRC_GEN:
                assert not any(bt.crcs(i)), i  # no CRC of unauthenticated plaintext either
        else:
            assert arr[i].status == E.OK, i
            assert bt.out(i) == ps[i].tobytes(), i
            if mode == E.CRC_GEN:
                assert bt.crcs(i) == crcs[i], i


@pytest.mark.parametrize("algo", ALGOS)
def test_device_open_in_place_tag_failure(eng, algo):
    """Open in place (dst == src, as encrypt.go:215 does): the ciphertext
    buffer ends up all zeros on a tag failure, the other block opens."""
    keys, ps = _items(81 + algo, [200000, 300000])
    sealed = [orc.seal(ORC[algo], k, nc, p, fast=True) for (k, nc), p in zip(keys, ps)]
    bt = Batch(eng, [c for c, _ in sealed])
    tags = [sealed[0][1], bytes(16)]
    specs = [dict(s, dst=s["src"]) for s in bt.specs(keys, tags)]
    arr, n = eng.make_blocks(specs)
    eng.open_batch(algo, arr, n, E.CRC_NONE, E.MEM_DEVICE)
    assert (arr[0].status, arr[1].status) == (E.OK, E.ETAG)
    assert bt.src[0].download(200000).tobytes() == ps[0].tobytes()
    assert not bt.src[1].download(300000).any()


# ---------------------------------------------------------------------------
# the ciphers' length limits (no buffer is touched: the arguments are refused
# before anything is launched)


def test_length_limits_refused_at_the_boundary(eng):
    fake = 1 << 40  # 16-B aligned, never dereferenced
    gcm_max = ((1 << 32) - 2) * 16
    cp_max = (1 << 38) - 64
    for algo, ln in ((E.AES256GCM, gcm_max + 1), (E.AES256GCM, gcm_max + 16), (E.AES256GCM, 1 << 36),
                     (E.CHACHA20P1305, cp_max + 1), (E.CHACHA20P1305, 1 << 38)):
        for op in (eng.L.jfsx_seal_batch, eng.L.jfsx_open_batch):
            arr, n = eng.make_blocks([{"key": bytes(32), "nonce": bytes(12), "src": fake, "dst": fake, "len": ln}])
            assert op(eng.ctx, algo, n, arr, E.CRC_NONE, E.MEM_DEVICE) == E.EINVAL, (algo, ln)


# ---------------------------------------------------------------------------
# cacheFile.ReadAt sweep vs the oracle


def _images():
    out = []
    for j, ln in enumerate([1, 1000, 32768, 32769, 100000, 5 * 32768, (1 << 20) + 5, 4 << 20]):
        d = orc.gen_block(91, j, ln)
        out.append((ln, d, orc.checksum(d)))
    return out


def test_cache_readat_sweep_matches_oracle(eng):
    """~500 seeded (image, level, off, size, corruption) cases, including
    unaligned ranges that widen (extend) or trim (shrink) to segment bounds,
    reads past the data into the CRC area, short reads, and no-CRC files."""
    rng = np.random.default_rng(20261016)
    imgs = _images()
    code = {0: 0, 1: E.ECRC, 2: E.EOF}
    seen = {}
    for case in range(520):
        ln, d, cs = imgs[case % len(imgs)]
        data = bytearray(d.tobytes())
        crc = bytearray(cs)
        kind = rng.integers(0, 4)
        if kind == 1:  # data corruption
            data[int(rng.integers(0, ln))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:  # CRC corruption
            crc[int(rng.integers(0, len(crc)))] ^= 1 << int(rng.integers(0, 8))
        img = bytes(data) + (b"" if kind == 3 else bytes(crc))  # kind 3: a file without CRCs
        level = int(rng.integers(0, 4))
        shape = rng.integers(0, 5)
        if shape == 0:
            off, size = 0, ln  # whole block (the VFS's aligned read)
        elif shape == 1:  # segment-aligned window
            s0 = int(rng.integers(0, _nseg(ln)))
            off, size = s0 * E.SEG, min(ln - s0 * E.SEG, E.SEG * int(rng.integers(1, 5)))
        elif shape == 2:  # unaligned inside the data
            off = int(rng.integers(0, ln))
            size = int(rng.integers(0, ln - off + 1))
        elif shape == 3:  # tail-anchored
            size = int(rng.integers(1, ln + 1))
            off = ln - size
        else:  # past the data: into the CRC area or beyond the file
            off = int(rng.integers(0, ln + 1))
            size = int(rng.integers(1, 2 * E.SEG))
        want = orc.cache_readat(img, ln, level, off, size)
        eff = orc.open_cache_file(len(img), ln, level)
        got = eng.cache_verify(img, ln, eff, off, size)
        rc, out, n = got[0], got[1], got[2]
        assert rc == code[want[0]], (case, ln, level, off, size, want[0], rc)
        assert n == want[2], (case, ln, level, off, size)
        assert out[:n] == want[1][:n], (case, ln, level, off, size)
        if want[0] == 1:
            assert got[3:] == want[3:], (case, ln, level, off, size)  # got, expect, bad_seg
        seen[(eff, want[0])] = seen.get((eff, want[0]), 0) + 1
    # the sweep reached every level with passes, and every checking level with failures
    for lv in range(4):
        assert seen.get((lv, 0)), seen
    for lv in (1, 2, 3):
        assert seen.get((lv, 1)), seen
    assert any(k[1] == 2 for k in seen), seen
