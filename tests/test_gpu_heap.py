"""GPU parity of host calls on ordinary pageable memory (the reference's
Go-heap slices: io.ReadAll's result and the fresh object buffer of
dataEncryptor.Encrypt, pkg/object/encrypt.go:183, :258; cache pages,
pkg/chunk/page.go:42-50), which the engine stages through its own pinned
bounce buffers; of JFSX_CRC_BOTH (plaintext checksum() and ciphertext segment
CRCs from one call, cached_store.go:439-451 + s3.go:173-176); of the
data_encrypt_ex / data_decrypt_ex calls; and of checksum() / the ReadAt verify
through the host pipeline (disk_cache.go:1218-1231, :1255-1329).  Every
result is compared with the oracle."""
import ctypes
import threading

import numpy as np
import pytest

from juicefs_amd import engine as E
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ORC = {E.AES256GCM: orc.AES256GCM, E.CHACHA20P1305: orc.CHACHA20P1305}
LENS = [0, 1, 15, 17, 4095, 32767, 32768, 32769, 100003, 1 << 20, (4 << 20) - 3, 4 << 20]


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def run_threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: B902 -- re-raised below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def heap(nbytes, skew=0):
    """a pageable numpy buffer whose data starts `skew` bytes past a 64-B
    boundary (Go slices start anywhere)"""
    raw = np.empty(nbytes + 64 + skew, np.uint8)
    o = (-raw.ctypes.data) % 64 + skew
    return raw[o:o + nbytes]


def nseg(n):
    return max(1, -(-n // E.SEG))


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_heap_seal_open_batch_matches_oracle(eng, algo):
    """A host batch of pageable blocks at odd offsets (one in place, one
    pinned beside them), sealed with CRC_GEN and opened with CRC_VERIFY."""
    specs, keep = [], []
    pin = eng.alloc_pinned(2 << 20)
    try:
        for i, n in enumerate(LENS):
            p = orc.gen_block(41, i, n)
            src = heap(max(n, 1), skew=i % 7)
            src[:n] = p
            inplace = i == 3
            dst = src if inplace else heap(max(n, 1), skew=(3 * i) % 11)
            crc = heap(4 * nseg(n), skew=i % 3)
            key, nonce = orc.gen_key(41, i)
            specs.append({"key": key, "nonce": nonce, "src": src.ctypes.data, "dst": dst.ctypes.data, "len": n,
                          "crc": crc.ctypes.data})
            keep.append((p, key, nonce, src, dst, crc))
        # one pinned block in the same batch
        pn = 1 << 20
        pp = orc.gen_block(41, 99, pn)
        ctypes.memmove(pin, pp.ctypes.data, pn)
        pcrc = np.zeros(4 * nseg(pn), np.uint8)
        kp, np_ = orc.gen_key(41, 99)
        specs.append({"key": kp, "nonce": np_, "src": pin, "dst": pin + pn, "len": pn, "crc": pcrc.ctypes.data})
        arr, cnt = eng.make_blocks(specs)
        eng.seal_batch(algo, arr, cnt, E.CRC_GEN, E.MEM_HOST)
        for i, (p, key, nonce, src, dst, crc) in enumerate(keep):
            c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
            assert arr[i].status == E.OK and bytes(arr[i].tag) == tag, i
            assert dst[:len(p)].tobytes() == c, i
            assert crc.tobytes() == orc.checksum(p), i
        c, tag = orc.seal(ORC[algo], kp, np_, pp, fast=True)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * pn).from_address(pin + pn)).tobytes()
        assert bytes(arr[cnt - 1].tag) == tag and got == c and pcrc.tobytes() == orc.checksum(pp)
        # open every ciphertext back into fresh pageable buffers, CRC verify
        ospecs, outs = [], []
        for i, (p, key, nonce, src, dst, crc) in enumerate(keep):
            o = heap(max(len(p), 1), skew=5)
            outs.append(o)
            ospecs.append({"key": key, "nonce": nonce, "src": dst.ctypes.data, "dst": o.ctypes.data,
                           "len": len(p), "crc": crc.ctypes.data, "tag": bytes(arr[i].tag)})
        oarr, ocnt = eng.make_blocks(ospecs)
        eng.open_batch(algo, oarr, ocnt, E.CRC_VERIFY, E.MEM_HOST)
        for i, (p, *_rest) in enumerate(keep):
            assert oarr[i].status == E.OK, i
            assert outs[i][:len(p)].tobytes() == p.tobytes(), i
    finally:
        eng.free_pinned(pin)


def test_heap_open_failed_tag_releases_nothing(eng):
    n = 300000
    p = orc.gen_block(43, 1, n)
    key, nonce = orc.gen_key(43, 1)
    c, tag = orc.seal(orc.AES256GCM, key, nonce, p, fast=True)
    src = heap(n, skew=3)
    src[:] = np.frombuffer(c, np.uint8)
    out = heap(n, skew=1)
    out[:] = 0x77
    crc = heap(4 * nseg(n))
    crc[:] = 0x55
    bad = bytes([tag[0] ^ 1]) + tag[1:]
    arr, cnt = eng.make_blocks([{"key": key, "nonce": nonce, "src": src.ctypes.data, "dst": out.ctypes.data,
                                 "len": n, "crc": crc.ctypes.data, "tag": bad}])
    eng.open_batch(orc.AES256GCM, arr, cnt, E.CRC_GEN, E.MEM_HOST)
    assert arr[0].status == E.ETAG
    assert not out.any() and not crc.any()


def test_heap_large_batch_bounce_window(eng):
    """A 320 MiB pageable host batch: groups >= 32 MiB (copied by helper
    threads), more groups in flight than the bounce window keeps."""
    nb, n = 80, 4 << 20
    src = heap(nb * n)
    dst = heap(nb * n, skew=16)
    crcs = np.zeros((nb, 4 * nseg(n)), np.uint8)
    specs = []
    for b in range(nb):
        src[b * n:(b + 1) * n] = orc.gen_block(47, b, n)
        key, nonce = orc.gen_key(47, b)
        specs.append({"key": key, "nonce": nonce, "src": src.ctypes.data + b * n, "dst": dst.ctypes.data + b * n,
                      "len": n, "crc": crcs[b].ctypes.data})
    arr, cnt = eng.make_blocks(specs)
    eng.seal_batch(E.AES256GCM, arr, cnt, E.CRC_GEN, E.MEM_HOST)
    etags, ecrcs, _ = orc.expect_batch(orc.AES256GCM, 8, [n] * nb, 47, 0, 4 * nseg(n))
    for b in range(nb):
        assert arr[b].status == E.OK and bytes(arr[b].tag) == etags[b].tobytes(), b
    assert (crcs == ecrcs).all()
    for b in (0, 37, nb - 1):
        key, nonce = orc.gen_key(47, b)
        c, _ = orc.seal(orc.AES256GCM, key, nonce, src[b * n:(b + 1) * n], fast=True)
        assert dst[b * n:(b + 1) * n].tobytes() == c, b


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
@pytest.mark.parametrize("mem", [E.MEM_DEVICE, E.MEM_HOST])
def test_crc_both_seal_and_open(eng, algo, mem):
    """JFSX_CRC_BOTH: crc = checksum(plaintext) || segment CRCs of C, for
    Seal and for an in-place Open; a failed tag zeroes the plaintext half
    only."""
    lens = [0, 17, 32768, 100003, 1 << 20, (4 << 20) - 3]
    bufs, specs = [], []
    for i, n in enumerate(lens):
        p = orc.gen_block(53, i, n)
        key, nonce = orc.gen_key(53, i)
        cw = 8 * nseg(n)
        if mem == E.MEM_DEVICE:
            src, dst, crc = eng.alloc(max(n, 16)), eng.alloc(max(n, 16)), eng.alloc(cw)
            if n:
                src.upload(p)
            ptrs = (src.ptr, dst.ptr, crc.ptr)
        else:
            src, dst, crc = heap(max(n, 1), 2), heap(max(n, 1), 9), np.full(cw, 0xEE, np.uint8)
            src[:n] = p
            ptrs = (src.ctypes.data, dst.ctypes.data, crc.ctypes.data)
        bufs.append((p, key, nonce, src, dst, crc))
        specs.append({"key": key, "nonce": nonce, "src": ptrs[0], "dst": ptrs[1], "len": n, "crc": ptrs[2]})

    def rd(buf, nbytes):
        if not nbytes:
            return b""
        return buf.download(nbytes).tobytes() if mem == E.MEM_DEVICE else buf[:nbytes].tobytes()
    arr, cnt = eng.make_blocks(specs)
    eng.seal_batch(algo, arr, cnt, E.CRC_GEN | E.CRC_BOTH, mem)
    for i, (p, key, nonce, src, dst, crc) in enumerate(bufs):
        c, tag = orc.seal(ORC[algo], key, nonce, p, fast=True)
        k = 4 * nseg(len(p))
        got = rd(crc, 2 * k)
        assert bytes(arr[i].tag) == tag and rd(dst, len(p)) == c, i
        assert got[:k] == orc.checksum(p) and got[k:] == orc.checksum(c), i
    # in-place open of the ciphertexts (dst), the last one with a bad tag
    ospecs = []
    for i, (p, key, nonce, src, dst, crc) in enumerate(bufs):
        tag = bytes(arr[i].tag)
        if i == len(bufs) - 1:
            tag = bytes([tag[0] ^ 0x80]) + tag[1:]
        d = dst.ptr if mem == E.MEM_DEVICE else dst.ctypes.data
        c = crc.ptr if mem == E.MEM_DEVICE else crc.ctypes.data
        ospecs.append({"key": key, "nonce": nonce, "src": d, "dst": d, "len": len(p), "crc": c, "tag": tag})
    oarr, ocnt = eng.make_blocks(ospecs)
    eng.open_batch(algo, oarr, ocnt, E.CRC_GEN | E.CRC_BOTH, mem)
    for i, (p, key, nonce, src, dst, crc) in enumerate(bufs):
        c, _ = orc.seal(ORC[algo], key, nonce, p, fast=True)
        k = 4 * nseg(len(p))
        got = rd(crc, 2 * k)
        assert got[k:] == orc.checksum(c), i  # the ciphertext CRCs stay either way
        if i == len(bufs) - 1:
            assert oarr[i].status == E.ETAG
            assert got[:k] == bytes(k) and rd(dst, len(p)) == bytes(len(p))
        else:
            assert oarr[i].status == E.OK and got[:k] == orc.checksum(p) and rd(dst, len(p)) == p.tobytes(), i


def test_crc_both_rejected_with_verify_or_ct(eng):
    src = heap(64)
    crc = np.zeros(8, np.uint8)
    arr, cnt = eng.make_blocks([{"key": bytes(32), "nonce": bytes(12), "src": src.ctypes.data,
                                 "dst": src.ctypes.data, "len": 64, "crc": crc.ctypes.data}])
    for mode in (E.CRC_VERIFY | E.CRC_BOTH, E.CRC_GEN | E.CRC_CT | E.CRC_BOTH, E.CRC_BOTH):
        with pytest.raises(E.EngineError) as ei:
            eng.seal_batch(E.AES256GCM, arr, cnt, mode, E.MEM_HOST)
        assert ei.value.code == E.EINVAL


@pytest.mark.parametrize("algo", [E.AES256GCM, E.CHACHA20P1305])
def test_data_encrypt_ex_all_checksum_combinations(eng, algo):
    """data_encrypt_ex / data_decrypt_ex on the context and through the
    aggregator: the object of encrypt.go:182-193 and, from the same call,
    checksum() of the plaintext and / or the object-store CRC."""
    wrapped = bytes((7 * k + 3) & 255 for k in range(256))
    with E.Aggregator(eng, window_us=300) as agg:
        for i, n in enumerate([0, 1, 32768, 100003, (4 << 20) - 3]):
            p = orc.gen_block(59, i, n)
            key, nonce = orc.gen_key(59, i)
            want = orc.data_encrypt(ORC[algo], key, nonce, wrapped, p.tobytes())
            wcrc = int(orc.object_checksum(want))
            wseg = orc.checksum(p)
            for front in (eng, agg):
                assert front.data_encrypt(algo, key, nonce, wrapped, p) == want
                assert front.data_encrypt(algo, key, nonce, wrapped, p, obj_crc=True) == (want, wcrc)
                assert front.data_encrypt(algo, key, nonce, wrapped, p, seg_crc=True) == (want, wseg)
                assert front.data_encrypt(algo, key, nonce, wrapped, p, obj_crc=True, seg_crc=True) == \
                    (want, wcrc, wseg)
            assert agg.data_decrypt(algo, key, want, seg_crc=True) == (p.tobytes(), wseg)
            assert eng.data_decrypt(algo, key, want, seg_crc=True) == (0, p.tobytes(), wseg)
            assert eng.data_decrypt(algo, key, want, expect_crc=wcrc, seg_crc=True) == (0, p.tobytes(), wseg)
            # a wrong stored object CRC: ECRC first, nothing released
            rc, pt, seg = eng.data_decrypt(algo, key, want, expect_crc=wcrc ^ 1, seg_crc=True)
            assert rc == E.ECRC and pt == b"" and seg == bytes(len(wseg)) and eng.last_got_crc == wcrc
            if n:
                bad = want[:-1] + bytes([want[-1] ^ 1])  # the tag
                rc, pt, seg = eng.data_decrypt(algo, key, bad, seg_crc=True)
                assert rc == E.ETAG and seg == bytes(len(wseg))


def test_per_object_heap_calls_from_many_threads(eng):
    """20 callers, each encrypting its own heap blocks into fresh heap objects
    and decrypting them back, through the aggregator (max-uploads shape)."""
    wrapped = bytes(range(256))
    T, per = 20, 3
    res = {}
    with E.Aggregator(eng, window_us=500, max_bytes=16 << 20) as agg:
        def work(t):
            for j in range(per):
                i = t * per + j
                n = [4 << 20, 1 << 20, 65536 + 13][j]
                p = orc.gen_block(61, i, n)
                key, nonce = orc.gen_key(61, i)
                obj, ocrc, seg = agg.data_encrypt(E.AES256GCM, key, nonce, wrapped, p, obj_crc=True, seg_crc=True)
                back, seg2 = agg.data_decrypt(E.AES256GCM, key, obj, seg_crc=True)
                res[i] = (p, key, nonce, obj, ocrc, seg, back, seg2)
        run_threads(T, work)
    for i, (p, key, nonce, obj, ocrc, seg, back, seg2) in res.items():
        assert obj == orc.data_encrypt(orc.AES256GCM, key, nonce, wrapped, p.tobytes()), i
        assert ocrc == int(orc.object_checksum(obj)) and seg == orc.checksum(p) == seg2, i
        assert back == p.tobytes(), i


def test_host_crc_pipeline_concurrent(eng):
    """checksum() and the ReadAt CRC verify on host memory through the
    pipeline: concurrent threads, pageable and pinned ranges, odd addresses,
    GEN and VERIFY (with a corrupted segment)."""
    pin = eng.alloc_pinned(8 << 20)
    try:
        T = 12

        def work(t):
            n = [0, 5, 32768, 32769, 1 << 20, (4 << 20) - 7][t % 6]
            p = orc.gen_block(67, t, n)
            if t % 4 == 3 and n:
                ctypes.memmove(pin + (t % 2) * (4 << 20) + 1, p.ctypes.data, n)  # pinned, unaligned
                ptr = pin + (t % 2) * (4 << 20) + 1
            else:
                buf = heap(max(n, 1), skew=t % 13)
                buf[:n] = p
                ptr = buf.ctypes.data
            want = orc.checksum(p)
            out = np.zeros(len(want), np.uint8)
            R = (E.jfsx_range * 1)()
            R[0].data, R[0].len, R[0].crc = ptr, n, out.ctypes.data
            eng.crc32c_segments(R, 1, E.CRC_GEN, E.MEM_HOST)
            assert out.tobytes() == want, t
            assert eng.checksum(p) == want
            if n > 40000:
                exp = np.frombuffer(want, np.uint8).copy()
                exp[4:8] ^= 0x10  # segment 1's stored CRC
                R[0].crc = exp.ctypes.data
                eng.crc32c_segments(R, 1, E.CRC_VERIFY, E.MEM_HOST)
                assert R[0].status == E.ECRC and R[0].bad_seg == 1
        # pinned-unaligned callers share one pool: run them one at a time
        run_threads(T, lambda t: work(t) if t % 4 != 3 else None)
        for t in range(3, T, 4):
            work(t)
    finally:
        eng.free_pinned(pin)


@pytest.mark.parametrize("level", [1, 2, 3])
def test_cache_verify_concurrent_heap_images(eng, level):
    """cacheFile.ReadAt (jfsx_cache_verify) from many threads on heap
    cache-file images at random unaligned ranges, against the oracle's
    ReadAt; one image has a corrupted segment."""
    rng = np.random.default_rng(level)
    imgs = []
    for b in range(6):
        n = int(rng.integers(65536, 4 << 20))
        p = orc.gen_block(71, b, n)
        img = heap(n + 4 * nseg(n), skew=b)
        img[:n] = p
        img[n:] = np.frombuffer(orc.checksum(p), np.uint8)
        if b == 5:
            img[n // 2] ^= 1
        imgs.append((n, img))
    reads = []
    for b, (n, _) in enumerate(imgs):
        reads.append((b, 0, n))
        for _ in range(5):
            off = int(rng.integers(0, n))
            reads.append((b, off, int(rng.integers(1, n - off + 1))))
    got = [None] * len(reads)

    def work(t):
        for r in range(t, len(reads), 8):
            b, off, size = reads[r]
            n, img = imgs[b]
            got[r] = eng.cache_verify(img, n, level, off, size)
    run_threads(8, work)
    for r, (b, off, size) in enumerate(reads):
        n, img = imgs[b]
        rc, data, nn, g, e, seg = orc.cache_readat(img.tobytes(), n, level, off, size)
        grc, gdata, gn, gg, ge, gseg = got[r]
        assert grc == {0: 0, 1: E.ECRC, 2: E.EOF}[rc], r
        assert gn == nn and gdata[:gn] == data[:nn], r
        if rc == 1:
            assert (gg, ge, gseg) == (g, e, seg), r
