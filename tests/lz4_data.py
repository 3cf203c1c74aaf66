"""Seeded synthetic inputs for the LZ4 stage tests (test data only).

Kinds cover the compressor's paths: incompressible bytes (search with growing
skip steps, one long last-literal run), a 4-symbol alphabet (short matches
everywhere), word text (typical literal/match mix), zeros (one long overlapping
match: match-length 255-runs), runs (offset-1 matches between random spans)
and repeat (a 1 KiB chunk repeated with sparse mutations: long far matches).
"""
import numpy as np

KINDS = ("random", "alphabet", "text", "zeros", "runs", "repeat")


def sample(kind, n, seed=0):
    rng = np.random.default_rng([seed, KINDS.index(kind), n])
    if n == 0:
        return b""
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "alphabet":
        return rng.integers(97, 101, n, dtype=np.uint8).tobytes()
    if kind == "zeros":
        return bytes(n)
    if kind == "text":
        nw = 300
        lens = rng.integers(1, 10, nw)
        tab = np.full((nw, 11), 32, np.uint8)
        for i in range(nw):
            tab[i, :lens[i]] = rng.integers(97, 123, lens[i], dtype=np.uint8)
        idx = rng.zipf(1.3, n // 2 + 8) % nw
        L = lens[idx] + 1
        ends = np.cumsum(L)
        k = int(np.searchsorted(ends, n)) + 1
        idx, L = idx[:k], L[:k]
        wid = np.repeat(idx, L)
        off = np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L)
        return tab[wid, off][:n].tobytes()
    if kind == "runs":
        out = np.empty(n, np.uint8)
        pos = 0
        while pos < n:
            m = int(rng.integers(1, 400))
            if rng.random() < 0.5:
                out[pos:pos + m] = rng.integers(0, 256, min(m, n - pos), dtype=np.uint8)
            else:
                out[pos:pos + m] = rng.integers(0, 256)
            pos += m
        return out.tobytes()
    if kind == "repeat":
        chunk = rng.integers(0, 256, 1024, dtype=np.uint8)
        out = np.resize(chunk, n).copy()
        flips = rng.integers(0, n, max(1, n // 5000))
        out[flips] ^= 0x5A
        return out.tobytes()
    raise ValueError(kind)


# (kind, n) grid for the golden fixtures and the GPU parity tests: the LZ4
# minimum (13), the 64 KiB + 11 table-type boundary (65547), block sizes
GOLDEN_SIZES = (0, 1, 5, 12, 13, 14, 64, 100, 4096, 65535, 65546, 65547, 65548, 100003, 1 << 20, 4 << 20)
