"""Generate tests/golden/lz4_golden.json with the system LZ4 C library.

The reference's "lz4" compressor is github.com/hungys/go-lz4 (go.mod:34), a
cgo wrapper over the LZ4 C library (LZ4_compress_default,
LZ4_decompress_safe; pkg/compress/compress.go:107-125).  Its vendored C
sources are not in /root/reference; this script records what the LZ4 C
library installed here (liblz4.so.1, version printed into the fixture)
writes for each (kind, n) input of tests/lz4_data.py: the compressed length
and SHA-256.  Inputs are regenerated from their seed, so only hashes are
committed.  Run: python tests/golden/make_lz4_golden.py
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import lz4_data  # noqa: E402


def main():
    L = ctypes.CDLL("liblz4.so.1")
    ver = L.LZ4_versionNumber()
    rows = []
    for kind in lz4_data.KINDS:
        for n in lz4_data.GOLDEN_SIZES:
            src = lz4_data.sample(kind, n, seed=7)
            cap = L.LZ4_compressBound(n)
            dst = ctypes.create_string_buffer(max(cap, 1))
            r = L.LZ4_compress_default(src, dst, n, cap)
            assert r > 0
            c = dst.raw[:r]
            back = ctypes.create_string_buffer(max(n, 1))
            assert L.LZ4_decompress_safe(c, back, r, n) == n and back.raw[:n] == src
            rows.append({"kind": kind, "n": n, "seed": 7, "in_sha256": hashlib.sha256(src).hexdigest(),
                         "bound": cap, "out_len": r, "out_sha256": hashlib.sha256(c).hexdigest()})
    json.dump({"liblz4_version": ver, "cases": rows}, open(os.path.join(HERE, "lz4_golden.json"), "w"), indent=0)
    print("wrote %d cases (liblz4 %d)" % (len(rows), ver))


if __name__ == "__main__":
    main()
