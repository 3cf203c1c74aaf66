"""Diagnostic: per-section cycle shares of zstd_decompress_k from a
-DJFSX_ZSTD_STAMP build (JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP.so).
Shares only: the stamps' waits change the kernel's timing."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from juicefs_amd import engine as E  # noqa: E402
from tests import zstd_lib  # noqa: E402

names = ["literals", "seq headers", "ml/ll/states", "seq execute", "block start/raw", "table reads", "offset", "-"]
if os.environ.get("JFSX_ZSTD_SERIAL") != "1":  # block-parallel kernel: phases of jfsx_zstd2.h
    names = ["scan+tables", "huffman lanes", "sequence lanes+chain", "exec: seq loads/scans",
             "exec: flush/tails/raw", "checksum", "exec: literals", "exec: match rounds"]
nb, L = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 4 << 20
eng = E.Engine(0)
lib = E._lib
lib.jfsx_debug_zstd_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
pool = bench._text_pool(16 << 20, 7)
blocks = [pool[(b * 2654435761) % (pool.size - L):][:L].tobytes() for b in range(16)]
frames = [zstd_lib.compress(b, 1) for b in blocks]
got = eng.zstd_decompress([frames[i % 16] for i in range(nb)], [L] * nb)
assert all(st == E.OK for st, _ in got)
out = (ctypes.c_ulonglong * 12)()
lib.jfsx_debug_zstd_stamps(out, 1)
eng.zstd_decompress([frames[i % 16] for i in range(nb)], [L] * nb)
lib.jfsx_debug_zstd_stamps(out, 1)
tot = sum(out[k] for k in range(8))
print("cycles per frame (per wave) %.3e" % (tot / nb))
for k in range(8):
    print("%-22s %5.1f %%" % (names[k], 100.0 * out[k] / tot))
if os.environ.get("JFSX_ZSTD_SERIAL") != "1":
    print("per frame: windows %.0f, match rounds %.0f (%.2f per window), far-match lanes %.0f, sequence bytes %.0f"
          % (out[8] / nb, out[9] / nb, out[9] / max(out[8], 1), out[10] / nb, out[11] / nb))
eng.close()
