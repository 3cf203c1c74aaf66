"""Diagnostic: per-workgroup timeline of gcm_main_k on a batch (needs the
make variant V=TRACE library).  usage: JFSX_LIB=juicefs_amd/_build/libjfsx_TRACE.so
python3 scripts/wgtrace.py [--ragged] [--blocks N] [--block-bytes L]"""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import SEED, ragged_len  # noqa: E402
from juicefs_amd import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ragged", action="store_true")
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--block-bytes", type=int, default=4 << 20)
a = ap.parse_args()
eng = E.Engine(0)
L, nb = a.block_bytes, a.blocks
lens = [ragged_len(SEED, b, L) if a.ragged else L for b in range(nb)]
src, dst, crc = eng.alloc(nb * L), eng.alloc(nb * L), eng.alloc(nb * 4 * (L // E.SEG + 1))
eng.gen_synthetic_batch(src, L, lens, SEED, 0)
specs = []
for b in range(nb):
    k, n = E.gen_key(SEED, b)
    specs.append({"key": k, "nonce": n, "src": src.ptr + b * L, "dst": dst.ptr + b * L, "len": lens[b],
                  "crc": crc.ptr + 4 * (L // E.SEG + 1) * b})
blks, n = eng.make_blocks(specs)
for _ in range(3):
    eng.seal_batch(E.AES256GCM, blks, n, E.CRC_GEN, E.MEM_DEVICE)
tr = np.zeros(4 * 65536, np.uint64)
f = eng.L.jfsx_debug_wgtrace
f.argtypes, f.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
assert f(tr.ctypes.data, 65536) == 0
nt = min(n, 65536)
t0, t1, hw, by = tr[0:4 * nt:4].astype(np.int64), tr[1:4 * nt:4].astype(np.int64), tr[2:4 * nt:4], tr[3:4 * nt:4].astype(np.int64)
base = t0.min()
t0, t1 = (t0 - base) / 100.0, (t1 - base) / 100.0  # 100 MHz -> microseconds
span = t1.max()
dur = t1 - t0
cu = [(int(h) >> 32, (int(h) >> 8) & 0xff) for h in hw]
per = collections.defaultdict(list)
for i, c in enumerate(cu):
    per[c].append((t0[i], t1[i], by[i]))
busy = {c: sum(e - s for s, e, _ in v) for c, v in per.items()}
last = sorted(max(e for _, e, _ in v) for v in per.values())
gaps = []
for v in per.values():
    v.sort()
    gaps += [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
A = np.vstack([np.ones(nt), by / 1e6]).T
coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
print("tasks %d  CUs seen %d  kernel span %.1f us" % (nt, len(per), span))
print("mean CU busy %.1f%% of span; CU last-end spread: min %.1f  p50 %.1f  max %.1f us" % (
    100 * np.mean(list(busy.values())) / span, last[0], last[len(last) // 2], last[-1]))
print("gap between WGs on a CU: mean %.2f  p90 %.2f us" % (np.mean(gaps), np.percentile(gaps, 90)))
print("task duration = %.1f us + %.1f us/MB (fit);  mean duration %.1f us" % (coef[0], coef[1], dur.mean()))
for lo, hi in ((0, 256e3), (256e3, 1e6), (1e6, 2e6), (2e6, 3e6), (3e6, 5e6)):
    m = (by >= lo) & (by < hi)
    if m.any():
        print("  size %7.0f-%7.0f KB: n %5d  us/MB %.1f" % (lo / 1e3, hi / 1e3, m.sum(), (dur[m] / (by[m] / 1e6)).mean()))
