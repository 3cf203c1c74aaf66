"""The level matrix of the reference's TestChecksum (pkg/chunk/disk_cache_test.go:134-221),
as data: five cache files and eleven reads, run at each verify level."""
import numpy as np

SEG = 32 << 10


def crc_bytes(data, checksum):
    return checksum(bytes(data))


def build_files(checksum, rng_seed=7):
    """Returns {key: (file_image_bytes, data_length)} as the reference writes them."""
    rng = np.random.default_rng(rng_seed)
    hello = b"helloworld"
    buf = rng.integers(0, 256, 102400, dtype=np.uint8).tobytes()
    corrupt = bytearray(buf)
    corrupt[98304:102400] = bytes(4096)  # "reset 96K ~ 100K"
    big = rng.integers(0, 256, 1048576, dtype=np.uint8).tobytes()
    return {
        "k1": (hello, 10),                             # cached while checksum = none
        "k2": (hello + checksum(hello), 10),
        "k3": (buf + checksum(buf), 102400),
        "k4": (buf + checksum(bytes(corrupt)), 102400),  # CRCs of a corrupted copy
        "k5": (big + checksum(big), 1048576),
    }


CASES = [  # key, off, size, expect ok (before the level adjustments below)
    ("k1", 0, 10, True), ("k1", 3, 5, True), ("k2", 0, 10, True), ("k2", 3, 5, True),
    ("k3", 0, 102400, True), ("k3", 8192, 92160, True),
    ("k4", 0, 102400, True), ("k4", 8192, 92160, True),
    ("k5", 0, 1048576, True), ("k5", 131072, 131072, True), ("k5", 102400, 512000, True),
]
LEVELS = ["none", "full", "shrink", "extend"]


def expected(level):
    cases = [list(c) for c in CASES]
    if level != "none":
        cases[6][3] = False          # k4 whole-file read fails for full/shrink/extend
    if level == "extend":
        cases[7][3] = False          # only extend widens 8K..98K to the corrupt segment
    return [tuple(c) for c in cases]


def run(read, checksum):
    """read(file_img, length, level, off, size) -> ok (bool).  Returns list of mismatches."""
    files = build_files(checksum)
    bad = []
    for level in LEVELS:
        for key, off, size, exp in expected(level):
            img, length = files[key]
            ok = read(img, length, level, off, size)
            if ok != exp:
                bad.append((level, key, off, size, exp, ok))
    return bad
