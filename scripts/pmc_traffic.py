"""HBM traffic per plaintext byte of each transform kernel, from the FETCH_SIZE /
WRITE_SIZE passes of scripts/gpu_suite_r2.sh (one counter per rocprofv3 run;
the batch size in GiB is the second argument: 64 = the bench's configs[1]).

Corrections, as MI355X_MICROARCH.md's HBM section prescribes for gfx950:
FETCH_SIZE (KiB) counts 64 B per 128-B read request of a 16-B/lane streaming
read, so it is doubled; WRITE_SIZE (KiB) is exact for 16-B/lane stores.

usage: python3 scripts/pmc_traffic.py gpurun_out/<dir> [GiB] > profiles/<round>/pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys

PLAIN = (int(sys.argv[2]) if len(sys.argv) > 2 else 4) * 2**30  # plaintext bytes per pass

PASSES = {  # bench variant -> (fetch dir, write dir, kernel name prefix)
    "gcm_ttable": ("gcm_fetch", "gcm_write", "void jfsx::gcm_main_k<false, 1, 1, 0>"),
    "gcm_bitslice": ("gcmbs_fetch", "gcmbs_write", "void jfsx::gcm_main_k<false, 1, 1, 1>"),
    "chacha": ("cp_fetch", "cp_write", "void jfsx::cp_main_k<false, 1>"),
    "crc_verify": ("crc_fetch", None, "jfsx::crc_segments_k"),
}


def counter(root, sub, name, kernel):
    vals = []
    for f in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == name and row.get("Kernel_Name", "").startswith(kernel):
                vals.append(float(row["Counter_Value"]))
    return vals


def main(root):
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, %d GiB batch per pass (%s)" % (PLAIN >> 30, root),
           "correction": "fetch_bytes = 2 x FETCH_SIZE x 1024 (gfx950 wide-read tally); write_bytes = WRITE_SIZE x 1024",
           "plain_bytes_per_pass": PLAIN, "kernels": {}}
    for key, (fd, wd, kern) in PASSES.items():
        f = counter(root, fd, "FETCH_SIZE", kern)
        w = counter(root, wd, "WRITE_SIZE", kern) if wd else []
        if not f:
            continue
        # crc_verify runs a GEN launch then the VERIFY launch: take the last
        fetch = 2 * f[-1] * 1024
        write = w[-1] * 1024 if w else 0.0
        out["kernels"][key] = {"kernel": kern, "fetch_bytes": fetch, "write_bytes": write,
                               "batch": "%d GiB" % (PLAIN >> 30),
                               "bytes_per_plain_byte": round((fetch + write) / PLAIN, 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
