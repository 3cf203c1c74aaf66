"""Round-3 PMC summary: one labelled record per rocprofv3 --pmc pass.

Every pass is a directory gpurun_out/<suite>/pmc_<variant>__<set> holding the
counter CSVs of one `bench.py --steps 1 --warmup 0` run, and its log
<dir>.log ends with the bench's JSON line (plaintext bytes per launch).  For
each variant this writes, with the pass each number came from:

  traffic   HBM bytes per plaintext byte of the dominant kernel's LAST
            dispatch (an open run seals first): 2 x FETCH_SIZE x 1 KiB (the
            gfx950 wide-read correction of MI355X_MICROARCH.md) + WRITE_SIZE x 1 KiB
  binding   the compute pipes' busy fractions over the same kernel:
            lds_busy   = SQ_LDS_IDX_ACTIVE / (cycles x CUs)
            valu_issue = SQ_INSTS_VALU / (cycles x CUs)   (a CU issues at most one
                         wave64 VALU instruction per cycle over its 4 SIMDs)
            with cycles = GRBM_GUI_ACTIVE / 8 XCDs, CUs = 256

            salu_issue = SQ_INSTS_SALU / (cycles x CUs)  (codec passes)

usage: python3 scripts/pmc_r3.py gpurun_out/<suite> [more suites...] > profiles/r4/pmc_r4.json
(later suites' passes of the same variant and counter set replace earlier ones)
"""
import csv
import glob
import json
import os
import sys

KERNELS = {  # variant -> kernel-name prefix of the dominant kernel
    "seal_gcm": "void jfsx::gcm_main_k<false", "seal_gcm_bitslice": "void jfsx::gcm_main_k<false",
    "open_gcm": "void jfsx::gcm_main_k<true", "seal_gcm_ragged": "void jfsx::gcm_main_k<false",
    "open_gcm_ragged": "void jfsx::gcm_main_k<true", "ingest_gcm": "void jfsx::gcm_main_k<false",
    "seal_chacha": "void jfsx::cp_main_k<false", "open_chacha": "void jfsx::cp_main_k<true",
    "seal_chacha_ragged": "void jfsx::cp_main_k<false", "open_chacha_ragged": "void jfsx::cp_main_k<true",
    "crc_verify": "jfsx::crc_segments_k", "zstd_text": "jfsx::zstd_compress_k",
    "unzstd_text": "jfsx::zstd_decompress", "lz4_text": "jfsx::lz4_compress_",  # _k (global table) or _lds_k
    "unlz4_text": "void jfsx::lz4_decompress_k",
}
CUS, XCDS = 256, 8


def rows(d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        out += list(csv.DictReader(open(f)))
    return out


def bench_line(log):
    try:
        for line in reversed(open(log).read().splitlines()):
            if line.startswith("{"):
                return json.loads(line)
    except (OSError, ValueError):
        pass
    return None


def main(roots):
    out = {"source": roots, "method": __doc__.split("\n\n")[1].strip(), "passes": {}, "variants": {}}
    dirs = [d for root in roots for d in sorted(glob.glob(os.path.join(root, "pmc_*__*")))]
    for d in dirs:
        root = os.path.dirname(d)
        if not os.path.isdir(d):
            continue
        variant, cset = os.path.basename(d)[4:].split("__", 1)
        pref = KERNELS.get(variant)
        if pref is None:
            continue
        rs = [r for r in rows(d) if r.get("Kernel_Name", "").startswith(pref)]
        if not rs:
            continue
        # the last dispatch of the kernel (open runs seal once first)
        last = max(int(r.get("Dispatch_Id", 0)) for r in rs)
        vals = {}
        for r in rs:
            if int(r.get("Dispatch_Id", 0)) == last:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        b = bench_line(d + ".log") or {}
        plain = (b.get("roofline") or {}).get("plain_bytes_per_launch")
        # a pass is named <suite>/pmc_<variant>__<set>; its raw counter values
        # are kept under that key in "passes"
        pname = os.path.relpath(d, os.path.dirname(root))
        rec = {"pass": pname, "kernel_prefix": pref, "dispatch_id": last,
               "counters": vals, "plain_bytes_per_launch": plain,
               "bench_config": (b.get("config") or {}).get("workload")}
        out["passes"][pname] = rec
        v = out["variants"].setdefault(variant, {"kernel_prefix": pref})
        if "FETCH_SIZE" in vals and plain:
            v["fetch_bytes"] = 2 * vals["FETCH_SIZE"] * 1024
            v["fetch_pass"] = rec["pass"]
            v["plain_bytes_per_launch"] = plain
        if "WRITE_SIZE" in vals and plain:
            v["write_bytes"] = vals["WRITE_SIZE"] * 1024
            v["write_pass"] = rec["pass"]
        if "GRBM_GUI_ACTIVE" in vals:
            cyc = vals["GRBM_GUI_ACTIVE"] / XCDS * CUS
            if "SQ_LDS_IDX_ACTIVE" in vals:
                v["lds_busy"] = round(vals["SQ_LDS_IDX_ACTIVE"] / cyc, 4)
                v["lds_pass"] = rec["pass"]
            if "SQ_INSTS_VALU" in vals:
                v["valu_issue"] = round(vals["SQ_INSTS_VALU"] / cyc, 4)
                v["valu_pass"] = rec["pass"]
            if "SQ_INSTS_SALU" in vals:
                v["salu_issue"] = round(vals["SQ_INSTS_SALU"] / cyc, 4)
                v["salu_pass"] = rec["pass"]
                if plain:
                    # wave instructions per plaintext byte (scalar and vector)
                    v["salu_per_byte"] = round(vals["SQ_INSTS_SALU"] / plain, 4)
                    if "SQ_INSTS_VALU" in vals:
                        v["valu_per_byte"] = round(vals["SQ_INSTS_VALU"] / plain, 4)
            if "SQ_LDS_BANK_CONFLICT" in vals and "SQ_LDS_IDX_ACTIVE" in vals and vals["SQ_LDS_IDX_ACTIVE"]:
                v["lds_conflict_share"] = round(vals["SQ_LDS_BANK_CONFLICT"] / vals["SQ_LDS_IDX_ACTIVE"], 4)
    for v in out["variants"].values():
        if "fetch_bytes" in v:
            v["bytes_per_plain_byte"] = round((v["fetch_bytes"] + v.get("write_bytes", 0.0)) /
                                              v["plain_bytes_per_launch"], 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
