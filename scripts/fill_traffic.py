"""Fill `roofline.traffic` / `binding` of suite bench lines that ran before
their round's PMC summary existed, with bench.py's own formula (pmc_traffic):
traffic = HBM bytes per plaintext byte of the variant's PMC passes x this
line's plaintext bytes per launch.  The variant is the line's file name
(bench_<variant>.json, the names scripts/gpu_r3_suite.sh gives both).  A
filled line says so in roofline.traffic_filled_by.

A traffic figure a line took from an older round's file (traffic_source
under profiles/r2 or r3) is replaced by the newer summary's.

--replace: also replace traffic / binding a line already carries (a line
that ran before its kernel's new PMC passes were summarised).

usage: python3 scripts/fill_traffic.py [--replace] profiles/r4/pmc_r4.json profiles/r4/bench_*.json
"""
import json
import os
import sys


def main(pmc_path, paths, replace=False):
    variants = json.load(open(pmc_path))["variants"]
    for p in paths:
        lines = open(p).read().splitlines()
        idx = max((i for i, l in enumerate(lines) if l.startswith("{")), default=None)
        if idx is None:
            continue
        d = json.loads(lines[idx])
        key = os.path.basename(p)[len("bench_"):-len(".json")]
        v = variants.get(key)
        rf = d.get("roofline") or {}
        plain = rf.get("plain_bytes_per_launch")
        if v is None or not plain:
            continue
        changed = False
        older = str(rf.get("traffic_source") or "").startswith(("profiles/r2", "profiles/r3"))
        if (rf.get("traffic") is None or older or replace) and "bytes_per_plain_byte" in v:
            rf["traffic"] = int(v["bytes_per_plain_byte"] * plain)
            rf["traffic_source"] = "%s %s (%s; %s)" % (pmc_path, key, v.get("fetch_pass"), v.get("write_pass"))
            changed = True
        if (rf.get("binding") is None or replace) and ("lds_busy" in v or "valu_issue" in v or "salu_issue" in v):
            b = {k: v[k] for k in ("lds_busy", "valu_issue", "lds_conflict_share", "salu_issue", "salu_per_byte",
                                   "valu_per_byte") if k in v}
            b["source"] = "%s %s (%s)" % (pmc_path, key, v.get("lds_pass") or v.get("valu_pass") or v.get("salu_pass"))
            rf["binding"] = b
            changed = True
        if changed:
            rf["traffic_filled_by"] = "scripts/fill_traffic.py (PMC passes ran after this line)"
            d["roofline"] = rf
            lines[idx] = json.dumps(d)
            open(p, "w").write("\n".join(lines) + "\n")
            print("filled", p)


if __name__ == "__main__":
    args = sys.argv[1:]
    rep = "--replace" in args
    args = [a for a in args if a != "--replace"]
    main(args[0], args[1:], rep)
