"""Markdown table of committed bench lines.
usage: python3 scripts/lines_table.py profiles/r4/bench_*.json"""
import json
import sys


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


print("| line | value GB/s | kernel | kernel ms | achieved GB/s | frac | HBM B / plaintext B | CPU baseline GB/s (threads) | check |")
print("|---|---|---|---|---|---|---|---|---|")
for p in sys.argv[1:]:
    d = last_json(p)
    if not d:
        continue
    r = d.get("roofline") or {}
    cpu = d.get("cpu_baseline") or {}
    plain = r.get("plain_bytes_per_launch")
    tr = r.get("traffic")
    bpb = "%.3f" % (tr / plain) if tr and plain else "—"
    fc = d.get("full_check") or {}
    chk = "all %d blocks" % fc["blocks"] if fc else ("%s sampled" % d.get("verified_blocks", 0))
    print("| `%s` | %s | %s | %s | %s | %s | %s | %s | %s |" % (
        p.split("/")[-1], d.get("value"), r.get("kernel", "—"), r.get("kernel_avg_ms", "—"),
        r.get("achieved", "—"), r.get("frac", "—"), bpb,
        "%s (%s)" % (cpu.get("value"), cpu.get("cores")) if cpu else "—", chk))
