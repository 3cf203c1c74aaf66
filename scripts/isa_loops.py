"""Print instruction mix of the loops in one kernel of a gfx950 .s file.
usage: python scripts/isa_loops.py file.s kernel_symbol_prefix"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pref = sys.argv[2]
i = s.index("\n" + pref) + 1
name = s[i:s.index(":", i)]
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
labels = {}
for n, l in enumerate(body):
    t = l.strip().split(";")[0].strip()
    if t.endswith(":") and t.startswith(".LBB"):
        labels[t[:-1]] = n
print(name[:90])
for n, l in enumerate(body):
    t = l.strip().split()
    if t and (t[0].startswith("s_cbranch") or t[0] == "s_branch"):
        tgt = t[-1]
        if tgt in labels and labels[tgt] < n:
            seg = body[labels[tgt]:n]
            ins = [x.strip().split()[0] for x in seg
                   if x.strip() and not x.strip().startswith((".", ";")) and not x.strip().split(";")[0].strip().endswith(":")]
            c = Counter(ins)
            v = sum(k2 for k, k2 in c.items() if k.startswith("v_"))
            print("loop %s len %d valu %d ds %d smem %d scratch %d" % (
                tgt, len(ins), v, sum(k2 for k, k2 in c.items() if k.startswith("ds_")),
                sum(k2 for k, k2 in c.items() if k.startswith("s_load") or k.startswith("s_buffer_load")),
                sum(k2 for k, k2 in c.items() if "scratch" in k)))
            if len(ins) > 200:
                for k, k2 in sorted(c.items(), key=lambda x: -x[1])[:18]:
                    print("     %-28s %d" % (k, k2))
