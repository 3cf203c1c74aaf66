"""Summarise rocprofv3 --pmc CSVs per kernel (sum over dispatches, per dispatch avg)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")[:60]
        name = row.get("Counter_Name")
        acc[k][name] += float(row.get("Counter_Value", 0))
        cnt[k][name] += 1
for k in acc:
    print(k)
    disp = max(cnt[k].values())
    for name in sorted(acc[k]):
        print("   %-24s total %.4g  per-dispatch %.4g" % (name, acc[k][name], acc[k][name] / max(1, cnt[k][name] / max(1, 1))))
