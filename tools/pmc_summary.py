"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: mean counter
value per dispatch.  Usage: python tools/pmc_summary.py gpurun_out/TAG [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "rsg::"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f)):
        if filt not in row["Kernel_Name"]:
            continue
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] += float(row["Counter_Value"])
        names[row["Dispatch_Id"]] = row["Kernel_Name"]
    for (d, c), v in per.items():
        acc[names[d]][c].append(v)
for k, cs in acc.items():
    print(k[:90])
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} mean {sum(vs)/len(vs):16.1f}  n={len(vs)}")
