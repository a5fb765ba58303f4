"""Turn a tools/pmc.sh run into per-launch HBM traffic for bench.py's
roofline.traffic, following /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so it is doubled.

Usage: python tools/pmc_traffic.py gpurun_out/TAG KEY "kernel substring"
Writes/updates tools/pmc_traffic.json[KEY] (shipped to the GPU box with the tree, read by bench.py)."""
import collections
import csv
import glob
import json
import os
import sys

root, key, filt = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        if filt in row["Kernel_Name"] and row["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (_, c), v in per.items():
        vals[c].append(v)
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024 * 2
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_traffic.json")
data = json.load(open(out_path)) if os.path.exists(out_path) else {}
data[key] = {"bytes_per_launch": int(fetch + write), "fetch_bytes_corrected": int(fetch), "write_bytes": int(write),
             "kernel": filt, "source": root, "dispatches": len(vals["FETCH_SIZE"]),
             "note": "FETCH_SIZE x2 (gfx950 wide-stream correction), KiB -> bytes"}
json.dump(data, open(out_path, "w"), indent=1)
print(key, data[key])
