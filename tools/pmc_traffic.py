"""Per-launch HBM traffic for bench.py's roofline.traffic, following
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so it is doubled.

    python tools/pmc_traffic.py --from profiles/r05/pmc

rebuilds tools/pmc_traffic.json (shipped with the tree, read by bench.py)
from tools/pmc_table.sh's passes: per key directory, meta.json (the kernel-name
substring of the measured dispatches and the calls made) and the raw
FETCH_SIZE / WRITE_SIZE run_counter_collection.csv; the measured dispatches
are the last `calls` ones whose name holds the substring (the setup's launches
come first), each dispatch's counter summed over its rows, averaged over the
dispatches.  Every entry's `source` is its key directory."""
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "pmc_traffic.json")


def dispatch_values(csv_path, counter, filt, calls):
    """The counter per measured dispatch (the last `calls` whose kernel name
    holds `filt`), in dispatch order."""
    per = collections.OrderedDict()
    for row in csv.DictReader(open(csv_path)):
        if filt in row["Kernel_Name"] and row["Counter_Name"] == counter:
            d = int(row["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(row["Counter_Value"])
    vals = [per[d] for d in sorted(per)]
    if len(vals) < calls:
        raise ValueError(f"{csv_path}: {len(vals)} dispatches of {filt!r}, want {calls}")
    return vals[-calls:]


def entry(keydir):
    meta = json.load(open(os.path.join(keydir, "meta.json")))
    fetch = dispatch_values(os.path.join(keydir, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE",
                            meta["kernel"], meta["calls"])
    write = dispatch_values(os.path.join(keydir, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE",
                            meta["kernel"], meta["calls"])
    f = sum(fetch) / len(fetch) * 1024 * 2
    w = sum(write) / len(write) * 1024
    return meta["key"], {"bytes_per_launch": int(f + w), "fetch_bytes_corrected": int(f), "write_bytes": int(w),
                         "kernel": meta["kernel"], "source": os.path.relpath(keydir, ROOT),
                         "dispatches": len(fetch),
                         "note": "FETCH_SIZE x2 (gfx950 wide-stream correction) + WRITE_SIZE, KiB -> bytes"}


def main():
    if len(sys.argv) != 3 or sys.argv[1] != "--from":
        raise SystemExit(__doc__)
    base = sys.argv[2]
    data = {}
    for d in sorted(os.listdir(base)):
        kd = os.path.join(base, d)
        if os.path.exists(os.path.join(kd, "meta.json")):
            k, v = entry(kd)
            data[k] = v
            print(k, v["bytes_per_launch"], v["kernel"])
    json.dump(data, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
