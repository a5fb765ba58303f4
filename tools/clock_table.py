"""Per-dispatch clock table of the one-pass engines (round 5, VERDICT r4 item
1): for each engine call, the kernel's duration (rocprofv3 kernel trace) and
its cycle count (GRBM_GUI_ACTIVE summed over the 8 XCDs, / 8) from the PMC
pass of the same loop, and the effective clock = cycles / duration
(MI355X_MICROARCH.md, "DVFS give-back").  A rising cycle count would mean the
kernel stalls (ring, DMA); a constant one with a falling clock means the chip
lowered its clock.  Usage: python tools/clock_table.py DIR [DIR ...] (each
DIR holds pmc_<what>/run_counter_collection.csv) > table.md"""
import collections
import csv
import os
import sys


def rows(path):
    by = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "records" not in r["Kernel_Name"]:
            continue
        d = by.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        d["start"] = int(r["Start_Timestamp"])
        d["end"] = int(r["End_Timestamp"])
    return list(by.values())


def main():
    for base in sys.argv[1:]:
        for what in sorted(os.listdir(base)):
            p = os.path.join(base, what, "run_counter_collection.csv")
            if not what.startswith("pmc_") or not os.path.exists(p):
                continue
            rs = rows(p)
            print(f"### {what[4:]}: `{rs[0]['name'].split('(')[0]}`, {len(rs)} calls\n")
            print("| call | after | duration ms | Mcycles (GRBM_GUI_ACTIVE / 8) | effective clock GHz |")
            print("|---|---|---|---|---|")
            prev = None
            for i, d in enumerate(rs):
                gap = (d["start"] - prev) / 1e6 if prev is not None else None
                after = "start" if gap is None else ("idle %.0f ms" % gap if gap > 100 else "back to back")
                cyc = d["GRBM_GUI_ACTIVE"] / 8
                print(f"| {i} | {after} | {d['dur_ms']:.4f} | {cyc / 1e6:.3f} | {cyc / (d['dur_ms'] * 1e-3) / 1e9:.3f} |")
                prev = d["end"]
            cyc = [d["GRBM_GUI_ACTIVE"] / 8 for d in rs]
            dur = [d["dur_ms"] for d in rs]
            print(f"\ncycles max/min {max(cyc) / min(cyc):.3f}; duration max/min {max(dur) / min(dur):.3f}\n")


if __name__ == "__main__":
    main()
