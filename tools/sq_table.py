"""SQ counter table of the one-pass engine kernels from tools/pmc_engine.sh
passes (p1: SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE; p2: SQ_INSTS_LDS
SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_COUNT), the last 3 dispatches of the
engine's decode kernel averaged.  VALU-busy = SQ_ACTIVE_INST_VALU x 4 (quad-
cycles) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) — the share of SIMD cycles
a wave64 VALU instruction would occupy at 4 cycles each, an upper bound (two
waves interleave at 2 cycles, MI355X_MICROARCH.md); wait = SQ_WAIT_ANY /
SQ_WAVE_CYCLES (the share of wave time stalled on any dependency).
Usage: python tools/sq_table.py DIR [DIR ...]   (DIR = gpurun_out/<tag>)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def last3(path):
    rows = list(csv.DictReader(open(path)))
    disp = defaultdict(dict)
    for r in rows:
        if "k_decode_records" not in r["Kernel_Name"]:
            continue
        d = disp[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = sorted(disp)[-3:]
    if not keys:
        return None
    out = {"name": disp[keys[-1]]["name"]}
    for c in set().union(*(disp[k].keys() for k in keys)) - {"name"}:
        out[c] = sum(disp[k].get(c, 0.0) for k in keys) / len(keys)
    return out


def main():
    print("| engine | kernel | ms | clock GHz | VALU instr | VALU-busy | LDS instr | SALU instr | wait share |")
    print("|---|---|---|---|---|---|---|---|---|")
    for d in sys.argv[1:]:
        for what in sorted(os.listdir(d)):
            p1, p2 = (os.path.join(d, what, f"p{i}", "run_counter_collection.csv") for i in (1, 2))
            if not (os.path.exists(p1) and os.path.exists(p2)):
                continue
            a, b = last3(p1), last3(p2)
            if not a or not b:
                continue
            cyc = a["GRBM_GUI_ACTIVE"] / 8
            busy = a["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024)
            name = a["name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(rsg::")[0]
            print(f"| {os.path.basename(d)}/{what} | `{name[:70]}` | {a['ns'] / 1e6:.3f} | {cyc / a['ns']:.2f} | "
                  f"{a['SQ_INSTS_VALU']:.3g} | {busy:.2f} | {b['SQ_INSTS_LDS']:.3g} | {b['SQ_INSTS_SALU']:.3g} | "
                  f"{a['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:.2f} |")


if __name__ == "__main__":
    main()
