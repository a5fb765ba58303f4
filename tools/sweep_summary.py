"""Summarise tools/sweep_fused.sh output (bench.py JSON lines) as a markdown table."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep"
rows = {}
for f in glob.glob(os.path.join(d, "s*k_*.json")):
    name = os.path.basename(f)[1:-5]
    kib, mode = name.split("k_")
    line = [l for l in open(f) if l.startswith("{")][-1]
    rows.setdefault(int(kib), {})[mode] = json.loads(line)

print("| stripe | batch | encode + fused HH256S: GiB/s payload | ms/launch | HBM frac | encode only: GiB/s | HBM frac |")
print("|---|---|---|---|---|---|---|")
for kib in sorted(rows):
    h, p = rows[kib].get("hash"), rows[kib].get("plain")
    size = f"{kib // 1024} MiB" if kib >= 1024 else f"{kib} KiB"
    hb = h["config"].get("stripes_per_gpu") if h else None
    cells = [size, str(hb or (p["config"].get("stripes_per_gpu") if p else ""))]
    cells += [f"{h['value']:.0f}", f"{h['ms_per_step']:.3f}", f"{h['roofline']['frac']:.3f}"] if h else ["", "", ""]
    cells += [f"{p['value']:.0f}", f"{p['roofline']['frac']:.3f}"] if p else ["", ""]
    print("| " + " | ".join(cells) + " |")
    g = rows[kib].get("hash4g")
    if g:
        print(f"| {size} | {g['config']['stripes_per_gpu']} (4 GiB payload) | {g['value']:.0f} | {g['ms_per_step']:.3f} | "
              f"{g['roofline']['frac']:.3f} | | |")
