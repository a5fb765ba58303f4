"""Steady-state per-kernel durations from a rocprofv3 kernel trace of
bench.py: bench.py times every kernel's last calls after a >= 0.5 s busy
warm-up, so the last N dispatches of each kernel are its timed, steady-state
ones; the whole-trace min / max (rocprof's --stats) also holds the warm-up
calls right after an idle or another kernel, when the chip's clock dips
(profiles/r05/clock/).  Usage: python tools/steady_stats.py run_kernel_trace.csv [N=20 | --by-grid]"""
import collections
import csv
import sys


def by_grid(path):
    """Every rsg kernel per launch shape (kernel, grid size): rocprof's --stats
    averages one kernel name over all its launches, and the same kernel also
    runs small launches (extras.host_path's sub-batches of
    rsg_encode_batch_host run k_gf_apply_vec<8,4> over 64 stripes) — the
    headline's own average is that of its n = 4096 grid."""
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "rsg::" not in r["Kernel_Name"]:
            continue
        by[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print("| kernel | grid (threads) | calls | average ms | median | min | max |")
    print("|---|---|---|---|---|---|---|")
    for (name, grid), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        t = sorted(d)
        print(f"| `{name.split('(rsg::')[0].replace('void ', '')}` | {grid} | {len(d)} | {sum(d) / len(d):.4f} | "
              f"{t[len(t) // 2]:.4f} | {t[0]:.4f} | {t[-1]:.4f} |")


def main():
    path = sys.argv[1]
    if len(sys.argv) > 2 and sys.argv[2] == "--by-grid":
        return by_grid(path)
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "rsg::" not in r["Kernel_Name"]:
            continue
        by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]),
                                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    print(f"| kernel | calls | last {last}: median ms | min | max | max/min | whole trace: min | max | max/min |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        d = [x for _, x in sorted(v)]
        if len(d) < last:
            continue
        t = sorted(d[-last:])
        print(f"| `{name.split('(rsg::')[0].replace('void ', '')}` | {len(d)} | {t[len(t) // 2]:.4f} | {t[0]:.4f} | "
              f"{t[-1]:.4f} | {t[-1] / t[0]:.3f} | {min(d):.4f} | {max(d):.4f} | {max(d) / min(d):.3f} |")


if __name__ == "__main__":
    main()
