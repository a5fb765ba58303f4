"""Turn a tools/pmc_bench.sh run (FETCH_SIZE and WRITE_SIZE passes over one
default bench run) into tools/pmc_traffic.json entries for the line's extras
that no dedicated pass covers: config 3's reconstruct with 1-4 lost shards,
config 5's RS(16,4) share, and the whole-file bitrot verify — following
/opt/skills/guides/MI355X_MICROARCH.md §HBM as tools/pmc_traffic.py does
(FETCH_SIZE in KiB and doubled on gfx950, WRITE_SIZE in KiB).

Kernels are told apart by name and, where two extras share a kernel, by
their place in the run: reconstruct with 4 lost runs k_gf_apply_vec<8, 4>
like the headline encode, after reconstruct with 3 lost; the bitrot verify
runs k_hh256_quad<0, 2> like the all-present GET, over 12 files (the larger
grid) instead of 8.

Usage: python tools/pmc_bench_traffic.py gpurun_out/TAG [k m S n]"""
import collections
import csv
import json
import os
import sys


def dispatches(path):
    """Dispatch id -> (kernel name, grid size, {counter: value summed over instances})."""
    out = {}
    for row in csv.DictReader(open(path)):
        d = int(row["Dispatch_Id"])
        if d not in out:
            out[d] = (row["Kernel_Name"], int(row["Grid_Size"]), collections.defaultdict(float))
        out[d][2][row["Counter_Name"]] += float(row["Counter_Value"])
    return out


def main():
    root = sys.argv[1]
    k, m, S, n = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (8, 4, 131072, 4096)
    fetch = dispatches(os.path.join(root, "p1", "run_counter_collection.csv"))
    write = dispatches(os.path.join(root, "p2", "run_counter_collection.csv"))

    def select(runs, pred):
        """Ids (in order) of the dispatches of one run whose (name, grid, position) pass pred."""
        ids = sorted(runs)
        return [d for i, d in enumerate(ids) if pred(runs[d][0], runs[d][1], i, ids)]

    def first_index(runs, sub):
        ids = sorted(runs)
        return next((i for i, d in enumerate(ids) if sub in runs[d][0]), None)

    def entry(pred, kernel):
        f = select(fetch, pred)
        w = select(write, pred)
        if not f or not w:
            return None
        fb = sum(fetch[d][2]["FETCH_SIZE"] for d in f) / len(f) * 1024 * 2
        wb = sum(write[d][2]["WRITE_SIZE"] for d in w) / len(w) * 1024
        return {"bytes_per_launch": int(fb + wb), "fetch_bytes_corrected": int(fb), "write_bytes": int(wb),
                "kernel": kernel, "source": root, "dispatches": len(f),
                "note": "FETCH_SIZE x2 (gfx950 wide-stream correction), KiB -> bytes"}

    keys = {}
    for r in (1, 2, 3):
        name = f"k_gf_apply_vec<{k}, {r},"
        keys[f"reconstruct_e{r}_rs{k}{m}_S{S}_n{n}"] = (lambda nm, g, i, ids, name=name: name in nm, name)

    def after_e3(runs):
        i3 = first_index(runs, f"k_gf_apply_vec<{k}, 3,")
        name = f"k_gf_apply_vec<{k}, 4,"
        return lambda nm, g, i, ids: name in nm and i3 is not None and i > i3

    def verify_12(runs):
        grids = [g for nm, g, _ in runs.values() if "k_hh256_quad<0, 2>" in nm]
        big = max(grids) if grids else None
        return lambda nm, g, i, ids: "k_hh256_quad<0, 2>" in nm and g == big

    out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for key, (pred, kernel) in keys.items():
        e = entry(pred, kernel)
        if e:
            data[key] = e
    # the two extras that share a kernel with another: position and grid decide
    for key, mk, kernel in ((f"reconstruct_e4_rs{k}{m}_S{S}_n{n}", after_e3, f"k_gf_apply_vec<{k}, 4, (after e3)"),
                            (f"verify_all_rs{k}{m}_S{S}_n{n}", verify_12, "k_hh256_quad<0, 2> (12 files)")):
        pf, pw = mk(fetch), mk(write)
        f = select(fetch, pf)
        w = select(write, pw)
        if f and w:
            fb = sum(fetch[d][2]["FETCH_SIZE"] for d in f) / len(f) * 1024 * 2
            wb = sum(write[d][2]["WRITE_SIZE"] for d in w) / len(w) * 1024
            data[key] = {"bytes_per_launch": int(fb + wb), "fetch_bytes_corrected": int(fb), "write_bytes": int(wb),
                         "kernel": kernel, "source": root, "dispatches": len(f),
                         "note": "FETCH_SIZE x2 (gfx950 wide-stream correction), KiB -> bytes"}
    # config 5's share: RS(16,4), S = 65536, 4096 stripes (the only k_gf_apply_loop<4 of the line)
    e = entry(lambda nm, g, i, ids: "k_gf_apply_loop<4" in nm, "k_gf_apply_loop<4")
    if e:
        data["rs164_S65536_n4096"] = e
    json.dump(data, open(out_path, "w"), indent=1)
    for key in sorted(data):
        if data[key]["source"] == root:
            print(key, data[key]["bytes_per_launch"], data[key]["dispatches"])


if __name__ == "__main__":
    main()
