"""One-pass against two-pass GET / heal at the geometries without a network
(round 5: the run-time-table one-pass kernel for every k <= 16, m <= 4, and
EC:5..8's one- and two-loss patterns), at
1 MiB blocks (S = ceil(1 MiB / k)), n stripes of BitrotWriter records on the
device.  For each geometry: the in-place GET with the most data shards lost
that m allows (two, or one at m = 1), and the heal of one data + one parity
shard (one data shard at m = 1), each on both record engines
(rsg_set_record_engine ONE_PASS / TWO_PASS), timed like bench.py's engine
extras: back-to-back calls until the device has been busy 0.5 s, then 20
calls, kernel time from the in-call HIP events (median).  Prints one JSON line
per geometry.  --tune RSG_DECODE_NET=0 (repeatable) sets a kernel-choice knob
through rsg_set_tuning for the whole run (e.g. the table kernel in place of the
networks).  Usage: python tools/geom_engines.py 5,4 11,4 15,1 [--n 4096]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("geoms", nargs="+")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--get-lost", default=None, help="shards lost for the GET, e.g. 0 or 0,3 (default: 0,k-1)")
    ap.add_argument("--heal-lost", default=None, help="shards healed, e.g. 1,10 (default: 1,k)")
    ap.add_argument("--block", type=int, default=1 << 20, help="block bytes (S = ceil(block / k))")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the output checks (ablation builds whose kernels skip arithmetic)")
    a = ap.parse_args()
    import torch
    import bench
    from rustfs_amd import Erasure, _lib
    L = _lib.load()
    ctx = _lib.context(0).handle
    for kv in a.tune:
        name, value = kv.split("=", 1)
        _lib.set_tuning(name, value)
    for g in a.geoms:
        k, m = map(int, g.split(","))
        t, n = k + m, a.n
        S = -(-a.block // k)
        rec = 32 + S
        e = Erasure(k, m, a.block)
        st = bench.random_stripes(torch.device("cuda", 0), k, m, S, n, 77 + k)
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
        e.encode_batch(st, dig)
        files = []
        for i in range(t):
            f = torch.empty((n, rec), dtype=torch.uint8, device="cuda")
            f[:, :32] = dig[:, i]
            f[:, 32:] = st[:, i]
            files.append(f.reshape(-1))
        del dig
        lost_get = (0, k - 1) if m >= 2 and k >= 2 else (0,)
        lost_heal = (1 % k, k) if m >= 2 else (k - 1,)
        if a.get_lost is not None:
            lost_get = tuple(int(x) for x in a.get_lost.split(","))
        if a.heal_lost is not None:
            lost_heal = tuple(int(x) for x in a.heal_lost.split(","))
        slots = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        tg = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") if i in lost_heal else None for i in range(t)]
        gsrc = [None if i in lost_get else files[i] for i in range(t)]
        hsrc = [None if i in lost_heal else files[i] for i in range(t)]
        want = {i: st[n - 1, i].clone() for i in range(k)}
        out = {"geometry": f"RS({k},{m})", "shard_bytes": S, "stripes": n, "get_lost": list(lost_get),
               "heal_lost": list(lost_heal), "tuning": a.tune}
        cases = {
            "get": (lambda: e.decode_records_into_batch(gsrc, S, n, targets=slots),
                    n * ((t - len(lost_get)) * rec + len(lost_get) * S)),
            "heal": (lambda: e.heal_records_batch(hsrc, tg, S, n),
                     n * ((t - len(lost_heal)) * rec + len(lost_heal) * rec)),
        }
        for engine, code in (("one_pass", _lib.RSG_RECORD_ENGINE_ONE_PASS), ("two_pass", _lib.RSG_RECORD_ENGINE_TWO_PASS)):
            _lib.check(L.rsg_set_record_engine(ctx, code))
            for what, (fn, alg) in cases.items():
                bench.steady_loop(fn, 0.5)
                kms = []
                _lib.check(L.rsg_set_kernel_timing(ctx, 1))
                for _ in range(a.reps):
                    r = fn()
                    v = ctypes.c_float(-1)
                    _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
                    kms.append(v.value)
                _lib.check(L.rsg_set_kernel_timing(ctx, 0))
                torch.cuda.synchronize()
                if a.no_check:
                    pass
                elif what == "get":
                    _, src, status = r
                    assert all(x == 0 for x in status)
                    for i in lost_get:
                        if i < k:  # a lost parity shard has no slot
                            assert torch.equal(slots.view(n, k, S)[n - 1, i], want[i]), (g, engine, i)
                else:
                    assert all(x == 0 for x in r)
                    for i in lost_heal:
                        assert torch.equal(tg[i], files[i]), (g, engine, i)
                km = sorted(kms)[len(kms) // 2]
                out[f"{what}_{engine}"] = {"kernel_ms": round(km, 4), "min": round(min(kms), 4),
                                           "max": round(max(kms), 4), "alg_bytes": alg,
                                           "frac": round(alg / (km * 1e-3) / 1e9 / HBM, 4)}
        _lib.check(L.rsg_set_record_engine(ctx, _lib.RSG_RECORD_ENGINE_AUTO))
        # what AUTO picks (the library's policy) for the same calls
        for what, (fn, alg) in cases.items():
            bench.steady_loop(fn, 0.3)
            _lib.check(L.rsg_set_kernel_timing(ctx, 1))
            kms = []
            for _ in range(a.reps):
                fn()
                v = ctypes.c_float(-1)
                _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
                kms.append(v.value)
            _lib.check(L.rsg_set_kernel_timing(ctx, 0))
            km = sorted(kms)[len(kms) // 2]
            out[f"{what}_auto"] = {"kernel_ms": round(km, 4), "frac": round(alg / (km * 1e-3) / 1e9 / HBM, 4)}
        print(json.dumps(out), flush=True)
        del files, slots, tg, gsrc, hsrc, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
