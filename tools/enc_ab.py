"""Interleaved A/B of encode launch shapes (rsg_set_tuning knobs) at 1 MiB
blocks, n stripes, device-resident, HIP-event kernel time per launch (the
headline's protocol: 0.5 s busy warm-up per variant and round, then --reps
launches; median).  Rounds alternate the variants (A B C A B C ...) so a
box's clock drift spreads over all of them.  One JSON line per geometry.
Usage: python tools/enc_ab.py 12,4 --variant base= --variant b64=RSG_VEC_BLOCK:64
       [--digests] [--rounds 3] [--n 4096]"""
import argparse
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--digests", action="store_true")
    ap.add_argument("--block", type=int, default=1 << 20, help="block bytes (S = ceil(block / k))")
    ap.add_argument("--variant", action="append", default=[],
                    help="name=KNOB:VALUE[,KNOB:VALUE] (empty after = : the defaults)")
    a = ap.parse_args()
    import torch
    import bench
    from rustfs_amd import Erasure, _lib
    variants = []
    for v in a.variant or ["base="]:
        name, spec = v.split("=", 1)
        knobs = dict(kv.split(":", 1) for kv in spec.split(",") if kv)
        variants.append((name, knobs))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for g in a.geoms:
        k, m = map(int, g.split(","))
        t, n = k + m, a.n
        S = -(-a.block // k)
        e = Erasure(k, m, a.block)
        st = bench.random_stripes(dev, k, m, S, n, 11 + k)
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device=dev) if a.digests else None
        ref = None
        alg = n * t * S + (n * t * 32 if a.digests else 0)
        res = {name: [] for name, _ in variants}
        for _ in range(a.rounds):
            for name, knobs in variants:
                with _lib.tuned(**knobs):
                    avg, _mn = bench.time_encode(e, st, dig, stream, a.reps, warm=3, warm_seconds=0.5)
                    torch.cuda.synchronize()
                    chk = st[:, k:].clone() if dig is None else torch.cat([st[:, k:].reshape(-1), dig.reshape(-1)])
                    if ref is None:
                        ref = chk
                    assert torch.equal(chk, ref), f"{g} variant {name}: output differs from the first variant"
                res[name].append(avg)
        out = {"geometry": f"RS({k},{m})", "shard_bytes": S, "stripes": n, "digests": a.digests}
        for name, knobs in variants:
            ms = sorted(res[name])
            med = ms[len(ms) // 2]
            out[name] = {"knobs": knobs, "kernel_ms_rounds": [round(x, 4) for x in res[name]],
                         "kernel_ms": round(med, 4), "frac": round(alg / (med * 1e-3) / 1e9 / HBM, 4)}
        print(json.dumps(out), flush=True)
        del st, dig, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
