"""Device-resident rates of the §8(f) engines on one GPU, RS(8,4), 1 MiB
stripes, n = 4096 (6 GiB of BitrotWriter records per call):

* GET engine (rsg_decode_records_dev): verify-and-gather the data records
  (parity read only for degraded stripes), rebuild, surplus-parity check; with
  0 and 2 lost data shards;
* heal (rsg_heal_records_dev): one data and one parity disk replaced;
* whole-file bitrot_verify (rsg_bitrot_verify_dev) of the 12 shard files.

The calls are synchronous (per-stripe status to the host), so times are
wall-clock per call including that sync.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--stripe-bytes", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from rustfs_amd import Erasure
    from rustfs_amd.bitrot import HashAlgorithm, bitrot_verify_batch
    k, m, n = a.k, a.m, a.batch
    S = -(-a.stripe_bytes // k)
    rec = 32 + S
    t = k + m
    e = Erasure(k, m, a.stripe_bytes)
    st = torch.zeros((n, t, S), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    for s0 in range(0, n, 256):
        s1 = min(n, s0 + 256)
        st[s0:s1, :k] = torch.randint(0, 256, (s1 - s0, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    files = []
    for i in range(t):
        f = torch.empty((n, rec), dtype=torch.uint8, device="cuda")
        f[:, :32] = dig[:, i]
        f[:, 32:] = st[:, i]
        files.append(f.reshape(-1))
    want = st[:, :k].reshape(n, k * S)
    del st, dig
    out = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    payload = n * k * S

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps, r

    res = {}
    ms, (o, status) = timed(lambda: e.decode_records_batch(files, S, n, out=out))
    assert all(x == 0 for x in status) and torch.equal(o, want)
    res["get_all_present"] = {"ms": round(ms * 1e3, 3), "GiB_s_payload": round(payload / ms / GiB, 1),
                              # data records read once (verify + gather), data written once
                              "hbm_GB_s": round((k * n * rec + payload) / ms / 1e9, 1)}
    lost = [files[i] if i not in (0, 3) else None for i in range(t)]
    ms, (o, status) = timed(lambda: e.decode_records_batch(lost, S, n, out=out))
    assert all(x == 0 for x in status) and torch.equal(o, want)
    res["get_2_data_lost"] = {"ms": round(ms * 1e3, 3), "GiB_s_payload": round(payload / ms / GiB, 1)}
    tg = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") if i in (1, k) else None for i in range(t)]
    src = [files[i] if i not in (1, k) else None for i in range(t)]
    ms, status = timed(lambda: e.heal_records_batch(src, tg, S, n, work=out))
    assert all(x == 0 for x in status) and torch.equal(tg[1], files[1]) and torch.equal(tg[k], files[k])
    res["heal_1data_1parity"] = {"ms": round(ms * 1e3, 3), "GiB_s_payload": round(payload / ms / GiB, 1)}
    part = n * S
    ms, status = timed(lambda: bitrot_verify_batch(files, n * rec, part, HashAlgorithm.HighwayHash256S, S))
    assert status == [0] * t
    res["bitrot_verify_12_files"] = {"ms": round(ms * 1e3, 3),
                                     "GB_s_files": round(t * n * rec / ms / 1e9, 1)}
    print(json.dumps({"workload": f"RS({k},{m}) {a.stripe_bytes} B stripes, n={n}, device-resident records",
                      "results": res}), flush=True)


if __name__ == "__main__":
    main()
