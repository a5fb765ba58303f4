"""The all-present in-place GET and the whole-file bitrot_verify at 1 MiB
blocks (S = ceil(1 MiB / k)), n stripes of BitrotWriter records on the device,
per geometry: kernel ms from the in-call HIP events (rsg_set_kernel_timing),
median of 20 calls after 0.5 s of back-to-back calls, as bench.py's engine
extras, and the fraction of 8 TB/s on the calls' algorithmic bytes.  Prints
one JSON line per geometry.  Usage: python tools/verify_geoms.py 12,4 6,4"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from rustfs_amd import Erasure, _lib
    from rustfs_amd.bitrot import HashAlgorithm, bitrot_verify_batch
    L = _lib.load()
    ctx = _lib.context(0).handle
    n = 4096
    for g in sys.argv[1:]:
        k, m = map(int, g.split(","))
        t = k + m
        S = -(-(1 << 20) // k)
        rec = 32 + S
        e = Erasure(k, m, 1 << 20)
        st = bench.random_stripes(torch.device("cuda", 0), k, m, S, n, 5 + k)
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
        e.encode_batch(st, dig)
        files = []
        for i in range(t):
            f = torch.empty((n, rec), dtype=torch.uint8, device="cuda")
            f[:, :32] = dig[:, i]
            f[:, 32:] = st[:, i]
            files.append(f.reshape(-1))
        del st, dig
        slots = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        out = {"geometry": f"RS({k},{m})", "shard_bytes": S, "record_mod16": rec % 16}
        cases = {"get_all_present": (lambda: e.decode_records_into_batch(files, S, n, targets=slots), n * k * rec),
                 "bitrot_verify_all_files": (lambda: bitrot_verify_batch(files, n * rec, n * S,
                                                                         HashAlgorithm.HighwayHash256S, S), t * n * rec)}
        for what, (fn, alg) in cases.items():
            bench.steady_loop(fn, 0.5)
            kms = []
            _lib.check(L.rsg_set_kernel_timing(ctx, 1))
            for _ in range(20):
                r = fn()
                v = ctypes.c_float(-1)
                _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
                kms.append(v.value)
            _lib.check(L.rsg_set_kernel_timing(ctx, 0))
            torch.cuda.synchronize()
            if what == "get_all_present":
                _, src, status = r
                assert all(x == 0 for x in status) and all(bool(src[i].all()) for i in range(k))
            else:
                assert r == [0] * t, r
            km = sorted(kms)[10]
            out[what] = {"kernel_ms": round(km, 4), "frac": round(alg / (km * 1e-3) / 8e12, 4)}
        print(json.dumps(out), flush=True)
        del files, slots
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
