"""Whole-file bitrot_verify of RS(12,4)-sized record files at two record
pitches: S = 87382 (the 1 MiB block's shard: records at 2 mod 8, as rustfs
writes them) and S = 87392 (records at 0 mod 32), same n and file count —
does the misalignment cost the quad hash kernel its rate?  Steady state as
bench.py (0.5 s busy, median of 20 HIP-event-timed calls).  Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from rustfs_amd.bitrot import HashAlgorithm, bitrot_verify_batch
    from rustfs_amd import Erasure
    n, t = 4096, 16
    out = {}
    for S in (87382, 87392, 87384, 87390):
        rec = 32 + S
        e = Erasure(12, 4, 12 * S)
        assert e.shard_size() == S
        st = torch.randint(0, 256, (n, t, S), dtype=torch.uint8, device="cuda")
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
        e.encode_batch(st, dig)  # parity and every shard's HH256S
        files = []
        for i in range(t):
            f = torch.empty((n, rec), dtype=torch.uint8, device="cuda")
            f[:, :32] = dig[:, i]
            f[:, 32:] = st[:, i]
            files.append(f.reshape(-1))
        del st, dig
        fn = lambda: bitrot_verify_batch(files, n * rec, n * S, HashAlgorithm.HighwayHash256S, S)  # noqa: E731
        r = fn()
        assert r == [0] * t, r
        bench.steady_loop(fn, 0.5)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ms = []
        for _ in range(20):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        ms.sort()
        alg = t * n * rec
        out[S] = {"rec_mod8": rec % 8, "call_ms_median": round(ms[10], 4), "frac_call": round(alg / (ms[10] * 1e-3) / 8e12, 4)}
        del files
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
