"""Fused encode + HH256S kernel time of one geometry under each RSG_FUSED_KIND
(rsg_set_tuning) on a device-resident batch at 1 MiB blocks: steady state
(0.5 s busy), median of 20 calls timed with HIP events around each (the
encode is one launch on the current stream).
Usage: python tools/fused_kinds.py K M KIND [KIND ...]  (e.g. 8 4 auto dma net);
FK_TUNE="RSG_DMA_NT=1 ..." sets further knobs for the run; FK_PLAIN=1 times the
plain encode (no digests) instead."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from rustfs_amd import Erasure, _lib
    k, m = int(sys.argv[1]), int(sys.argv[2])
    n, S = 4096, -(-(1 << 20) // int(sys.argv[1]))
    e = Erasure(k, m, 1 << 20)
    st = bench.random_stripes(torch.device("cuda", 0), k, m, S, n, 3)
    dig = torch.empty((n, k + m, 32), dtype=torch.uint8, device="cuda")
    out = {"geometry": f"RS({k},{m})", "n": n, "S": S}
    extra = dict(kv.split("=", 1) for kv in os.environ.get("FK_TUNE", "").split() if kv)  # e.g. FK_TUNE="RSG_DMA_NT=1"
    out["tune"] = extra
    for kind in sys.argv[3:]:
        with _lib.tuned(RSG_FUSED_KIND=kind, **extra):
            fn = lambda: e.encode_batch(st, None if os.environ.get("FK_PLAIN") else dig)  # noqa: E731
            bench.steady_loop(fn, 0.5)
            kms = []
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for _ in range(20):  # one launch per call: events on the current stream around it
                ev[0].record()
                fn()
                ev[1].record()
                torch.cuda.synchronize()
                kms.append(ev[0].elapsed_time(ev[1]))
        km = sorted(kms)[10]
        out[kind] = {"kernel_ms": round(km, 4), "frac": round(n * (k + m) * S / (km * 1e-3) / 8e12, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
