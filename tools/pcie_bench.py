"""Host-memory (PCIe-inclusive) rates for DESIGN.md: pinned H2D/D2H copy
bandwidth and rsg_encode_batch_host (H2D data -> encode [+HH256S] -> D2H parity
[+digests], pipelined over two streams) on RS(8,4) 1 MiB stripes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustfs_amd import Erasure  # noqa: E402

GiB = float(1 << 30)


def copy_rate(nbytes, h2d=True, reps=5):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    return reps * nbytes / (time.perf_counter() - t) / 1e9


def per_block_calls(k, m, S, calls=200, threads=8, layout="separate"):
    """The reference's call pattern: one 1 MiB block per ReedSolomonEncoder::encode
    call (encode.rs:504-530) through rsg_encode: latency per call on one thread,
    and the aggregate rate of `threads` callers.  layout: "separate" (one
    pageable buffer per shard), "block" (shards back to back in one pageable
    buffer, encode_buffer's layout, erasure.rs:848-887: one copy per
    direction), "pinned" (that block in page-locked memory, as a pool of
    rsg_pin'ed block buffers would give)."""
    import threading
    from rustfs_amd import ReedSolomonEncoder
    rng = np.random.default_rng(1)

    def worker(res, idx):
        enc = ReedSolomonEncoder(k, m)
        if layout == "separate":
            sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        else:
            blk = (torch.zeros((k + m) * S, dtype=torch.uint8).pin_memory().numpy() if layout == "pinned"
                   else np.zeros((k + m) * S, np.uint8)).reshape(k + m, S)
            blk[:k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
            sh = [blk[i] for i in range(k + m)]
        enc.encode(sh)
        ts = []
        for _ in range(calls):
            t0 = time.perf_counter()
            enc.encode(sh)
            ts.append(time.perf_counter() - t0)
        res[idx] = ts

    one = {}
    worker(one, 0)
    lat = sorted(one[0])
    many = {}
    th = [threading.Thread(target=worker, args=(many, i)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    return {"median_us": round(lat[len(lat) // 2] * 1e6, 1), "p99_us": round(lat[int(len(lat) * 0.99)] * 1e6, 1),
            "GiB_s_1_thread": round(k * S / lat[len(lat) // 2] / GiB, 2),
            f"GiB_s_{threads}_threads": round(threads * calls * k * S / el / GiB, 2),
            "note": f"host-buffer rsg_encode per 1 MiB block, H2D+kernel+D2H per call, layout {layout}"}


def main():
    k, m, S, n = 8, 4, 131072, int(os.environ.get("PCIE_STRIPES", "1024"))
    out = {"h2d_GB_s": round(copy_rate(1 << 30, True), 2), "d2h_GB_s": round(copy_rate(1 << 30, False), 2)}
    e = Erasure(k, m, k * S)
    st = torch.zeros((n, k + m, S), dtype=torch.uint8).pin_memory().numpy()
    st[:, :k] = np.random.default_rng(0).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8).pin_memory().numpy()
    for hashed in (False, True):
        e.encode_batch_host(st, dig if hashed else None)
        reps = 5
        t = time.perf_counter()
        for _ in range(reps):
            e.encode_batch_host(st, dig if hashed else None)
        el = (time.perf_counter() - t) / reps
        out["encode_host%s" % ("_hh256s" if hashed else "")] = {
            "GiB_s_payload": round(n * k * S / el / GiB, 2), "ms_per_batch": round(el * 1e3, 2),
            "pcie_bytes_GB_s": round(n * (k + m) * S / el / 1e9 if True else 0, 2)}
    out["config"] = f"RS({k},{m}) S={S} n={n} pinned host buffers"
    for layout in ("separate", "block", "pinned"):
        out[f"per_block_call_{layout}"] = per_block_calls(k, m, S, layout=layout)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
